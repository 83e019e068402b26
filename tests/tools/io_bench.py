"""Feature-store -> HBM measurement (run on the GPU box).

Builds a LINAS-shaped BigFile (frames of 4096-d float32 = resnext101 (+) resnet152,
LINAS-engine/util/do_combine_features.sh:4-5; ~30 frames per video) under $TMPDIR, then times
  native: VideoBatchLoader -- rows gathered from the mmapped feature.bin by a thread team,
          streamed to HBM through pinned double-buffered staging, collated by K2 on the GPU;
  reference-style: the oracle restatement of BigFile.read_one called once per frame
          (LINAS-engine/util/tag_data_provider.py:330-337 -> basic/bigfile.py:23-60) on a
          bounded sample of videos, plus the host collate.
The file is freshly written, so both read from the page cache.  Prints one JSON line."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root (tests/tools/..)
for p in (os.path.join(ROOT, "cross-modal-video-engine_amd"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    n_videos = int(os.environ.get("IO_VIDEOS", 3300))
    dim = int(os.environ.get("IO_DIM", 4096))
    rng = np.random.default_rng(0)
    counts = rng.integers(10, 51, size=n_videos)
    frames = [f"v{v:06d}_{k}" for v in range(n_videos) for k in range(1, int(counts[v]) + 1)]
    perm = rng.permutation(len(frames))
    names = [frames[i] for i in perm]
    d = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    with open(os.path.join(d, "shape.txt"), "w") as f:
        f.write("%d %d\n" % (len(names), dim))
    with open(os.path.join(d, "id.txt"), "w") as f:
        f.write(" ".join(names))
    with open(os.path.join(d, "feature.bin"), "wb") as f:
        for s in range(0, len(names), 8192):
            f.write(rng.standard_normal((min(8192, len(names) - s), dim), dtype=np.float32).tobytes())
    v2f = {f"v{v:06d}": [f"v{v:06d}_{k}" for k in range(1, int(counts[v]) + 1)] for v in range(n_videos)}
    gb = len(names) * dim * 4 / 1e9

    from cmve.linas.bigfile import BigFile, VideoBatchLoader
    from oracle import bigfile as OB
    bf = BigFile(d)
    ld = VideoBatchLoader(bf, v2f, batch_size=128)
    ld.batch(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for out in ld:
        pass
    torch.cuda.synchronize()
    t_native = time.perf_counter() - t0

    ob = OB.BigFileOracle(d)
    vids = list(v2f)
    t0 = time.perf_counter()
    nv = nf = 0
    while time.perf_counter() - t0 < 10.0 and nv < len(vids):
        fl = [ob.read_one(fr) for fr in v2f[vids[nv]]]
        OB.collate([fl])
        nv += 1
        nf += len(fl)
    t_ref = time.perf_counter() - t0
    print(json.dumps({
        "metric": "video frames loaded from BigFile and collated in HBM",
        "store": {"frames": len(names), "videos": n_videos, "dim": dim, "gbytes": gb},
        "native": {"frames_per_s": len(names) / t_native, "gbytes_per_s": gb / t_native, "seconds": t_native,
                   "threads": int(os.environ.get("CMVE_IO_THREADS", min(16, os.cpu_count() or 1))),
                   "batch": 128, "path": "mmap gather -> pinned double buffer -> H2D -> K2 collate"},
        "reference_style": {"frames_per_s": nf / t_ref, "videos": nv, "seconds": t_ref,
                            "path": "BigFile.read_one per frame (oracle restatement) + host collate"},
        "speedup": (len(names) / t_native) / (nf / t_ref)}))


if __name__ == "__main__":
    main()
