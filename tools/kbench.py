"""Developer micro-benchmark of the rank kernels (not the driver's bench): per sim mode,
the MFMA pass alone (thresholds +inf: no counts, no candidates), the MFMA pass with real
thresholds (counts + undecided pairs), and the fp64 fix-up.  Prints one JSON per line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cross-modal-video-engine_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cmve import engine, _lib  # noqa: E402


def timed(fn, reps=int(os.environ.get("REPS", 5))):
    fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def main():
    nq = int(os.environ.get("NQ", 16384)); ng = int(os.environ.get("NG", 131072)); d = int(os.environ.get("D", 1024))
    dev = torch.device("cuda", 0)
    probe = torch.zeros(10, dtype=torch.float32, device=dev)
    _lib.check(_lib.lib.cmve_mfma_probe(engine.handle(dev), engine._ptr(probe)))
    print(json.dumps({"mfma_probe": [float.hex(float(x)) for x in probe.cpu().numpy()]}), flush=True)
    gen = torch.Generator(device=dev).manual_seed(0)
    g = torch.randn((ng, d), generator=gen, device=dev)
    gt = torch.randint(0, ng, (nq,), generator=gen, device=dev)
    q = (g[gt] + 10.0 * torch.randn((nq, d), generator=gen, device=dev)).contiguous()
    G = engine.RowSet(g, with_lo=True, with_f16=True)
    Q = engine.RowSet(q, with_lo=True, with_f16=True)
    t_pack = timed(lambda: engine.RowSet(q, with_lo=False, with_f16=True))
    print(json.dumps({"pack_queries_ms": t_pack, "rows": nq, "dim": d}), flush=True)
    off, idx = engine.csr([[int(x)] for x in gt.cpu().numpy()], dev)
    ws = engine.RankWorkspace(dev, cap=1 << 25)
    inf = torch.full((Q.n_pad,), float("inf"), dtype=torch.float32, device=dev)
    flops = 2.0 * nq * ng * d
    modes = os.environ.get("MODES", "BF16,F16,BF16X3").split(",")
    for name, mode in (("BF16", _lib.SIM_BF16), ("F16", _lib.SIM_F16), ("BF16X3", _lib.SIM_BF16X3)):
        if name not in modes:
            continue
        sgt, hi, lo = engine.gt_thresholds(Q, G, off, idx, mode)
        cnt = torch.empty(Q.n_pad, dtype=torch.int32, device=dev)
        h = engine.handle(dev)

        def mfma(th_hi, th_lo):
            _lib.check(_lib.lib.cmve_rank_mfma(h, engine.C.byref(Q.desc), engine.C.byref(G.desc), mode, _lib.DIR_ROW,
                                               engine._ptr(th_hi), engine._ptr(th_lo), None, None, engine._ptr(cnt),
                                               None, engine._ptr(ws.cand), ws.cap, engine._ptr(ws.count)))

        def fix():
            _lib.check(_lib.lib.cmve_rank_fixup(h, engine.C.byref(Q.desc), engine.C.byref(G.desc), _lib.DIR_ROW,
                                                engine._ptr(sgt), None, engine._ptr(cnt), None, engine._ptr(ws.cand),
                                                ws.cap, engine._ptr(ws.count)))
        t_plain = timed(lambda: mfma(inf, inf))
        t_rank = timed(lambda: mfma(hi, lo))
        ncand = int(ws.count[0].item())
        t_fix = timed(fix) if not os.environ.get("KB_NOFIX") else float("nan")  # diagnostic builds: garbage pairs
        E = float((hi - lo)[:nq].double().mean().item()) / 2
        mult = 3 if mode == _lib.SIM_BF16X3 else 1
        print(json.dumps({"mode": name, "gemm_only_ms": t_plain, "rank_mfma_ms": t_rank, "fixup_ms": t_fix,
                          "candidates": ncand, "mean_E": E, "tflops_gemm_only": flops * mult / t_plain / 1e9,
                          "tflops_rank": flops * mult / t_rank / 1e9}), flush=True)
        if name == "F16":  # whole rank count (MFMA + fix-up), fix-ups overlapped across gallery chunks
            for ch in (1, 2, 4, 8):
                t = timed(lambda: engine.rank_count_launch(Q, G, mode, row=(sgt, hi, lo), ws=ws, chunks=ch))
                print(json.dumps({"mode": name, "chunks": ch, "rank_count_ms": t, "candidates": ws.ncand()}),
                      flush=True)


if __name__ == "__main__":
    main()
