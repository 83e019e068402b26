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
        if os.environ.get("KB_STAMPS"):  # libcmve_STAMPS.so: per-block s_memtime stamps in ws.cand
            if os.environ.get("KB_STAMPS") == "real":
                mfma(hi, lo)  # the bench's thresholds: bands hit, undecided pairs emitted
            else:
                mfma(inf, inf)
            torch.cuda.synchronize()
            nblk = (Q.n_pad // 256) * (G.n_pad // 256)
            st = ws.cand[:nblk * 8].view(nblk, 8).cpu().numpy().astype(np.float64)
            d = np.diff(st[:, :4], axis=1)
            span = st[:, 3].max() - st[:, 0].min()
            med = lambda x: float(np.median(x))  # noqa: E731
            print(json.dumps({"stamps": {"prologue_cyc": med(d[:, 0]), "main_cyc": med(d[:, 1]),
                                         "epilogue_cyc": med(d[:, 2]),
                                         "epi_thr_publish": med(st[:, 4] - st[:, 2]),
                                         "epi_scoring": med(st[:, 5] - st[:, 4]),
                                         "epi_emission": med(st[:, 6] - st[:, 5]),
                                         "epi_flush_atomics": med(st[:, 3] - st[:, 6]),
                                         "block_total_cyc": float(np.median(st[:, 3] - st[:, 0])),
                                         "kernel_span_cyc": float(span), "blocks": nblk,
                                         "sum_block_cyc_per_cu": float((st[:, 3] - st[:, 0]).sum() / 256)}}),
                  flush=True)
            # per-CU timelines: gap between a block's end and the next block's start on the same CU
            hw = ws.cand[:nblk * 8].view(nblk, 8)[:, 7].cpu().numpy().astype(np.uint64)
            hwid = hw & np.uint64(0xffffffff)
            cu = (hw >> np.uint64(32)) * np.uint64(4096) + ((hwid >> np.uint64(8)) & np.uint64(0xf)) + \
                np.uint64(16) * ((hwid >> np.uint64(12)) & np.uint64(0x7))  # xcc, cu_id, sh/se bits
            gaps = []
            per_cu = {}
            for k in np.unique(cu):
                idx = np.where(cu == k)[0]
                o = idx[np.argsort(st[idx, 0])]
                per_cu[int(k)] = len(o)
                if len(o) > 1:
                    gaps.append(st[o[1:], 0] - st[o[:-1], 3])
            g = np.concatenate(gaps) if gaps else np.zeros(1)
            print(json.dumps({"cu_timeline": {"cus_seen": len(per_cu), "blocks_per_cu_med": med(list(per_cu.values())),
                                              "gap_cyc_med": med(g), "gap_cyc_p90": float(np.percentile(g, 90)),
                                              "gap_cyc_min": float(g.min())}}), flush=True)
            return  # the stamps build overwrites candidate slots: nothing after this is meaningful
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
