"""Where a large split-bf16 LINEAR GEMM spends its time (the Combiner's K/V projection shape,
M = 1,048,576 rows x N = 1280 x K = 640): the same GEMM with the LINEAR epilogue (fp32 rows +
bias), the STORE epilogue, the single-plane bf16 loop, and a single-plane loop of K' = 3K (the
MFMA count of split-bf16).  Prints one JSON line of ms per call."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cross-modal-video-engine_amd"))

import torch  # noqa: E402
from cmve import engine  # noqa: E402
from cmve._lib import lib, check, SIM_BF16, SIM_BF16X3  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    M = int(os.environ.get("M", 1 << 20))
    N, K = int(os.environ.get("N", 1280)), int(os.environ.get("K", 640))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((M, K), generator=g, device=dev)
    w = torch.randn((N, K), generator=g, device=dev)
    b = torch.randn(N, generator=g, device=dev)
    xr = engine.RowSet(x, with_lo=True, with_f16=False, raw_rows=True, device=dev)
    wr = engine.RowSet(w, with_lo=True, with_f16=False, raw_rows=True, device=dev)
    out = torch.empty((M, N), dtype=torch.float32, device=dev)
    h = engine.handle(dev)

    def lin(mode, xs=xr, ws=wr, o=out):
        return lambda: check(lib.cmve_linear(h, engine.C.byref(xs.desc), engine.C.byref(ws.desc), mode, engine._ptr(b),
                                             None, None, None, 0, 1, engine._ptr(o), o.stride(0)), "cmve_linear")
    res = {"M": M, "N": N, "K": K}
    store = lambda: check(lib.cmve_sim_store(h, engine.C.byref(xr.desc), engine.C.byref(wr.desc), SIM_BF16X3, 1.0,  # noqa: E731
                                             0.0, engine._ptr(out), engine._dtype_code(out), out.stride(0)),
                          "cmve_sim_store")
    timed(store, 20)  # clocks settle
    res["store_bf16x3_first_ms"] = timed(store)
    res["linear_bf16x3_ms"] = timed(lin(SIM_BF16X3))
    res["linear_bf16_ms"] = timed(lin(SIM_BF16))
    x3 = torch.randn((M, 3 * K), generator=g, device=dev)
    w3 = torch.randn((N, 3 * K), generator=g, device=dev)
    x3r = engine.RowSet(x3, with_lo=False, with_f16=False, raw_rows=True, device=dev)
    w3r = engine.RowSet(w3, with_lo=False, with_f16=False, raw_rows=True, device=dev)
    res["linear_bf16_k3_ms"] = timed(lin(SIM_BF16, x3r, w3r))
    del x3, w3, x3r, w3r
    res["store_bf16x3_ms"] = timed(store)
    res["linear_bf16x3_again_ms"] = timed(lin(SIM_BF16X3))
    flop = 2.0 * M * N * K
    for k in list(res):
        if k.endswith("_ms"):
            mult = 3 if ("x3" in k or "k3" in k) else 1
            res[k.replace("_ms", "_mfma_tflops")] = flop * mult / (res[k] * 1e-3) / 1e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()
