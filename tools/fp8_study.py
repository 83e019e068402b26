"""fp8 (e4m3) gallery study for C5 (BASELINE.json configs[4] "fp8 MFMA"): how wide the
exactness band of DESIGN.md s4 gets when the MFMA operand planes are e4m3 instead of fp16, measured on the
gallery_shard leg's data (16,384 captions x a 131,072-video shard x 1024-d, sigma 10).

For each operand format the study packs REAL planes of the unit rows (torch float8_e4m3fn with power-of-two
scales: per row, or per 32-element block as MXFP8's E8M0 block scales; fp16 as the shipped rank path),
takes the rigorous per-row representation error e = ||x_hat - dequant(plane)||_2 in fp64 (rounded up,
as K1 does), the score bound E = e_q + (1 + e_q) e_g,max + gamma (score_error_bound, cmve_internal.h) and
counts, against the exact fp64 cosines:
  - rank band: pairs (i, j) with |cos_ij - s_gt,i| <= E_i (the undecided pairs the fp64 fix-up re-scores);
  - top-k band: columns with cos_ij >= T_k,i - 2 E_i (what the exact top-k must re-score, k = 10).
It also runs the e4m3 planes through the fp8 MFMA (torch._scaled_mm, row-wise scales when the build
takes them) and checks max (|s~ - cos| - bf16 output rounding) / E <= 1 (the bound holds for the real
fp8 accumulation).
Study tool (not the product path): prints one JSON line; the numbers are in profiles/r02_fp8_study.json.
    python tools/fp8_study.py [--nq 16384 --ng 131072 --chunk 1024]"""
import argparse
import json
import time

import torch

U = 2.0 ** -23


def pack(x, fmt):
    """(dequantised plane as fp64, plane for the MFMA, per-row scale or None) of unit rows x (fp64)."""
    if fmt == "f16":
        p = x.to(torch.float32).to(torch.float16)
        return p.double(), p, None
    n, d = x.shape
    if fmt == "e4m3_row":  # one power-of-two scale per row: amax -> (224, 448]
        amax = x.abs().amax(1, keepdim=True)
        sc = torch.exp2(torch.floor(torch.log2(448.0 / amax)))
        p = (x * sc).to(torch.float32).to(torch.float8_e4m3fn)
        return p.double() / sc, p, sc
    if fmt == "e4m3_mx32":  # MXFP8: a power-of-two (E8M0) scale per 32 elements, amax -> (224, 448]
        xb = x.view(n, d // 32, 32)
        amax = xb.abs().amax(2, keepdim=True).clamp_min(1e-300)
        sc = torch.exp2(torch.floor(torch.log2(448.0 / amax)))
        p = (xb * sc).to(torch.float32).to(torch.float8_e4m3fn)
        return (p.double() / sc).view(n, d), p.view(n, d), None
    raise ValueError(fmt)


def _mx_scales(x, n_b):
    """E8M0 dequantisation scales 2^-e of pack()'s MX blocks, [rows, n_b]."""
    amax = x.view(x.shape[0], n_b, 32).abs().amax(2).clamp_min(1e-300)
    return torch.exp2(-torch.floor(torch.log2(448.0 / amax))).float().to(torch.float8_e8m0fnu)


def row_err(x, deq):
    """rigorous per-row ||x - deq||_2 (fp64, rounded up as pack_row_planes does)."""
    e = ((x - deq) ** 2).sum(1).sqrt()
    return e * (1.0 + 1e-9) + 1e-12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=16384)
    ap.add_argument("--ng", type=int, default=131072)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--sigma", type=float, default=10.0)
    ap.add_argument("--chunk", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    gen = torch.Generator(device=dev).manual_seed(0)  # the gallery_shard leg's construction (bench.py)
    g = torch.randn((a.ng, a.dim), generator=gen, device=dev)
    gt = torch.randint(0, a.ng, (a.nq,), generator=gen, device=dev)
    q = g[gt] + a.sigma * torch.randn((a.nq, a.dim), generator=gen, device=dev)
    gx = g.double() / g.double().norm(dim=1, keepdim=True)
    qx = q.double() / q.double().norm(dim=1, keepdim=True)
    del g, q
    n_acc = a.dim * 33.0 / 32.0
    gamma = n_acc * U / (1.0 - n_acc * U)
    out = {"workload": f"{a.nq} captions x {a.ng} videos x {a.dim}-d, sigma {a.sigma} (gallery_shard data)",
           "k": a.k, "formats": {}}
    for fmt in ("f16", "e4m3_row", "e4m3_mx32"):
        gdq, gp, gsc = pack(gx, fmt)
        qdq, qp, qsc = pack(qx, fmt)
        eg, eq = row_err(gx, gdq), row_err(qx, qdq)
        egmax = float(eg.max())
        E = eq + (1.0 + eq) * egmax + gamma * (1.0 + eq) * (1.0 + egmax) + 1e-12
        band = 0
        topk_cols = 0.0
        worst = 0.0
        mfma = None
        for c0 in range(0, a.nq, a.chunk):
            c1 = min(a.nq, c0 + a.chunk)
            s = qx[c0:c1] @ gx.T  # exact fp64 cosines
            sgt = s.gather(1, gt[c0:c1, None])
            Ei = E[c0:c1, None]
            band += int(((s - sgt).abs() <= Ei).sum())
            tk = s.topk(a.k, dim=1).values[:, -1:]
            topk_cols += float((s >= tk - 2.0 * Ei).sum())
            if fmt != "f16" and c0 == 0:  # the real fp8 MFMA on the first chunk: does |s~ - cos| <= E hold?
                try:
                    # hipBLASLt's row-wise fp8 GEMM writes bf16 only: its output rounding (<= 2^-9 |s~|
                    # relative) is charged on top of E
                    if fmt == "e4m3_row":
                        st = torch._scaled_mm(qp[c0:c1], gp.T, scale_a=(1.0 / qsc[c0:c1]).float(),
                                              scale_b=(1.0 / gsc.T).float(), out_dtype=torch.bfloat16)
                        mfma = "torch._scaled_mm e4m3 x e4m3, row-wise fp32 scales, bf16 out (hipBLASLt)"
                    else:
                        n_b = a.dim // 32
                        sa = _mx_scales(qx[c0:c1], n_b)
                        sb = _mx_scales(gx, n_b)
                        st = torch._scaled_mm(qp[c0:c1], gp.T, scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
                        mfma = "torch._scaled_mm e4m3 x e4m3, E8M0 scales per 32 elements (MXFP8), bf16 out"
                    std = st.double()
                    worst = float((((std - s).abs() - std.abs() * 2.0 ** -9) / Ei).max())
                except Exception as ex:  # noqa: BLE001 -- report what the build lacks, keep the band numbers
                    mfma = f"not run: {type(ex).__name__}: {str(ex)[:160]}"
            del s
        pairs = a.nq * a.ng
        out["formats"][fmt] = {
            "e_row_mean": float(torch.cat([eq, eg]).mean()), "e_row_max": float(torch.cat([eq, eg]).max()),
            "E_mean": float(E.mean()),
            "rank_band_pairs": band, "rank_band_frac": band / pairs,
            "fixup_gather_GB_per_step": band * a.dim * 4 / 1e9,
            "topk_band_cols_per_query": topk_cols / a.nq, "topk_band_frac": topk_cols / pairs,
            "plane_bytes_per_row": a.dim * (2 if fmt == "f16" else 1) + (a.dim // 32 if fmt == "e4m3_mx32" else 0),
        }
        if fmt != "f16":
            out["formats"][fmt]["fp8_mfma_check"] = {"path": mfma, "max_abs_err_over_E": worst}
    out["seconds"] = time.time() - t0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
