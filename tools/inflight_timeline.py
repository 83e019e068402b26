"""Kernel-trace timeline of the headline's timed loop with its batches in flight (rocprofv3 --kernel-trace CSV):
busy fraction of the GPU (union of kernel intervals), concurrency histogram (how many launches overlap), and the
idle gaps, over the densest window of K14 batch launches.  Usage: inflight_timeline.py <run_kernel_trace.csv>"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        n = r["Kernel_Name"]
        if "sim_kernel" in n and ("false, true, 1>" in n or "ELb0ELb1ELi1E" in n):
            kind = "gemm"
        elif "eval_prep_fin_batch" in n or "eval_prep_pair_f16_batch" in n or "eval_prep_batch" in n:
            kind = "prep"
        elif "eval_finish_batch" in n:
            kind = "fin"
        else:
            continue
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    # the timed loop: the longest run of batch launches with no gap over 200 us
    runs, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - max(x[1] for x in cur[-8:]) > 200_000:
            runs.append(cur)
            cur = []
        cur.append(e)
    runs.append(cur)
    seg = max(runs, key=len)
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    pts = sorted([(s, 1, k) for s, _, k in seg] + [(e, -1, k) for _, e, k in seg])
    conc, last, hist, busy = 0, t0, {}, 0
    kinds = {"gemm": 0, "prep": 0, "fin": 0}
    kind_busy = {"gemm": 0, "prep": 0, "both": 0}
    for t, d, k in pts:
        dt = t - last
        hist[conc] = hist.get(conc, 0) + dt
        if conc > 0:
            busy += dt
        g, p = kinds["gemm"] > 0, (kinds["prep"] + kinds["fin"]) > 0
        if g and p:
            kind_busy["both"] += dt
        elif g:
            kind_busy["gemm"] += dt
        elif p:
            kind_busy["prep"] += dt
        conc += d
        kinds[k] += d
        last = t
    span = t1 - t0
    n_gemm = sum(1 for e in seg if e[2] == "gemm")
    print(f"launches {len(seg)} (gemm {n_gemm}), span {span / 1e3:.1f} us, per gemm launch {span / max(n_gemm, 1) / 1e3:.1f} us")
    print(f"busy {busy / span:.3f}; time with: gemm only {kind_busy['gemm'] / span:.3f}, prep/finish only "
          f"{kind_busy['prep'] / span:.3f}, both {kind_busy['both'] / span:.3f}")
    print("concurrency:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
    for k in ("gemm", "prep", "fin"):
        d = [e[1] - e[0] for e in seg if e[2] == k]
        if d:
            d.sort()
            print(f"{k}: n {len(d)} median {d[len(d) // 2] / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
