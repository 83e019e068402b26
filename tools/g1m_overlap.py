"""Timeline of the gallery_1m leg's chunked rank count from a rocprofv3 kernel trace (profiles/scripts/prof_g1m_r06.sh):
per timed step, each chunk's G256 rank-GEMM launch and the fp64 fix-up of the chunk before it (on the handle's auxiliary
stream).  Prints JSON: mean GEMM duration of a step's first chunk (nothing beside it) and of chunks 2..8 (the previous
chunk's fix-up beside it), the fix-up durations, and how much of each fix-up the concurrent GEMM absorbed."""
import csv
import json
import sys


def main(trace_csv, steps=5, chunks=8):
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    g256 = [r for r in rows if "sim_kernel<2, 1, 2, 4, 8, true" in r["Kernel_Name"]]
    fix = [r for r in rows if "fixup_kernel" in r["Kernel_Name"]]
    g = g256[-steps * chunks:]
    t0 = int(g[0]["Start_Timestamp"])
    f = [r for r in fix if int(r["Start_Timestamp"]) >= t0]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # noqa: E731
    gd = [dur(r) for r in g]
    first = [gd[i] for i in range(0, len(gd), chunks)]
    rest = [gd[i] for i in range(len(gd)) if i % chunks]
    fd = [dur(r) for r in f]
    out = {"source": trace_csv, "timed_steps": steps, "chunks": chunks,
           "gemm_ms_alone": sum(first) / len(first), "gemm_ms_beside_fixup": sum(rest) / len(rest),
           "fixup_ms": sum(fd) / len(fd),
           "step_ms_from_trace": (int(g[-1]["End_Timestamp"]) - int(g[-chunks]["Start_Timestamp"])) * 1e-6 + fd[-1]}
    out["gemm_growth_over_fixup"] = (out["gemm_ms_beside_fixup"] - out["gemm_ms_alone"]) / out["fixup_ms"]
    out["note"] = ("the fix-up's 1,024 blocks take the CUs first (launched ~7 us before the next chunk's GEMM); the "
                   "persistent G256 blocks (1 per CU, 256 VGPRs x 8 waves: the whole register file) start only as "
                   "those leave, so the GEMM grows by ~the fix-up's duration: chunking serialises the two")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
