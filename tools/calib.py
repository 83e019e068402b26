"""Counter calibration run (kernel studies; run under rocprofv3 by tools/calib.sh): known byte counts in the
K14 evaluation's access shapes (tools/calib.hip), one launch each, in this order:

  0 read16     1 GiB cold (a 1 GiB buffer was written in between: nothing of it in the Infinity Cache)
  1 read16     64 MiB, first read after a 1 GiB flush (cold)
  2 read16     the same 64 MiB again (Infinity-Cache resident, not L2: 64 MiB > 32 MiB of L2)
  3 read_prep  1 GiB cold, the prep's fp64 row shape
  4 read16     the 64 MiB buffer after the next flush (cold)
  5 read_prep  the 64 MiB buffer again (Infinity-Cache resident)
  6 write8     256 MiB, 8-B stores per lane
  7 write16    256 MiB, 16-B stores per lane

Writes the schedule to <out>/schedule.json; tools/calib_reduce.py matches it to the counter CSVs."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main(out):
    lib = ctypes.CDLL(os.path.join(HERE, "libcalib.so"))
    dev = torch.device("cuda", 0)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    GiB, MiB = 1 << 30, 1 << 20
    big = torch.zeros(GiB, dtype=torch.uint8, device=dev)
    flush = torch.zeros(GiB, dtype=torch.uint8, device=dev)
    small = torch.zeros(64 * MiB, dtype=torch.uint8, device=dev)
    wbuf = torch.zeros(256 * MiB, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1, dtype=torch.float64, device=dev)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    sched = []

    def run(name, fn, *a, nbytes):
        rc = fn(*a)
        torch.cuda.synchronize()
        if rc:
            raise RuntimeError(f"{name}: hip error {rc}")
        sched.append({"kernel": name, "bytes": nbytes})

    flush.fill_(1)
    torch.cuda.synchronize()
    run("read16_kernel", lib.calib_read16, P(big), ctypes.c_int64(GiB), P(sink), s, nbytes=GiB)
    flush.fill_(2)
    torch.cuda.synchronize()
    run("read16_kernel", lib.calib_read16, P(small), ctypes.c_int64(64 * MiB), P(sink), s, nbytes=64 * MiB)
    run("read16_kernel", lib.calib_read16, P(small), ctypes.c_int64(64 * MiB), P(sink), s, nbytes=64 * MiB)
    flush.fill_(3)
    torch.cuda.synchronize()
    run("read_prep_kernel", lib.calib_read_prep, P(big), ctypes.c_int64(GiB), P(sink), s, nbytes=GiB)
    run("read16_kernel", lib.calib_read16, P(small), ctypes.c_int64(64 * MiB), P(sink), s, nbytes=64 * MiB)
    run("read_prep_kernel", lib.calib_read_prep, P(small), ctypes.c_int64(64 * MiB), P(sink), s, nbytes=64 * MiB)
    run("write8_kernel", lib.calib_write8, P(wbuf), ctypes.c_int64(256 * MiB), s, nbytes=256 * MiB)
    run("write16_kernel", lib.calib_write16, P(wbuf), ctypes.c_int64(256 * MiB), s, nbytes=256 * MiB)
    os.makedirs(out, exist_ok=True)
    json.dump(sched, open(os.path.join(out, "schedule.json"), "w"), indent=1)
    print("calib done", len(sched))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "gpurun_out", "calib"))
