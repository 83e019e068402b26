"""The host side of the C ABI under AddressSanitizer: `make asan` builds libcmve_asan.so with
-fsanitize=address on every host translation unit (argument checks, workspace sizing, the BigFile mmap and
its gather threads; device code is not instrumented -- GPU ASan is not available on the pool), and the
CPU tests of the ABI and of BigFile run against it in a child process with the ASan runtime preloaded.
Any heap / stack overflow or use-after-free on those paths aborts the child."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cross-modal-video-engine_amd")
ASAN_LIB = os.path.join(PKG, "build", "asan", "libcmve_asan.so")


def test_host_abi_and_bigfile_under_asan():
    # (incremental: rebuilt only when a source or header changed since the last build)
    subprocess.run(["make", "-C", PKG, "-j", str(min(8, os.cpu_count() or 1)), "asan"], check=True,
                   stdout=subprocess.DEVNULL)
    blob = open(ASAN_LIB, "rb").read()
    assert b"__asan_report_load" in blob, "libcmve_asan.so is not instrumented"
    rt = subprocess.run(["make", "-s", "-C", PKG, "asan-runtime"], check=True, capture_output=True,
                        text=True).stdout.strip()
    assert os.path.exists(rt), rt
    env = dict(os.environ, LD_PRELOAD=rt, CMVE_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        os.path.join(ROOT, "tests", "test_abi.py"), os.path.join(ROOT, "tests", "test_bigfile.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout and "AddressSanitizer" not in r.stderr
