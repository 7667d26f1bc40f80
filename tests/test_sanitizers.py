"""Host-side sanitizer runs of the native library: ``make -C csrc asan tsan``
builds a self-test of every operator's host path -- every source file of libsrnn: the
templated shapes, 16-bit tables, the runtime-shape engine, the RCCL loader -- plus an
in-process R = 2 / 3 sharded-soup rehearsal (bitwise vs R = 1), under AddressSanitizer +
UBSan and ThreadSanitizer.  The test builds the binaries itself when they are missing or
older than the sources (host code instrumented, -O0: ~30 s per sanitizer with -j8) and
FAILS if the build fails -- it never skips."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")


def _stale(exe):
    if not os.path.exists(exe):
        return True
    t = os.path.getmtime(exe)
    srcs = glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) + \
        glob.glob(os.path.join(CSRC, "*.cpp")) + glob.glob(os.path.join(CSRC, "tests", "*.cpp"))
    return any(os.path.getmtime(s) > t for s in srcs)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_selftest_under_sanitizer(kind):
    exe = os.path.join(ROOT, "build", "sanitize", f"selftest_{kind}")
    if _stale(exe):
        b = subprocess.run(["make", "-C", CSRC, "-j8", kind], capture_output=True, text=True, timeout=1800)
        assert b.returncode == 0, "sanitizer build failed:\n" + b.stdout[-4000:] + b.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "host_selftest: ok" in p.stdout
