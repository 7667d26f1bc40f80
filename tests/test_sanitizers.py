"""Host-side sanitizer runs of the native library: ``make -C csrc asan tsan``
builds a self-test of every operator's host path plus an in-process R = 2 / 3 sharded-soup
rehearsal (bitwise vs R = 1) under AddressSanitizer + UBSan and ThreadSanitizer.  The
builds take minutes (device code is compiled too), so this test runs the binaries when
they exist and is skipped otherwise."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_selftest_under_sanitizer(kind):
    exe = os.path.join(ROOT, "build", "sanitize", f"selftest_{kind}")
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built (make -C csrc {kind})")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "host_selftest: ok" in p.stdout
