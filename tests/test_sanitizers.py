"""Race detection / sanitizers for the native runtime: the standalone
self-test (csrc/native/tests/native_selftest.cpp: observation store and slot pool hammered from
several threads, the trial supervisor's poll loop racing API-side reads, kill / deadline paths,
parser, samplers) built plain, under ASan+UBSan, and under TSan (host code only)."""
import subprocess

import pytest


@pytest.mark.parametrize("sanitize", ["", "address,undefined", "thread"])
def test_native_selftest_under_sanitizers(sanitize):
    from katib_amd import _build

    exe = _build.build_selftest(sanitize)
    env = {"PATH": "/usr/bin:/bin", "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
           "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1", "TSAN_OPTIONS": "halt_on_error=1"}
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "native_selftest: ok" in r.stdout
