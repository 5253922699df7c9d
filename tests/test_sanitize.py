"""SURVEY §5 aux: AddressSanitizer + UndefinedBehaviorSanitizer over the CPU-side code -- the C oracle and the
kernel's per-lane source built for the host -- run in lockstep over every mode and policy kind, including the
per-step opponent mix (tests/sanitize/).  GPU sanitizers are not available on the pool, so device code is
covered by the bit-exact GPU parity tests instead."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs the host toolchain")
def test_oracle_and_host_kernel_source_under_asan_ubsan(tmp_path):
    out = str(tmp_path / "hk_sanitize_check")
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "sanitize"), f"OUT={out}"])
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([out], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitized lockstep: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
