"""SURVEY.md section 5 / VERDICT r04 item 6: the CPU restatement and the C
ABI's host validators under AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/Makefile `sanitize`, driver oracle/sanitize_main.c): the oracle's
whole forward / backward chain on seeded scenes (SH degrees 0-3 and
precomputed colours, F = 0 / 4 / 32, both compat modes, an off-centre
principal point, Gaussians behind the camera and beyond the image) and
gs_check_plan_header / gs_check_ranges / gs_check_point_list on valid and
corrupted plans must run clean; a deliberate heap overflow (the negative
control) must be caught."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")
BIN = os.path.join(ORACLE, "build", "oracle_sanitize")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("make") is None,
                                reason="gcc / make not available")


def _build():
    subprocess.run(["make", "-s", "-C", ORACLE, "build/oracle_sanitize"], check=True, capture_output=True,
                   timeout=300)


def test_oracle_and_host_validators_are_sanitizer_clean():
    _build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("GS_SANITIZE_SELFTEST", None)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.count("case ") == 4


def test_sanitizer_build_catches_a_heap_overflow():
    _build()
    env = dict(os.environ, GS_SANITIZE_SELFTEST="1", ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120, env=env)
    # UBSan's object-size check or ASan's shadow memory, whichever sees it first
    caught = "heap-buffer-overflow" in r.stderr or "insufficient space" in r.stderr
    assert r.returncode != 0 and caught, (r.returncode, r.stderr[-2000:])
