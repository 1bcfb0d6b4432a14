"""AddressSanitizer + UndefinedBehaviorSanitizer runs (SURVEY.md §5 sanitizer row), host code only.

* the C oracle (oracle/asan_main.c: every oracle entry point over many shapes,
  specials, holes, illegal and out-of-range action ids) -- built and run here on
  every CPU test run (a few seconds);
* the device rule code's host build (tests/hostcore/asan_main.hip: every hostcore
  entry point over the specialised and frame shapes, the small-table overflow
  fallback and the paused cascade, cross-checked against the plain run). Its
  sanitized compile of the fully unrolled bitboard templates takes ~10 minutes,
  so the test runs the binary when it has been built (`make -C tests/hostcore
  asan`, or M3_BUILD_HOSTCORE_ASAN=1 to build it here) and skips otherwise.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HC = os.path.join(ROOT, "tests", "hostcore")
HC_BIN = os.path.join(HC, "build", "hostcore_asan")


def _clean(out):
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "oracle_asan")], capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    _clean(out)
    assert "asan oracle ok" in out


def test_hostcore_rule_code_under_asan_ubsan():
    if os.environ.get("M3_BUILD_HOSTCORE_ASAN") == "1":
        subprocess.run(["make", "-s", "-C", HC, "asan"], check=True)
    if not os.path.exists(HC_BIN):
        pytest.skip("sanitized hostcore not built (make -C tests/hostcore asan, ~10 min)")
    r = subprocess.run([HC_BIN], capture_output=True, text=True, timeout=1800)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    _clean(out)
    assert "no sanitizer report" in out


HC_MSAN = os.path.join(HC, "build", "hostcore_msan")


def test_hostcore_rule_code_under_msan():
    """MemorySanitizer over the same harness (round 6: ruling out an uninitialised read behind the
    lane interference): every hostcore entry point incl. rollouts on the headline and
    16 x 16-frame shapes, HC_N boards per shape (the instrumented -O0 build is slow; the committed
    run is profiles/r06_hostcore_msan.log). Built by `make -C tests/hostcore msan` (~30 min)."""
    if not os.path.exists(HC_MSAN):
        pytest.skip("MemorySanitizer hostcore not built (make -C tests/hostcore msan, ~30 min)")
    env = dict(os.environ, HC_N=os.environ.get("HC_N", "4"), MSAN_OPTIONS="halt_on_error=0")
    r = subprocess.run([HC_MSAN], capture_output=True, text=True, timeout=3000, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "MemorySanitizer" not in out, out[-4000:]
    assert "no sanitizer report" in out
