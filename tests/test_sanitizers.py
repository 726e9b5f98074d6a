"""Host-native code under sanitizers (reference debug build modes, configure:81-90): the runtime
cores (DAG analysis, threaded bulge chasing) with ASan+UBSan and with TSan, and the C ABI's native
dplasma_info_t with ASan+UBSan.  Built by tools/build.py (build_sanitized); no GPU, no Python in
the instrumented processes."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def drivers():
    sys.path.insert(0, str(ROOT / "tools"))
    import build
    try:
        return build.build_sanitized()
    except RuntimeError as e:  # pragma: no cover - toolchain without sanitizer runtimes
        pytest.skip(f"sanitizer build unavailable: {e}")


def _run(exe, token):
    env = dict(os.environ)
    env.update(ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and token in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_runtime_core_asan(drivers):
    _run(drivers["runtime_asan"], "NATIVE OK")


def test_runtime_core_tsan(drivers):
    _run(drivers["runtime_tsan"], "NATIVE OK")


def test_info_asan(drivers):
    _run(drivers["info_asan"], "INFO OK")
