"""C ABI (capi/include/dplasma.h, dplasma_amd/lib/libdplasma.so): compile a plain C program against
it and run the Cholesky / GEMM / complex-norm flow, on the CPU path and (gpu marker) on cuda:0."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dplasma_amd", "lib")


def _build(tmp_path):
    if not os.path.exists(os.path.join(LIB, "libdplasma.so")):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import build  # noqa: F401
        build.build_capi()
    exe = str(tmp_path / "test_capi")
    subprocess.run(["gcc", "-O1", "-o", exe, os.path.join(ROOT, "tests", "capi", "test_capi.c"),
                    "-I" + os.path.join(ROOT, "capi", "include"), "-L" + LIB, "-ldplasma", "-lm",
                    "-Wl,-rpath," + LIB], check=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "CAPI OK" in r.stdout
    return r.stdout


def test_capi_cpu(tmp_path):
    out = _run(_build(tmp_path), 0, 300, 64)
    assert "dpotrf N=300" in out


@pytest.mark.gpu
def test_capi_gpu(tmp_path):
    out = _run(_build(tmp_path), 1, 1000, 256)
    assert "dpotrf N=1000" in out


def test_capi_info(tmp_path):
    """dplasma_info_t (native, no interpreter): the checks of the reference's testing_info.c."""
    if not os.path.exists(os.path.join(LIB, "libdplasma.so")):
        _build(tmp_path)
    exe = str(tmp_path / "test_info")
    subprocess.run(["gcc", "-O1", "-o", exe, os.path.join(ROOT, "tests", "capi", "test_info.c"),
                    "-I" + os.path.join(ROOT, "capi", "include"), "-L" + LIB, "-ldplasma",
                    "-Wl,-rpath," + LIB], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "INFO OK" in r.stdout, r.stdout + r.stderr
