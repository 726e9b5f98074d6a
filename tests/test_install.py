"""Install into a prefix and build the out-of-tree example both ways the reference supports:
CMake ``find_package(dplasma)`` (cmake_modules/dplasma-config.cmake.in) and pkg-config
(src/include/dplasma.pc.in); run it on the CPU path."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def prefix(tmp_path_factory):
    if not (ROOT / "dplasma_amd" / "lib" / "libdplasma.so").exists():
        pytest.skip("native libraries not built")
    sys.path.insert(0, str(ROOT / "tools"))
    import install
    p = tmp_path_factory.mktemp("prefix")
    install.install(p)
    return p


def _run(exe):
    env = dict(os.environ)
    env.pop("PYTHONPATH", None)
    r = subprocess.run([str(exe), "0"], capture_output=True, text=True, timeout=300, env=env, cwd="/")
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not available")
def test_example_cmake(prefix, tmp_path):
    b = tmp_path / "build"
    subprocess.run(["cmake", "-S", str(ROOT / "examples"), "-B", str(b), f"-DCMAKE_PREFIX_PATH={prefix}"],
                   check=True, capture_output=True)
    subprocess.run(["cmake", "--build", str(b)], check=True, capture_output=True)
    _run(b / "potrf_example")


def _pc_flags(pc: Path):
    """--cflags --libs of a .pc file (pkg-config itself when installed, else the same expansion here)."""
    if shutil.which("pkg-config"):
        env = dict(os.environ, PKG_CONFIG_PATH=str(pc.parent))
        return subprocess.run(["pkg-config", "--cflags", "--libs", pc.stem], check=True, capture_output=True,
                              text=True, env=env).stdout.split()
    var, fields = {}, {}
    for ln in pc.read_text().splitlines():
        if "=" in ln and ":" not in ln.split("=")[0]:
            k, v = ln.split("=", 1)
            var[k.strip()] = v.strip()
        elif ":" in ln:
            k, v = ln.split(":", 1)
            fields[k.strip()] = v.strip()

    def expand(t):
        for _ in range(4):
            for k, v in var.items():
                t = t.replace("${" + k + "}", v)
        return t
    return expand(fields["Cflags"]).split() + expand(fields["Libs"]).split()


def test_example_pkgconfig(prefix, tmp_path):
    flags = _pc_flags(prefix / "lib" / "pkgconfig" / "dplasma.pc")
    exe = tmp_path / "potrf_example"
    subprocess.run(["gcc", "-O1", str(ROOT / "examples" / "potrf_example.c"), *flags, "-lm", "-o", str(exe)],
                   check=True)
    _run(exe)
