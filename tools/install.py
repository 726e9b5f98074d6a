#!/usr/bin/env python3
"""Install dplasma_amd into a prefix (the reference's ``make install`` + ``dplasma.pc`` +
``dplasma-config.cmake``, src/include/dplasma.pc.in, cmake_modules/dplasma-config.cmake.in).

  python tools/install.py --prefix /opt/dplasma [--build]

Layout:
  PREFIX/lib/dplasma_amd/               the Python package with its built libraries (lib/*.so)
  PREFIX/lib/libdplasma.so              -> dplasma_amd/lib/libdplasma.so (C ABI; finds the package by realpath)
  PREFIX/lib/libdplasma_kernels.so      -> dplasma_amd/lib/libdplasma_kernels.so (HIP kernels, gfx950)
  PREFIX/include/dplasma.h
  PREFIX/lib/pkgconfig/dplasma.pc
  PREFIX/lib/cmake/dplasma/dplasma-config.cmake, dplasma-config-version.cmake
A C program then builds with ``pkg-config --cflags --libs dplasma`` or ``find_package(dplasma)``
(see examples/), and Python code with ``PYTHONPATH=PREFIX/lib``.
"""
from __future__ import annotations

import argparse
import os
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
VERSION = "2.0.0"


def install(prefix: Path, build: bool = False) -> Path:
    if build:
        import importlib.util
        spec = importlib.util.spec_from_file_location("dplasma_build", ROOT / "tools" / "build.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.build_all()
    prefix = prefix.resolve()
    lib, inc = prefix / "lib", prefix / "include"
    pkg = lib / "dplasma_amd"
    for d in (lib, inc, lib / "pkgconfig", lib / "cmake" / "dplasma"):
        d.mkdir(parents=True, exist_ok=True)
    if pkg.exists():
        shutil.rmtree(pkg)
    shutil.copytree(ROOT / "dplasma_amd", pkg, ignore=shutil.ignore_patterns("__pycache__", "*.pyc"))
    for so in ("libdplasma.so", "libdplasma_kernels.so"):
        if not (pkg / "lib" / so).exists():
            raise FileNotFoundError(f"{so} is not built (python tools/build.py)")
        link = lib / so
        if link.is_symlink() or link.exists():
            link.unlink()
        os.symlink(Path("dplasma_amd") / "lib" / so, link)
    shutil.copy2(ROOT / "capi" / "include" / "dplasma.h", inc / "dplasma.h")
    subst = {"@PREFIX@": str(prefix), "@VERSION@": VERSION}

    def render(src: str, dst: Path):
        text = (ROOT / "packaging" / src).read_text()
        for k, v in subst.items():
            text = text.replace(k, v)
        dst.write_text(text)
    render("dplasma.pc.in", lib / "pkgconfig" / "dplasma.pc")
    render("dplasma-config.cmake.in", lib / "cmake" / "dplasma" / "dplasma-config.cmake")
    render("dplasma-config-version.cmake.in", lib / "cmake" / "dplasma" / "dplasma-config-version.cmake")
    print(f"[install] dplasma_amd {VERSION} -> {prefix}")
    return prefix


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefix", required=True)
    ap.add_argument("--build", action="store_true", help="build the native parts first")
    a = ap.parse_args()
    install(Path(a.prefix), build=a.build)
