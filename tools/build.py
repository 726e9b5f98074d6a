#!/usr/bin/env python3
"""Build the native parts of dplasma_amd in-tree.

* ``dplasma_amd/lib/libdplasma_kernels.so`` -- every HIP/CDNA4 kernel (gfx950),
  compiled with ``hipcc --offload-arch=gfx950`` (one object per ``.hip`` file,
  rebuilt only when the source or a header changed).
* ``dplasma_amd/lib/_dplasma_rt*.so`` -- the C++ runtime helpers as a pybind11
  module: tile-DAG level analysis / critical-path priorities (``dag.cpp``) and
  the band bulge-chasing kernels of the eigen/SVD reductions (``band.cpp``).

Usage: ``python tools/build.py [--force] [-j N]``.  Called by
``__graft_entry__.build()`` and imported lazily by ``dplasma_amd.ops._lib``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KSRC = ROOT / "csrc" / "kernels"
RSRC = ROOT / "csrc" / "runtime"
OUT = ROOT / "dplasma_amd" / "lib"
BUILD = ROOT / "build" / "obj"
ARCH = os.environ.get("DPLASMA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} {cmd[-1]}")
    return r


def build_kernels(force=False, jobs=8) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = sorted(KSRC.glob("*.h"))
    srcs = sorted(KSRC.glob("*.hip"))
    objs = []
    todo = []
    for s in srcs:
        o = BUILD / (s.stem + ".o")
        objs.append(o)
        if force or _newer(o, [s, *headers]):
            todo.append((s, o))

    def comp(so):
        s, o = so
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
              "-munsafe-fp-atomics", "-c", str(s), "-o", str(o)])
        return s.name

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for name in ex.map(comp, todo):
                print(f"[build] compiled {name}", flush=True)
    lib = OUT / "libdplasma_kernels.so"
    if force or todo or _newer(lib, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(lib)])
        print(f"[build] linked {lib.relative_to(ROOT)}", flush=True)
    return lib


def build_runtime(force=False) -> Path | None:
    srcs = sorted(RSRC.glob("*.cpp"))
    if not srcs:
        return None
    import pybind11

    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    lib = OUT / f"_dplasma_rt{suffix}"
    headers = sorted(RSRC.glob("*.h"))
    if not force and not _newer(lib, [*srcs, *headers]):
        return lib
    inc = [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{RSRC}",
           "-I/opt/rocm/include"]
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__",
           *inc, *map(str, srcs), "-o", str(lib), "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
           "-Wl,-rpath,/opt/rocm/lib"]
    _run(cmd)
    print(f"[build] linked {lib.relative_to(ROOT)}", flush=True)
    return lib


def build_capi(force=False) -> Path | None:
    """libdplasma.so: the C ABI (capi/include/dplasma.h) -- embeds CPython, forwards to dplasma_amd."""
    csrc = ROOT / "capi"
    srcs = sorted(csrc.glob("*.cpp"))
    if not srcs:
        return None
    lib = OUT / "libdplasma.so"
    kern = OUT / "libdplasma_kernels.so"
    if not force and not _newer(lib, [*srcs, *csrc.glob("*.h"), kern]):
        return lib
    pyinc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR") or "/usr/lib"
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    # native.cpp (interpreter-free engine) calls the HIP runtime and the kernel library directly
    _run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__",
          f"-I{pyinc}", f"-I{csrc}", "-I/opt/rocm/include", *map(str, srcs), "-o", str(lib), f"-L{libdir}",
          f"-lpython{ver}", f"-L{OUT}", "-ldplasma_kernels", "-L/opt/rocm/lib", "-lamdhip64", "-ldl",
          f"-Wl,-rpath,{libdir}", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])
    print(f"[build] linked {lib.relative_to(ROOT)}", flush=True)
    return lib


def build_tools(force=False) -> Path | None:
    """tools/gemmpeak/mfma_peak: the fp64/fp32 MFMA and VALU peak microbenchmark (built from source,
    never committed)."""
    src = ROOT / "tools" / "gemmpeak" / "mfma_peak.hip"
    if not src.exists():
        return None
    exe = src.with_suffix("")
    if force or _newer(exe, [src]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", str(src), "-o", str(exe)])
        print(f"[build] built {exe.relative_to(ROOT)}", flush=True)
    return exe


SAN_FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


def build_sanitized(kinds=("asan", "tsan")) -> dict:
    """Debug/sanitizer builds of the host-native code (reference configure --enable-debug modes,
    configure:81-90): the runtime cores (csrc/runtime/*_core.h) driven by
    tests/native/test_runtime_core.cpp, and the native dplasma_info_t of the C ABI driven by
    tests/capi/test_info.c.  GPU sanitizers are not used (host code only)."""
    out = ROOT / "build" / "sanitize"
    out.mkdir(parents=True, exist_ok=True)
    pyinc = sysconfig.get_paths()["include"]
    made = {}
    for kind in kinds:
        fl = ["-O1", "-g", *SAN_FLAGS[kind]]
        exe = out / f"test_runtime_core_{kind}"
        src = ROOT / "tests" / "native" / "test_runtime_core.cpp"
        deps = [src, *RSRC.glob("*_core.h")]
        if _newer(exe, deps):
            _run(["g++", "-std=c++17", *fl, f"-I{RSRC}", str(src), "-o", str(exe), "-lpthread"])
        made[f"runtime_{kind}"] = exe
        if kind == "asan":
            exe2 = out / "test_info_asan"
            deps2 = [ROOT / "capi" / "dplasma_info.cpp", ROOT / "tests" / "capi" / "test_info.c"]
            if _newer(exe2, deps2):
                obj = out / "test_info.o"
                _run(["gcc", *fl, f"-I{ROOT / 'capi' / 'include'}", "-c", str(deps2[1]), "-o", str(obj)])
                _run(["g++", "-std=c++17", *fl, f"-I{pyinc}", f"-I{ROOT / 'capi'}", str(deps2[0]), str(obj), "-o",
                      str(exe2)])
            made["info_asan"] = exe2
    return made


def build_all(force=False, jobs=8):
    k = build_kernels(force=force, jobs=jobs)
    r = build_runtime(force=force)
    build_capi(force=force)
    build_tools(force=force)
    return k, r


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--sanitize", action="store_true", help="also build the ASan/UBSan/TSan host test drivers")
    a = ap.parse_args()
    build_all(force=a.force, jobs=a.j)
    if a.sanitize:
        for k, v in build_sanitized().items():
            print(f"[build] sanitizer driver {k}: {v.relative_to(ROOT)}")
