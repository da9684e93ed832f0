"""Build the native libraries in-tree.

* ``lib/libpfml_hip.so``  - every ``csrc/*.hip`` kernel, compiled by hipcc for gfx950 only
  (``--offload-arch=gfx950``; CDNA4 code, no multi-arch fat binary, no CUDA path).
* ``lib/libpfml_rt.so``   - the host-side C++ runtime (``runtime/*.cpp``: panel indexer,
  universe state machine, rolling counts, segmented rank, EWMA scan for the CPU path).

Both expose a plain C ABI and are loaded with ctypes (``ops/_native.py``); nothing is JIT
compiled at import time, so the built ``.so`` files travel with the repo snapshot to the GPU
box.  ``python -m pfml.build`` (or ``__graft_entry__.build()``) rebuilds what is stale.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
RTSRC = os.path.join(HERE, "runtime")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "build", "obj")
HIP_LIB = os.path.join(LIBDIR, "libpfml_hip.so")
RT_LIB = os.path.join(LIBDIR, "libpfml_rt.so")
ARCH = os.environ.get("PFML_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the HIP kernels)")


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd: list[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_hip(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")))
    if not force and not _stale(HIP_LIB, srcs + headers):
        return HIP_LIB
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hipcc = _hipcc()
    flags = [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics"]

    def one(src):
        obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
        if force or _stale(obj, [src] + headers):
            _run([hipcc, *flags, "-c", src, "-o", obj], verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(one, srcs))
    tmp = HIP_LIB + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], verbose)
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(RTSRC, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(RTSRC, "*.h")))
    if not srcs:
        return ""
    if not force and not _stale(RT_LIB, srcs + headers):
        return RT_LIB
    os.makedirs(LIBDIR, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = RT_LIB + ".tmp"
    # runtime/sqlite_io.cpp links the system SQLite (no header in the image: the C-API
    # prototypes are declared in the source)
    _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-o", tmp, *srcs,
          "-l:libsqlite3.so.0"], verbose)
    os.replace(tmp, RT_LIB)
    return RT_LIB


def build_all(force: bool = False, verbose: bool = False) -> dict:
    return {"hip": build_hip(force, verbose), "runtime": build_runtime(force, verbose)}


if __name__ == "__main__":
    out = build_all(force="--force" in sys.argv, verbose=True)
    print(out)
