"""ctypes bindings of the in-tree native libraries.

Device ops call the gfx950 kernels in ``lib/libpfml_hip.so`` with raw device pointers and the
caller's current torch stream, so they compose with torch kernels, streams and HIP-graph
capture.  There is no silent fallback: a CUDA (HIP) tensor reaching an op whose library is
missing raises ``NativeUnavailable``; only CPU tensors take the fp64 torch/numpy oracle path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

from .. import build as _build

_lock = threading.Lock()
_hip = None
_rt = None


class NativeUnavailable(RuntimeError):
    pass


def _declare_hip(lib):
    P, I, L, D = C.c_void_p, C.c_int, C.c_int64, C.c_double
    lib.pfml_dgemm.argtypes = [I, I, I, I, I, I, D, P, L, L, P, L, L, D, P, L, L, P, L, P, L, P]
    lib.pfml_dgemm.restype = I
    lib.pfml_ridge_grid.argtypes = [P, L, P, P, I, I, P, I, P, P, L, P, P, I, P, I, P, P, P]
    lib.pfml_ridge_grid.restype = I
    lib.pfml_ridge_work_doubles.argtypes = [I, I]
    lib.pfml_ridge_work_doubles.restype = L
    lib.pfml_ridge_cell_desc_size.restype = I
    lib.pfml_ridge_band_nmax.restype = I
    lib.pfml_quadform.argtypes = [P, L, P, P, L, P, I, P, I, I, I, P, P, P]
    lib.pfml_quadform.restype = I
    lib.pfml_quadform_job_desc_size.restype = I
    lib.pfml_quadform_rows_per_tile.restype = I
    lib.pfml_quadform_row_tiles.argtypes = [I]
    lib.pfml_quadform_row_tiles.restype = I
    lib.pfml_segsum.argtypes = [P, L, P, P, I, P, P]
    lib.pfml_segsum.restype = I
    lib.pfml_spd_inverse.argtypes = [P, I, L, L, I, P, P, P]
    lib.pfml_spd_inverse.restype = I
    lib.pfml_spd_inverse_work_doubles.argtypes = [I, I]
    lib.pfml_spd_inverse_work_doubles.restype = L
    lib.pfml_lu_solve.argtypes = [P, I, I, L, L, I, I, I, P, P, P]
    lib.pfml_lu_solve.restype = I
    lib.pfml_lu_solve_work_doubles.argtypes = [I, I, I]
    lib.pfml_lu_solve_work_doubles.restype = L
    lib.pfml_lu_solve_max_n.restype = I
    lib.pfml_ridge_set_timing.argtypes = [P]
    lib.pfml_ridge_set_timing.restype = None
    for name, argt in _EXTRA_HIP.items():
        fn = getattr(lib, name)
        fn.argtypes = argt[0]
        fn.restype = argt[1]


# Additional kernels register their signatures here (name -> (argtypes, restype)).
_EXTRA_HIP: dict = {}


def register_hip(name: str, argtypes: list, restype=C.c_int) -> None:
    _EXTRA_HIP[name] = (argtypes, restype)
    if _hip is not None:
        fn = getattr(_hip, name)
        fn.argtypes, fn.restype = argtypes, restype


def hip_lib():
    """Load (building if stale and a toolchain exists) ``libpfml_hip.so``."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            # PFML_HIP_LIB: an alternative build of the kernels (A/B timing of two versions)
            path = os.environ.get("PFML_HIP_LIB") or _build.HIP_LIB
            if not os.path.exists(path):
                try:
                    _build.build_hip()
                except Exception as e:  # pragma: no cover - depends on toolchain
                    raise NativeUnavailable(f"libpfml_hip.so missing and build failed: {e}")
            try:
                lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
            except OSError as e:
                raise NativeUnavailable(f"cannot load {path}: {e}")
            _declare_hip(lib)
            _hip = lib
    return _hip


def rt_lib():
    """Load ``libpfml_rt.so`` (host C++ runtime); builds it with g++ when stale."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            path = _build.RT_LIB
            try:
                _build.build_runtime()
            except Exception as e:  # pragma: no cover
                if not os.path.exists(path):
                    raise NativeUnavailable(f"libpfml_rt.so missing and build failed: {e}")
            lib = C.CDLL(path)
            from ..runtime import declare
            declare(lib)
            _rt = lib
    return _rt


def check(err: int, what: str) -> None:
    if err != 0:
        raise RuntimeError(f"{what} failed with hipError {err}")


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def is_device(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def loaded_libraries() -> list[str]:
    out = []
    if _hip is not None:
        out.append(_build.HIP_LIB)
    if _rt is not None:
        out.append(_build.RT_LIB)
    return out
