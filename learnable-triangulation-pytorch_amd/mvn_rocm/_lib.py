"""ctypes binding of libmvn_hip.so (the C ABI declared in include/mvn_hip.h).

The shared library is built in-tree (``make -C learnable-triangulation-pytorch_amd``)
and loaded from this directory.  There is no CPU fallback anywhere in the product
path: if the library is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MVN_HIP_LIB selects another in-tree build, e.g. the debug build with device-side assertions
# (``make -C learnable-triangulation-pytorch_amd debug`` -> libmvn_hip_debug.so); read once, at
# import — never on a launch path
LIB_PATH = os.path.abspath(os.environ.get("MVN_HIP_LIB") or os.path.join(_HERE, "libmvn_hip.so"))

MVN_OK = 0
MVN_DTYPE_F32 = 0
MVN_DTYPE_BF16 = 1
MVN_AGG_SUM, MVN_AGG_MAX, MVN_AGG_SOFTMAX, MVN_AGG_CONF = 0, 1, 2, 3
MVN_LAYOUT_NCDHW, MVN_LAYOUT_NDHWC = 0, 1
MVN_PRECISION_EXACT, MVN_PRECISION_FAST = 0, 1

_c_int, _c_void_p, _c_float, _c_i64, _c_size_t = (
    ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_int64, ctypes.c_size_t)

# name -> (restype, argtypes); kept in the order of include/mvn_hip.h
SIGNATURES = {
    "mvn_version": (_c_int, []),
    "mvn_strerror": (ctypes.c_char_p, [_c_int]),
    "mvn_unproject": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int]
                      + [_c_int] * 8 + [_c_int, _c_int, _c_void_p]),
    "mvn_softargmax3d_workspace_bytes": (_c_size_t, [_c_int] * 5),
    "mvn_softargmax3d": (_c_int, [_c_void_p, _c_int, _c_i64, _c_i64, _c_void_p, _c_float, _c_int,
                                  _c_void_p, _c_void_p, _c_int, _c_void_p, _c_size_t]
                         + [_c_int] * 5 + [_c_void_p]),
    "mvn_dlt": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_void_p]),
    "mvn_softargmax2d": (_c_int, [_c_void_p, _c_int, _c_float, _c_int, _c_void_p, _c_void_p, _c_int]
                         + [_c_int] * 4 + [_c_void_p]),
    "mvn_coord_volumes": (_c_int, [_c_void_p] * 5 + [_c_int, _c_int, _c_int, _c_void_p]),
    "mvn_unproject_cuboid": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_void_p,
                                      _c_int, _c_int] + [_c_int] * 6 + [_c_int, _c_int, _c_void_p]),
    "mvn_softargmax3d_cuboid": (_c_int, [_c_void_p, _c_int, _c_i64, _c_i64, _c_void_p, _c_int, _c_float, _c_int,
                                         _c_void_p, _c_void_p, _c_int, _c_void_p, _c_size_t]
                                + [_c_int] * 3 + [_c_void_p]),
    "mvn_nearest_voxel": (_c_int, [_c_void_p] * 3 + [_c_int] * 5 + [_c_void_p]),
    "mvn_unproject_ex": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int]
                         + [_c_int] * 8 + [_c_int, _c_int, _c_void_p]),
    "mvn_unproject_precision": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p,
                                         _c_void_p, _c_int, _c_int] + [_c_int] * 8 + [_c_int, _c_int, _c_int, _c_void_p]),
    "mvn_unproject_v2v_front_workspace_bytes": (_c_size_t, [_c_int, _c_int]),
    "mvn_unproject_v2v_front": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_int,
                                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_void_p, _c_size_t,
                                         _c_int] + [_c_int] * 6 + [_c_void_p]),
    "mvn_unproject_v2v_front_ex": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_int, _c_int,
                                            _c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int,
                                            _c_void_p, _c_size_t, _c_int] + [_c_int] * 6 + [_c_void_p]),
    "mvn_v2v_front_packed_weight_bytes": (_c_size_t, []),
    "mvn_v2v_front": (_c_int, [_c_void_p] * 5 + [_c_int, _c_int, _c_int, _c_void_p]),
    "mvn_unproject_backward": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int,
                                        _c_void_p, _c_void_p] + [_c_int] * 8 + [_c_int, _c_int, _c_void_p]),
    "mvn_unproject_backward_workspace_bytes": (_c_size_t, [_c_int] * 5),
    "mvn_unproject_backward_deterministic": (_c_int, [_c_void_p, _c_int, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                                      _c_int, _c_void_p, _c_void_p, _c_void_p, _c_size_t]
                                             + [_c_int] * 8 + [_c_int, _c_int, _c_void_p]),
    "mvn_softargmax3d_backward_workspace_bytes": (_c_size_t, [_c_int] * 5),
    "mvn_softargmax3d_backward": (_c_int, [_c_void_p, _c_int, _c_i64, _c_i64, _c_void_p, _c_float, _c_int,
                                           _c_void_p, _c_void_p, _c_int, _c_void_p, _c_int, _c_void_p, _c_size_t]
                                  + [_c_int] * 5 + [_c_void_p]),
    "mvn_dlt_backward": (_c_int, [_c_void_p] * 6 + [_c_int, _c_int, _c_int, _c_void_p]),
    "mvn_debug_set_unproject": (_c_int, [_c_int, _c_int]),
    "mvn_debug_device_asserts": (_c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint),
                                          ctypes.POINTER(ctypes.c_uint)]),
    "mvn_debug_dassert_selftest": (_c_int, [_c_int, _c_void_p]),
    "mvn_debug_unproject_occupancy": (_c_int, [_c_int]),
}

_lib = None


class MvnError(RuntimeError):
    """A negative MVN_ERR_* code returned by libmvn_hip."""


def load():
    """Load (once) and return the ctypes handle; raise loudly if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libmvn_hip.so not found at {LIB_PATH}; build it with "
                "`make -C learnable-triangulation-pytorch_amd` (or __graft_entry__.build()). "
                "mvn_rocm has no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(code: int, what: str) -> None:
    if code != MVN_OK:
        msg = load().mvn_strerror(code).decode()
        raise MvnError(f"{what}: {msg} (code {code})")


class unproject_knobs:
    """Context manager (tests only): force unprojection paths through the C ABI's test hook
    ``mvn_debug_set_unproject`` and restore the defaults on exit."""

    def __init__(self, lds_slots: int = 0, simple: bool = False, generic: bool = False):
        self.args = (int(lds_slots), 1 if simple else 2 if generic else 0)

    def __enter__(self):
        check(load().mvn_debug_set_unproject(*self.args), "mvn_debug_set_unproject")
        return self

    def __exit__(self, *exc):
        check(load().mvn_debug_set_unproject(0, 0), "mvn_debug_set_unproject")
        return False


def device_asserts():
    """(enabled, failures, first failing source line) of the debug build's device-side
    assertions since the last call (the counters are cleared); enabled is False for the
    release build.  Synchronises the current device first."""
    import torch
    torch.cuda.synchronize()
    en, cnt, line = ctypes.c_int(0), ctypes.c_uint(0), ctypes.c_uint(0)
    check(load().mvn_debug_device_asserts(ctypes.byref(en), ctypes.byref(cnt), ctypes.byref(line)),
          "mvn_debug_device_asserts")
    return bool(en.value), int(cnt.value), int(line.value)
