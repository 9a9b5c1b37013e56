"""ORACLE — test infrastructure only.  ctypes wrapper of oracle/_build/libmvn_oracle.so."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "libmvn_oracle.so")
_lib = None

AGG = {"sum": 0, "max": 1, "softmax": 2}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        p, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        _lib.oracle_unproject.argtypes = [p, i, p, p, p, p] + [i] * 10
        _lib.oracle_softargmax3d.argtypes = [p, p, f, i, p, p] + [i] * 5
        _lib.oracle_dlt_design.argtypes = [p, p, p, p] + [i] * 5
    return _lib


def _c(a: np.ndarray, dtype) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=dtype)


def agg_code(method: str) -> int:
    return 3 if method.startswith("conf") else AGG[method]


def unproject(feat, proj, coords, method="sum", conf=None, align_corners=False, feat_bf16_bits=False):
    """feat (B,N,C,H,W) float32 (or uint16 bf16 bits with feat_bf16_bits) -> (B,C,Vx,Vy,Vz) float32."""
    lib = _load()
    feat = _c(feat, np.uint16 if feat_bf16_bits else np.float32)
    proj = _c(proj, np.float32)
    coords = _c(coords, np.float32)
    B, N, C, H, W = feat.shape
    Vx, Vy, Vz = coords.shape[1:4]
    out = np.empty((B, C, Vx, Vy, Vz), np.float32)
    cf = _c(conf, np.float32) if conf is not None else None
    rc = lib.oracle_unproject(feat.ctypes.data, int(feat_bf16_bits), proj.ctypes.data, coords.ctypes.data,
                              cf.ctypes.data if cf is not None else None, out.ctypes.data,
                              B, N, C, H, W, Vx, Vy, Vz, agg_code(method), int(align_corners))
    assert rc == 0
    return out


def softargmax3d(vol, coords, softmax=True, multiplier=1.0, return_volume=True):
    lib = _load()
    vol = _c(vol, np.float32)
    coords = _c(coords, np.float32)
    B, J, Vx, Vy, Vz = vol.shape
    xyz = np.empty((B, J, 3), np.float32)
    out = np.empty_like(vol) if return_volume else None
    lib.oracle_softargmax3d(vol.ctypes.data, coords.ctypes.data, float(multiplier), int(softmax), xyz.ctypes.data,
                            out.ctypes.data if out is not None else None, B, J, Vx, Vy, Vz)
    return xyz, out


def dlt_design(proj, pts, conf, b, j):
    """(2N, 4) float32 design matrix of multiview.py:150-152 for one (b, j)."""
    lib = _load()
    proj = _c(proj, np.float32)
    pts = _c(pts, np.float32)
    B, N, J = pts.shape[:3]
    cf = _c(conf, np.float32) if conf is not None else None
    A = np.empty((2 * N, 4), np.float32)
    lib.oracle_dlt_design(proj.ctypes.data, pts.ctypes.data, cf.ctypes.data if cf is not None else None,
                          A.ctypes.data, B, N, J, b, j)
    return A
