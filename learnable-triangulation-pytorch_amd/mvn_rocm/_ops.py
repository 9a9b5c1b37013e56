"""PyTorch-ROCm custom ops over the libmvn_hip C ABI.

Each op is registered with ``torch.library.custom_op`` under the ``mvn_rocm``
namespace (``torch.ops.mvn_rocm.unproject`` …), launches on torch's current HIP
stream of the input's device, and has a fake (meta) kernel so it traces.  Inputs
must already live on the GPU: there is deliberately no CPU path.

Eager calls skip the dispatcher: ``call(op, *args)`` runs the op's own Python body
directly (the same ctypes launch) unless a tracer is active (torch.compile, or a
dispatch mode such as make_fx / FakeTensor), where the registered op is what must be
recorded.  The dispatcher round trip of a ``custom_op`` costs ~20 µs of host time per
call, on the order of the small launches it dispatches.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib

_DTYPE_CODE = {torch.float32: _lib.MVN_DTYPE_F32, torch.bfloat16: _lib.MVN_DTYPE_BF16}
_CODE_DTYPE = {v: k for k, v in _DTYPE_CODE.items()}


def _stream(t: Tensor) -> int:
    # the raw pointer of the device's current stream, without building a torch.cuda.Stream
    # object per call (host cost per op: the small-batch algebraic path is launch-bound)
    return torch._C._cuda_getCurrentRawStream(t.device.index)


def f32c(t: Tensor) -> Tensor:
    """t as contiguous float32, with no dispatcher round trip when it already is."""
    return t if (t.dtype is torch.float32 and t.is_contiguous()) else t.float().contiguous()


def _require_gpu(*tensors: Optional[Tensor]) -> None:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "mvn_rocm ops run on the MI355X only (got a tensor on "
                f"{t.device}); there is no CPU fallback")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"mvn_rocm: tensors on different devices ({dev} vs {t.device})")


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _op(name: str):
    """Register fn as torch.ops.mvn_rocm.<name>, keeping the plain function as .eager."""
    def deco(fn):
        d = torch.library.custom_op(f"mvn_rocm::{name}", fn, mutates_args=())
        d.eager = fn
        return d
    return deco


def _tracing() -> bool:
    """Something records or transforms the call: torch.compile, a torch-dispatch mode,
    torch.jit.trace, or a functorch transform (vmap / grad / jvp wrap storage-less tensors)."""
    if torch.compiler.is_compiling() or torch._C._len_torch_dispatch_stack():
        return True
    if torch._C._get_tracing_state() is not None:
        return True
    try:
        return torch._C._functorch.peek_interpreter_stack() is not None
    except AttributeError:        # older torch: no functorch interpreter stack
        return False


def call(op, *args):
    """op(*args) — through the dispatcher only while something traces."""
    if _tracing():
        return op(*args)
    return op.eager(*args)


# --------------------------------------------------------------------------- unproject
@_op("unproject")
def unproject(feat: Tensor, proj: Tensor, coords: Tensor, conf: Optional[Tensor], agg: int,
              align_corners: bool, out_dtype: int, precision: int = 0) -> Tensor:
    """feat (B,N,C,H,W) f32|bf16, proj (B,N,3,4) f32, coords (B,Vx,Vy,Vz,3) f32,
    conf (B,N,C) f32 or None -> (B,C,Vx,Vy,Vz) of dtype code `out_dtype`; `precision`
    MVN_PRECISION_EXACT (the reference's rounding) or MVN_PRECISION_FAST."""
    _require_gpu(feat, proj, coords, conf)
    B, N, C, H, W = feat.shape
    Vx, Vy, Vz = coords.shape[1:4]
    out = torch.empty((B, C, Vx, Vy, Vz), dtype=_CODE_DTYPE[out_dtype], device=feat.device)
    if out.numel() == 0:                  # empty batch: the reference returns the empty volume
        return out
    lib = _lib.load()
    if precision == _lib.MVN_PRECISION_EXACT:
        code = lib.mvn_unproject(
            feat.data_ptr(), _DTYPE_CODE[feat.dtype], proj.data_ptr(), coords.data_ptr(), _ptr(conf),
            out.data_ptr(), out_dtype, B, N, C, H, W, Vx, Vy, Vz, agg, int(align_corners), _stream(feat))
    else:
        code = lib.mvn_unproject_precision(
            feat.data_ptr(), _DTYPE_CODE[feat.dtype], proj.data_ptr(), coords.data_ptr(), None, 0, _ptr(conf),
            out.data_ptr(), out_dtype, _lib.MVN_LAYOUT_NCDHW, B, N, C, H, W, Vx, Vy, Vz, agg, int(align_corners),
            int(precision), _stream(feat))
    _lib.check(code, "mvn_unproject")
    return out


@unproject.register_fake
def _(feat, proj, coords, conf, agg, align_corners, out_dtype, precision=0):
    B, N, C, H, W = feat.shape
    return feat.new_empty((B, C, *coords.shape[1:4]), dtype=_CODE_DTYPE[out_dtype])


# --------------------------------------------------------------------------- soft-argmax
@_op("softargmax3d")
def softargmax3d(vol: Tensor, coords: Tensor, softmax: bool, multiplier: float, return_volume: bool,
                 out_dtype: int) -> Tuple[Tensor, Tensor]:
    """vol (B,J,Vx,Vy,Vz) f32|bf16 (inner three dims contiguous; batch / joint strides
    arbitrary), coords (B,Vx,Vy,Vz,3) f32 -> (xyz (B,J,3) f32, normalised volume or an
    empty tensor when return_volume is False)."""
    _require_gpu(vol, coords)
    B, J, Vx, Vy, Vz = vol.shape
    xyz = torch.empty((B, J, 3), dtype=torch.float32, device=vol.device)
    if return_volume:
        out = torch.empty((B, J, Vx, Vy, Vz), dtype=_CODE_DTYPE[out_dtype], device=vol.device)
    else:
        out = torch.empty((0,), dtype=_CODE_DTYPE[out_dtype], device=vol.device)
    lib = _lib.load()
    ws_bytes = lib.mvn_softargmax3d_workspace_bytes(B, J, Vx, Vy, Vz)
    ws = torch.empty((ws_bytes + 15) // 16 * 4, dtype=torch.float32, device=vol.device)
    code = lib.mvn_softargmax3d(
        vol.data_ptr(), _DTYPE_CODE[vol.dtype], vol.stride(0), vol.stride(1), coords.data_ptr(),
        float(multiplier), int(softmax), xyz.data_ptr(), out.data_ptr() if return_volume else None,
        out_dtype, ws.data_ptr(), ws.numel() * 4, B, J, Vx, Vy, Vz, _stream(vol))
    _lib.check(code, "mvn_softargmax3d")
    return xyz, out


@softargmax3d.register_fake
def _(vol, coords, softmax, multiplier, return_volume, out_dtype):
    B, J = vol.shape[:2]
    xyz = vol.new_empty((B, J, 3), dtype=torch.float32)
    shape = tuple(vol.shape) if return_volume else (0,)
    return xyz, vol.new_empty(shape, dtype=_CODE_DTYPE[out_dtype])


# --------------------------------------------------------------------------- in-kernel coordinates
@_op("unproject_cuboid")
def unproject_cuboid(feat: Tensor, proj: Tensor, cuboids: Tensor, volume_size: int, transfer: bool,
                     conf: Optional[Tensor], agg: int, align_corners: bool, out_dtype: int,
                     precision: int = 0) -> Tensor:
    """unproject with coordinates formed in-kernel from cuboids (B, 18) f32 (V^3 grid)."""
    _require_gpu(feat, proj, cuboids, conf)
    B, N, C, H, W = feat.shape
    V = int(volume_size)
    out = torch.empty((B, C, V, V, V), dtype=_CODE_DTYPE[out_dtype], device=feat.device)
    if out.numel() == 0:
        return out
    code = _lib.load().mvn_unproject_precision(
        feat.data_ptr(), _DTYPE_CODE[feat.dtype], proj.data_ptr(), None, cuboids.data_ptr(), int(transfer), _ptr(conf),
        out.data_ptr(), out_dtype, _lib.MVN_LAYOUT_NCDHW, B, N, C, H, W, V, V, V, agg, int(align_corners),
        int(precision), _stream(feat))
    _lib.check(code, "mvn_unproject_cuboid")
    return out


@unproject_cuboid.register_fake
def _(feat, proj, cuboids, volume_size, transfer, conf, agg, align_corners, out_dtype, precision=0):
    B, N, C = feat.shape[:3]
    V = int(volume_size)
    return feat.new_empty((B, C, V, V, V), dtype=_CODE_DTYPE[out_dtype])


@_op("softargmax3d_cuboid")
def softargmax3d_cuboid(vol: Tensor, cuboids: Tensor, transfer: bool, softmax: bool, multiplier: float,
                        return_volume: bool, out_dtype: int) -> Tuple[Tensor, Tensor]:
    """softargmax3d with coordinates formed in-kernel from cuboids (B, 18) f32."""
    _require_gpu(vol, cuboids)
    B, J, V = vol.shape[:3]
    xyz = torch.empty((B, J, 3), dtype=torch.float32, device=vol.device)
    if return_volume:
        out = torch.empty(tuple(vol.shape), dtype=_CODE_DTYPE[out_dtype], device=vol.device)
    else:
        out = torch.empty((0,), dtype=_CODE_DTYPE[out_dtype], device=vol.device)
    lib = _lib.load()
    ws_bytes = lib.mvn_softargmax3d_workspace_bytes(B, J, V, V, V)
    ws = torch.empty((ws_bytes + 15) // 16 * 4, dtype=torch.float32, device=vol.device)
    code = lib.mvn_softargmax3d_cuboid(
        vol.data_ptr(), _DTYPE_CODE[vol.dtype], vol.stride(0), vol.stride(1), cuboids.data_ptr(), int(transfer),
        float(multiplier), int(softmax), xyz.data_ptr(), out.data_ptr() if return_volume else None,
        out_dtype, ws.data_ptr(), ws.numel() * 4, B, J, V, _stream(vol))
    _lib.check(code, "mvn_softargmax3d_cuboid")
    return xyz, out


@softargmax3d_cuboid.register_fake
def _(vol, cuboids, transfer, softmax, multiplier, return_volume, out_dtype):
    B, J = vol.shape[:2]
    shape = tuple(vol.shape) if return_volume else (0,)
    return vol.new_empty((B, J, 3), dtype=torch.float32), vol.new_empty(shape, dtype=_CODE_DTYPE[out_dtype])


# --------------------------------------------------------------------------- 2D soft-argmax
@_op("softargmax2d")
def softargmax2d(hm: Tensor, softmax: bool, multiplier: float, return_maps: bool,
                 out_dtype: int) -> Tuple[Tensor, Tensor]:
    """hm (B,J,H,W) f32|bf16 contiguous -> (xy (B,J,2) f32, maps (B,J,H,W) or an empty tensor)."""
    _require_gpu(hm)
    B, J, H, W = hm.shape
    xy = torch.empty((B, J, 2), dtype=torch.float32, device=hm.device)
    if return_maps:
        maps = torch.empty((B, J, H, W), dtype=_CODE_DTYPE[out_dtype], device=hm.device)
    else:
        maps = torch.empty((0,), dtype=_CODE_DTYPE[out_dtype], device=hm.device)
    code = _lib.load().mvn_softargmax2d(hm.data_ptr(), _DTYPE_CODE[hm.dtype], float(multiplier), int(softmax),
                                        xy.data_ptr(), maps.data_ptr() if return_maps else None, out_dtype,
                                        B, J, H, W, _stream(hm))
    _lib.check(code, "mvn_softargmax2d")
    return xy, maps


@softargmax2d.register_fake
def _(hm, softmax, multiplier, return_maps, out_dtype):
    B, J = hm.shape[:2]
    shape = tuple(hm.shape) if return_maps else (0,)
    return hm.new_empty((B, J, 2), dtype=torch.float32), hm.new_empty(shape, dtype=_CODE_DTYPE[out_dtype])


# --------------------------------------------------------------------------- DLT
@_op("dlt")
def dlt(proj: Tensor, pts: Tensor, conf: Optional[Tensor]) -> Tensor:
    """proj (B,N,3,4) f32, pts (B,N,J,2) f32, conf (B,N,J) f32 or None -> (B,J,3) f32."""
    _require_gpu(proj, pts, conf)
    B, N, J = pts.shape[:3]
    out = torch.empty((B, J, 3), dtype=torch.float32, device=pts.device)
    if out.numel() == 0:                  # multiview.py:164-174 on an empty batch: (0, J, 3)
        return out
    code = _lib.load().mvn_dlt(proj.data_ptr(), pts.data_ptr(), _ptr(conf), out.data_ptr(), B, N, J,
                               _stream(pts))
    _lib.check(code, "mvn_dlt")
    return out


@dlt.register_fake
def _(proj, pts, conf):
    B, N, J = pts.shape[:3]
    return pts.new_empty((B, J, 3), dtype=torch.float32)
