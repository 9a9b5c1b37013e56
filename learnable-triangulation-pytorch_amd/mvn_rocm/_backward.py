"""Backward passes of the mvn_rocm autograd functions.

Custom ops ``torch.ops.mvn_rocm.{unproject,softargmax3d,dlt}_backward`` over the C ABI
backward entry points (csrc/unproject_bwd.hip, csrc/backward.hip).  They replace the
ATen autograd the reference relies on (grid_sampler_2d / softmax / einsum / svd
backward, mvn/utils/op.py:84-163, mvn/utils/multiview.py:132-174).
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor

from . import _lib
from ._ops import _DTYPE_CODE, _op, _ptr, _require_gpu, _stream, call


# Accumulation of the unprojection backward: "fixed" (default) — 64-bit fixed point scaled
# per (frame, channel) plane (mvn_unproject_backward_deterministic): bit-identical across
# runs, the f32 rounding of the exact sums above 2^-38 of the plane's bound, the reference's
# per-element NaN / inf semantics, and ~3x faster than "float_atomic" (mvn_unproject_backward,
# order-dependent f32 atomics; kept for A/B and for callers that want no workspace).
UNPROJECT_BACKWARD = "fixed"


@_op("unproject_backward")
def unproject_bwd(feat: Tensor, proj: Tensor, coords: Tensor, conf: Optional[Tensor], grad_out: Tensor, agg: int,
                  align_corners: bool, want_conf: bool) -> List[Tensor]:
    """-> [grad_feat (B,N,C,H,W) in feat's dtype, grad_conf (B,N,C) f32 (empty unless want_conf)]"""
    _require_gpu(feat, proj, coords, conf, grad_out)
    B, N, C, H, W = feat.shape
    Vx, Vy, Vz = coords.shape[1:4]
    g = grad_out.contiguous()
    if g.dtype not in _DTYPE_CODE:
        g = g.float()
    gfeat = torch.zeros((B, N, C, H, W), dtype=torch.float32, device=feat.device)
    gconf = torch.zeros((B, N, C) if want_conf else (0,), dtype=torch.float32, device=feat.device)
    if feat.numel() == 0 or coords.numel() == 0:
        # empty batch / volume / maps: the reference's autograd returns zero-sized (or zero)
        # gradients; the forward launched nothing either (ops return the empty volume)
        return [gfeat.to(feat.dtype), gconf]
    lib = _lib.load()
    if UNPROJECT_BACKWARD == "fixed" or torch.are_deterministic_algorithms_enabled():
        # fixed-point accumulation, bit-identical across runs (always under
        # torch.use_deterministic_algorithms(True))
        ws = torch.empty(lib.mvn_unproject_backward_workspace_bytes(B, N, C, H, W), dtype=torch.uint8,
                         device=feat.device)
        code = lib.mvn_unproject_backward_deterministic(
            feat.data_ptr(), _DTYPE_CODE[feat.dtype], proj.data_ptr(), coords.data_ptr(), _ptr(conf), g.data_ptr(),
            _DTYPE_CODE[g.dtype], gfeat.data_ptr(), gconf.data_ptr() if want_conf else None, ws.data_ptr(),
            ws.numel(), B, N, C, H, W, Vx, Vy, Vz, agg, int(align_corners), _stream(feat))
        _lib.check(code, "mvn_unproject_backward_deterministic")
        return [gfeat.to(feat.dtype), gconf]
    code = lib.mvn_unproject_backward(
        feat.data_ptr(), _DTYPE_CODE[feat.dtype], proj.data_ptr(), coords.data_ptr(), _ptr(conf), g.data_ptr(),
        _DTYPE_CODE[g.dtype], gfeat.data_ptr(), gconf.data_ptr() if want_conf else None, B, N, C, H, W, Vx, Vy, Vz,
        agg, int(align_corners), _stream(feat))
    _lib.check(code, "mvn_unproject_backward")
    return [gfeat.to(feat.dtype), gconf]


@unproject_bwd.register_fake
def _(feat, proj, coords, conf, grad_out, agg, align_corners, want_conf):
    B, N, C = feat.shape[:3]
    return [torch.empty_like(feat), feat.new_empty((B, N, C) if want_conf else (0,), dtype=torch.float32)]


@_op("softargmax3d_backward")
def softargmax3d_bwd(vol: Tensor, coords: Tensor, softmax: bool, multiplier: float, grad_xyz: Optional[Tensor],
                     grad_vol: Optional[Tensor]) -> Tensor:
    """-> grad w.r.t. vol (B,J,Vx,Vy,Vz), contiguous, vol's dtype."""
    _require_gpu(vol, coords, grad_xyz, grad_vol)
    B, J, Vx, Vy, Vz = vol.shape
    gx = None if grad_xyz is None else grad_xyz.float().contiguous()
    gv = None if grad_vol is None else grad_vol.contiguous()
    if gv is not None and gv.dtype not in _DTYPE_CODE:
        gv = gv.float()
    gin = torch.empty((B, J, Vx, Vy, Vz), dtype=vol.dtype, device=vol.device)
    lib = _lib.load()
    ws_bytes = lib.mvn_softargmax3d_backward_workspace_bytes(B, J, Vx, Vy, Vz)
    ws = torch.empty((ws_bytes + 15) // 16 * 4, dtype=torch.float32, device=vol.device)
    code = lib.mvn_softargmax3d_backward(
        vol.data_ptr(), _DTYPE_CODE[vol.dtype], vol.stride(0), vol.stride(1), coords.data_ptr(), float(multiplier),
        int(softmax), _ptr(gx), _ptr(gv), _DTYPE_CODE[gv.dtype] if gv is not None else 0, gin.data_ptr(),
        _DTYPE_CODE[vol.dtype], ws.data_ptr(), ws.numel() * 4, B, J, Vx, Vy, Vz, _stream(vol))
    _lib.check(code, "mvn_softargmax3d_backward")
    return gin


@softargmax3d_bwd.register_fake
def _(vol, coords, softmax, multiplier, grad_xyz, grad_vol):
    return vol.new_empty(vol.shape)


@_op("dlt_backward")
def dlt_bwd(proj: Tensor, pts: Tensor, conf: Optional[Tensor], grad_out: Tensor) -> List[Tensor]:
    """-> [grad_pts (B,N,J,2), grad_conf (B,N,J) or empty]"""
    _require_gpu(proj, pts, conf, grad_out)
    B, N, J = pts.shape[:3]
    g = grad_out.float().contiguous()
    gpts = torch.empty_like(pts)
    gconf = torch.empty((B, N, J) if conf is not None else (0,), dtype=torch.float32, device=pts.device)
    if pts.numel() == 0:                   # empty batch: zero-sized gradients, as the reference's autograd
        return [gpts, gconf]
    code = _lib.load().mvn_dlt_backward(proj.data_ptr(), pts.data_ptr(), _ptr(conf), g.data_ptr(), gpts.data_ptr(),
                                        gconf.data_ptr() if conf is not None else None, B, N, J, _stream(pts))
    _lib.check(code, "mvn_dlt_backward")
    return [gpts, gconf]


@dlt_bwd.register_fake
def _(proj, pts, conf, grad_out):
    B, N, J = pts.shape[:3]
    return [torch.empty_like(pts), pts.new_empty((B, N, J) if conf is not None else (0,))]


# --------------------------------------------------------------------------- autograd glue
def unproject_backward(ctx, grad_out):
    feat, proj, coords, conf = ctx.saved_tensors
    agg, align_corners = ctx.cfg
    want_conf = conf is not None and ctx.needs_input_grad[3]
    if not (ctx.needs_input_grad[0] or want_conf):
        return None, None, None, None, None, None, None
    gfeat, gconf = call(unproject_bwd, feat, proj, coords, conf, grad_out, agg, align_corners, want_conf)
    return (gfeat if ctx.needs_input_grad[0] else None, None, None, gconf if want_conf else None,
            None, None, None)


def softargmax_backward(ctx, grad_xyz, grad_out):
    vol, coords = ctx.saved_tensors
    softmax, multiplier, return_volume = ctx.cfg
    if not ctx.needs_input_grad[0]:
        return None, None, None, None, None, None
    gv = grad_out if (return_volume and grad_out is not None and grad_out.numel() > 0) else None
    gin = call(softargmax3d_bwd, vol, coords, softmax, multiplier, grad_xyz, gv)
    return gin, None, None, None, None, None


def dlt_backward(ctx, grad_out):
    proj, pts, conf = ctx.saved_tensors
    want_pts, want_conf = ctx.needs_input_grad[1], conf is not None and ctx.needs_input_grad[2]
    if not (want_pts or want_conf):
        return None, None, None
    gpts, gconf = call(dlt_bwd, proj, pts, conf, grad_out)
    return None, gpts if want_pts else None, gconf if want_conf else None


def softargmax2d_backward(ctx, grad_xy, grad_maps):
    """d/d(heatmaps) of op.integrate_tensor_2d, as GPU tensor algebra (the op is (B*N, J,
    96, 96)-small; no kernel of its own).  With v = multiplier * h, e = exp(v - max) or
    relu(v), S = sum e, p = e / S, (X, Y) = sum p * (w, h):
      softmax: dL/dv = p * ((w - X) gX + (h - Y) gY + g_map - sum(g_map * p))
      relu:    dL/dv = [v > 0] * (((w - X) gX + (h - Y) gY) / S + g_map)
    """
    hm, xy = ctx.saved_tensors
    softmax, mult = ctx.cfg
    v = hm.float() * mult
    B, J, H, W = v.shape
    ws = torch.arange(W, dtype=torch.float32, device=v.device).view(1, 1, 1, W)
    hs = torch.arange(H, dtype=torch.float32, device=v.device).view(1, 1, H, 1)
    X, Y = xy[..., 0:1, None], xy[..., 1:2, None]
    gx = grad_xy[..., 0:1, None] if grad_xy is not None else None
    gy = grad_xy[..., 1:2, None] if grad_xy is not None else None
    geo = torch.zeros_like(v)
    if grad_xy is not None:
        geo = (ws - X) * gx + (hs - Y) * gy
    has_gm = grad_maps is not None and grad_maps.numel() > 0
    if softmax:
        p = torch.softmax(v.flatten(2), dim=2).view_as(v)
        g = geo
        if has_gm:
            gm = grad_maps.float()
            g = g + gm - (gm * p).sum(dim=(2, 3), keepdim=True)
        gv = p * g
    else:
        e = torch.relu(v)
        S = e.sum(dim=(2, 3), keepdim=True)
        g = geo / S
        if has_gm:
            g = g + grad_maps.float()
        gv = g * (v > 0).to(g.dtype)
    return (gv * mult).to(hm.dtype), None, None, None, None
