"""Drop-in replacements for the hot-path functions of ``mvn/utils/op.py``.

Same names, positional / keyword order, defaults, return values and exception
types as the reference (cited per function).  Extra keyword-only arguments have
defaults that reproduce the reference behaviour.
"""
from __future__ import annotations

import torch

from . import _lib
from . import _ops

_AGG = {"sum": _lib.MVN_AGG_SUM, "max": _lib.MVN_AGG_MAX, "softmax": _lib.MVN_AGG_SOFTMAX}
_PRECISION = {"exact": _lib.MVN_PRECISION_EXACT, "fast": _lib.MVN_PRECISION_FAST}
_default_precision = "exact"


def set_unproject_precision(precision: str) -> str:
    """Process-wide default arithmetic of ``unproject_heatmaps`` calls that pass no
    ``precision=`` (as ``torch.backends`` flags do for matmul): ``'exact'`` (the default: the
    reference's f32 rounding, 'sum' / 'max' / 'conf*' bit-exact) or ``'fast'`` (the north_star
    tolerance) — the switch for a model rebound by ``install()``.  Returns the
    previous setting."""
    global _default_precision
    precision_code(precision)
    prev, _default_precision = _default_precision, precision
    return prev


def precision_code(precision) -> int:
    p = _default_precision if precision is None else precision
    if p not in _PRECISION:
        raise ValueError(f"Unknown unprojection precision: {p!r} (expected 'exact' or 'fast')")
    return _PRECISION[p]


def aggregation_code(method: str) -> int:
    """Map the reference's aggregation string to its code (op.py:147-161)."""
    if method.startswith("conf"):          # op.py:147 — any 'conf*' string
        return _lib.MVN_AGG_CONF
    if method in _AGG:
        return _AGG[method]
    raise ValueError("Unknown volume_aggregation_method: {}".format(method))   # op.py:161


def _is_cuboids(x) -> bool:
    from .volumetric import Cuboids
    return isinstance(x, Cuboids)


def _needs_grad(*tensors) -> bool:
    """Whether autograd must record the call (else the op runs without an autograd node)."""
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.float32:
        return _lib.MVN_DTYPE_F32
    if dtype == torch.bfloat16:
        return _lib.MVN_DTYPE_BF16
    raise TypeError(f"mvn_rocm supports float32 and bfloat16, got {dtype}")


def unproject_inputs(heatmaps, proj_matricies, vol_confidences, agg, method, cuboids=None):
    """Checked, contiguous (features, projections, confidences-or-None) of an unprojection
    call (shared by every unprojection entry point): features cast to float32 unless they
    are float32 / bfloat16 (op.py:99 takes any float tensor), projections (B, N, 3, 4),
    confidences (B, N, C) for 'conf*' only, and a ``Cuboids`` — when given — for B frames."""
    if agg == _lib.MVN_AGG_CONF and vol_confidences is None:
        raise TypeError("volume_aggregation_method '{}' needs vol_confidences".format(method))
    feat = heatmaps.contiguous()
    if feat.dtype not in (torch.float32, torch.bfloat16):
        feat = feat.float()
    if feat.dim() != 5:
        raise RuntimeError(f"heatmaps must be (B, N, C, H, W), got {tuple(feat.shape)}")
    proj = _ops.f32c(proj_matricies)
    conf = _ops.f32c(vol_confidences) if agg == _lib.MVN_AGG_CONF else None
    if proj.shape[:2] != feat.shape[:2] or proj.shape[2:] != (3, 4):
        raise RuntimeError(f"proj_matricies shape {tuple(proj.shape)} does not match heatmaps {tuple(feat.shape)}")
    if conf is not None and conf.shape != feat.shape[:3]:
        raise RuntimeError(f"vol_confidences must be {tuple(feat.shape[:3])}, got {tuple(conf.shape)}")
    if cuboids is not None and cuboids.batch != feat.shape[0]:
        raise RuntimeError(f"cuboids for {cuboids.batch} frames, heatmaps have {feat.shape[0]}")
    return feat, proj, conf


def unproject_heatmaps(heatmaps, proj_matricies, coord_volumes, volume_aggregation_method='sum',
                       vol_confidences=None, *, align_corners=False, out_dtype=None, precision=None):
    """Lift N views of C-channel maps into a (B, C, Vx, Vy, Vz) volume.

    Reference: ``mvn/utils/op.py:99-163``.
      heatmaps (B, N, C, H, W), proj_matricies (B, N, 3, 4), coord_volumes (B, Vx, Vy, Vz, 3),
      volume_aggregation_method in {'sum', 'max', 'softmax', 'conf*'}, vol_confidences (B, N, C).
    ``align_corners`` selects grid_sample semantics (False = torch>=1.3, the importable
    oracle; True = the torch 1.0.1 the reference pins).  ``out_dtype`` defaults to the
    heatmap dtype (float32 for float32 input, as in the reference).  ``precision`` —
    ``'exact'`` or ``'fast'``, default ``set_unproject_precision``'s — selects the arithmetic
    (DESIGN.md §4.1a); the backward is the exact function's in both.
    """
    agg = aggregation_code(volume_aggregation_method)
    prec = precision_code(precision)
    cub = coord_volumes if _is_cuboids(coord_volumes) else None
    feat, proj, conf = unproject_inputs(heatmaps, proj_matricies, vol_confidences, agg, volume_aggregation_method, cub)
    od = _dtype_code(out_dtype if out_dtype is not None else feat.dtype)
    if cub is not None:
        if feat.shape[1] > 8:
            # in-kernel coordinates need the tiled kernel (N <= 8): materialise the volume
            coord_volumes, cub = cub.coord_volumes(), None
        else:
            args = (feat, proj, cub.params, cub.volume_size, cub.transfer, conf, agg, bool(align_corners), od, prec)
            if _needs_grad(feat, conf):
                return UnprojectCuboidFunction.apply(*args)
            return _ops.call(_ops.unproject_cuboid, *args)
    coords = _ops.f32c(coord_volumes)
    if coords.dim() != 5 or coords.shape[0] != feat.shape[0] or coords.shape[4] != 3:
        raise RuntimeError(f"coord_volumes must be (B, Vx, Vy, Vz, 3), got {tuple(coords.shape)}")
    if _needs_grad(feat, conf):
        return UnprojectFunction.apply(feat, proj, coords, conf, agg, bool(align_corners), od, prec)
    return _ops.call(_ops.unproject, feat, proj, coords, conf, agg, bool(align_corners), od, prec)


def integrate_tensor_3d_with_coordinates(volumes, coord_volumes, softmax=True, *, multiplier=1.0,
                                         return_volumes=True, out_dtype=None):
    """3D soft-argmax: returns (coordinates (B, J, 3), normalised volumes (B, J, Vx, Vy, Vz)).

    Reference: ``mvn/utils/op.py:84-96``.  ``multiplier`` fuses the caller's
    ``volumes * volume_multiplier`` (triangulation.py:353).  With ``softmax=False``
    the reference applies relu and does NOT normalise the mass (op.py:91); so do we.
    """
    vol = volumes
    if vol.dtype not in (torch.float32, torch.bfloat16):
        vol = vol.float()
    if vol.dim() != 5:
        raise RuntimeError(f"volumes must be (B, J, Vx, Vy, Vz), got {tuple(vol.shape)}")
    Vx, Vy, Vz = vol.shape[2:]
    if vol.stride(4) != 1 or vol.stride(3) != Vz or vol.stride(2) != Vy * Vz:
        vol = vol.contiguous()
    od = _dtype_code(out_dtype if out_dtype is not None else vol.dtype)
    if _is_cuboids(coord_volumes):
        cub = coord_volumes
        if cub.shape != (vol.shape[0], Vx, Vy, Vz, 3):
            raise RuntimeError(f"cuboids {tuple(cub.shape)} do not match volumes {tuple(vol.shape)}")
        if _needs_grad(vol):
            xyz, out = SoftArgmaxCuboidFunction.apply(vol, cub.params, cub.volume_size, cub.transfer, bool(softmax),
                                                      float(multiplier), bool(return_volumes), od)
        else:
            xyz, out = _ops.call(_ops.softargmax3d_cuboid, vol, cub.params, cub.transfer, bool(softmax),
                                 float(multiplier), bool(return_volumes), od)
        return xyz, (out if return_volumes else None)
    coords = _ops.f32c(coord_volumes)
    if coords.shape != (vol.shape[0], Vx, Vy, Vz, 3):
        raise RuntimeError(f"coord_volumes {tuple(coords.shape)} does not match volumes {tuple(vol.shape)}")
    args = (vol, coords, bool(softmax), float(multiplier), bool(return_volumes), od)
    xyz, out = SoftArgmaxFunction.apply(*args) if _needs_grad(vol) else _ops.call(_ops.softargmax3d, *args)
    return xyz, (out if return_volumes else None)


def integrate_tensor_2d(heatmaps, softmax=True, *, multiplier=1.0, return_heatmaps=True, out_dtype=None):
    """2D soft-argmax: returns (coordinates (B, J, 2) as (x, y) in pixels, heatmaps (B, J, H, W)).

    Reference: ``mvn/utils/op.py:11-47``.  ``multiplier`` fuses the caller's
    ``heatmaps * heatmap_multiplier`` (triangulation.py:164).  The returned maps are
    softmax-normalised, or relu'd and NOT normalised for ``softmax=False`` (op.py:27),
    whose coordinates are divided by the mass (op.py:40-42).
    """
    hm = heatmaps
    if hm.dtype not in (torch.float32, torch.bfloat16):
        hm = hm.float()
    if hm.dim() != 4:
        raise RuntimeError(f"heatmaps must be (B, J, H, W), got {tuple(hm.shape)}")
    hm = hm.contiguous()
    od = _dtype_code(out_dtype if out_dtype is not None else hm.dtype)
    args = (hm, bool(softmax), float(multiplier), bool(return_heatmaps), od)
    xy, maps = SoftArgmax2dFunction.apply(*args) if _needs_grad(hm) else _ops.call(_ops.softargmax2d, *args)
    return xy, (maps if return_heatmaps else None)


class UnprojectFunction(torch.autograd.Function):
    """autograd surface of op.py:99-163; backward: csrc/unproject_bwd.hip (grads w.r.t. the
    features and, for 'conf*', the confidences)."""

    @staticmethod
    def forward(ctx, feat, proj, coords, conf, agg, align_corners, out_dtype, precision=_lib.MVN_PRECISION_EXACT):
        out = _ops.call(_ops.unproject, feat, proj, coords, conf, agg, align_corners, out_dtype, precision)
        ctx.save_for_backward(feat, proj, coords, conf)
        ctx.cfg = (agg, align_corners)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import _backward
        return _backward.unproject_backward(ctx, grad_out) + (None,)


class SoftArgmaxFunction(torch.autograd.Function):
    """autograd surface of op.py:84-96; backward: csrc/backward.hip."""

    @staticmethod
    def forward(ctx, vol, coords, softmax, multiplier, return_volume, out_dtype):
        xyz, out = _ops.call(_ops.softargmax3d, vol, coords, softmax, multiplier, return_volume, out_dtype)
        ctx.save_for_backward(vol, coords)
        ctx.cfg = (softmax, multiplier, return_volume)
        return xyz, out

    @staticmethod
    def backward(ctx, grad_xyz, grad_out):
        from . import _backward
        return _backward.softargmax_backward(ctx, grad_xyz, grad_out)


class UnprojectCuboidFunction(torch.autograd.Function):
    """UnprojectFunction with the coordinates formed in-kernel from per-frame cuboids
    (csrc/unproject_tiled.hip, cuboid_coord); backward materialises the coordinate volume
    (one small kernel) and runs the same backward kernel."""

    @staticmethod
    def forward(ctx, feat, proj, cub, V, transfer, conf, agg, align_corners, out_dtype,
                precision=_lib.MVN_PRECISION_EXACT):
        out = _ops.call(_ops.unproject_cuboid, feat, proj, cub, V, transfer, conf, agg, align_corners, out_dtype,
                        precision)
        ctx.save_for_backward(feat, proj, cub, conf)
        ctx.cfg = (V, transfer, agg, align_corners)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import _backward
        from .volumetric import Cuboids
        feat, proj, cub, conf = ctx.saved_tensors
        V, transfer, agg, align_corners = ctx.cfg
        want_conf = conf is not None and ctx.needs_input_grad[5]
        if not (ctx.needs_input_grad[0] or want_conf):
            return (None,) * 10
        coords = Cuboids(cub, V, transfer).coord_volumes()
        gfeat, gconf = _ops.call(_backward.unproject_bwd, feat, proj, coords, conf, grad_out, agg, align_corners, want_conf)
        return (gfeat if ctx.needs_input_grad[0] else None, None, None, None, None,
                gconf if want_conf else None, None, None, None, None)


class SoftArgmaxCuboidFunction(torch.autograd.Function):
    """SoftArgmaxFunction with in-kernel coordinates (csrc/softargmax.hip, cuboid_coord)."""

    @staticmethod
    def forward(ctx, vol, cub, V, transfer, softmax, multiplier, return_volume, out_dtype):
        xyz, out = _ops.call(_ops.softargmax3d_cuboid, vol, cub, transfer, softmax, multiplier, return_volume, out_dtype)
        ctx.save_for_backward(vol, cub)
        ctx.cfg = (V, transfer, softmax, multiplier, return_volume)
        return xyz, out

    @staticmethod
    def backward(ctx, grad_xyz, grad_out):
        from . import _backward
        from .volumetric import Cuboids
        vol, cub = ctx.saved_tensors
        V, transfer, softmax, multiplier, return_volume = ctx.cfg
        if not ctx.needs_input_grad[0]:
            return (None,) * 8
        coords = Cuboids(cub, V, transfer).coord_volumes()
        gv = grad_out if (return_volume and grad_out is not None and grad_out.numel() > 0) else None
        gin = _ops.call(_backward.softargmax3d_bwd, vol, coords, softmax, multiplier, grad_xyz, gv)
        return (gin,) + (None,) * 7


class SoftArgmax2dFunction(torch.autograd.Function):
    """autograd surface of op.py:11-47; backward in _backward.softargmax2d_backward."""

    @staticmethod
    def forward(ctx, hm, softmax, multiplier, return_maps, out_dtype):
        xy, maps = _ops.call(_ops.softargmax2d, hm, softmax, multiplier, return_maps, out_dtype)
        ctx.save_for_backward(hm, xy)
        ctx.cfg = (softmax, multiplier)
        return xy, maps

    @staticmethod
    def backward(ctx, grad_xy, grad_maps):
        from . import _backward
        return _backward.softargmax2d_backward(ctx, grad_xy, grad_maps)
