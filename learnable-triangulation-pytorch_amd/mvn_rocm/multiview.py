"""Drop-in replacements for the DLT functions of ``mvn/utils/multiview.py``."""
from __future__ import annotations

import torch

from . import _ops


def triangulate_batch_of_points(proj_matricies_batch, points_batch, confidences_batch=None):
    """Confidence-weighted linear triangulation of (B, J) points from N views.

    Reference: ``mvn/utils/multiview.py:162-174`` (+ solver ``:132-159``).
      proj_matricies_batch (B, N, 3, 4), points_batch (B, N, J, 2),
      confidences_batch (B, N, J) or None  ->  (B, J, 3) float32.
    The null vector is computed in float64 (the float32 reference
    SVD itself deviates from float64 by up to ~2e-4 relative).
    """
    if proj_matricies_batch.shape[:2] != points_batch.shape[:2]:   # multiview.py:143
        raise AssertionError("proj_matricies and points must have the same number of views")
    proj = _ops.f32c(proj_matricies_batch)
    pts = _ops.f32c(points_batch)
    conf = None if confidences_batch is None else _ops.f32c(confidences_batch)
    if torch.is_grad_enabled() and (pts.requires_grad or (conf is not None and conf.requires_grad)):
        return DLTFunction.apply(proj, pts, conf)
    return _ops.call(_ops.dlt, proj, pts, conf)


def triangulate_point_from_multiple_views_linear_torch(proj_matricies, points, confidences=None):
    """Single point: proj (N, 3, 4), points (N, 2), confidences (N,) -> (3,).

    Reference: ``mvn/utils/multiview.py:132-159``.
    """
    if len(proj_matricies) != len(points):                          # multiview.py:143
        raise AssertionError("proj_matricies and points must have the same number of views")
    conf = None if confidences is None else confidences.reshape(1, -1, 1)
    return triangulate_batch_of_points(proj_matricies.unsqueeze(0), points.reshape(1, -1, 1, 2), conf)[0, 0]


class DLTFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, proj, pts, conf):
        out = _ops.call(_ops.dlt, proj, pts, conf)
        ctx.save_for_backward(proj, pts, conf)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import _backward
        return _backward.dlt_backward(ctx, grad_out)
