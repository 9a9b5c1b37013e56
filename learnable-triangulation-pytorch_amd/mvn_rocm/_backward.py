"""Backward passes of the mvn_rocm autograd functions (HIP kernels: csrc/*_bwd.hip)."""
from __future__ import annotations


def unproject_backward(ctx, grad_out):
    raise NotImplementedError("mvn_rocm: unproject backward is not built yet")


def softargmax_backward(ctx, grad_xyz, grad_out):
    raise NotImplementedError("mvn_rocm: soft-argmax backward is not built yet")


def dlt_backward(ctx, grad_out):
    raise NotImplementedError("mvn_rocm: DLT backward is not built yet")
