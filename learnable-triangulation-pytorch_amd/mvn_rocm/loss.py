"""VolumetricCELoss on the GPU (mvn/models/loss.py:52-80).

Same module name, forward signature and value as the reference.  The reference builds a
(J, V^3) distance volume per frame and moves the argmin indices to the host
(``.detach().cpu().numpy()``, loss.py:66-67) — a device sync per frame.  Here one kernel
(``mvn_nearest_voxel``) finds every (frame, joint)'s nearest voxel on the device and the
loss is a gather: ``sum(validity * -log(p[b, j, idx] + 1e-6)) / (B * J)``, differentiable
w.r.t. the predicted volumes through torch's gather.
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib
from ._ops import _require_gpu


def nearest_voxel(coord_volumes: torch.Tensor, keypoints: torch.Tensor) -> torch.Tensor:
    """(B, Vx, Vy, Vz, 3), (B, J, 3) -> (B, J) int64 flat index of each keypoint's nearest voxel."""
    c = coord_volumes.float().contiguous()
    k = keypoints.float().contiguous()
    _require_gpu(c, k)
    B, Vx, Vy, Vz = c.shape[:4]
    J = k.shape[1]
    if k.shape != (B, J, 3) or c.shape[4] != 3:
        raise RuntimeError(f"coord_volumes {tuple(c.shape)} / keypoints {tuple(k.shape)} mismatch")
    out = torch.empty((B, J), dtype=torch.int32, device=c.device)
    code = _lib.load().mvn_nearest_voxel(c.data_ptr(), k.data_ptr(), out.data_ptr(), B, J, Vx, Vy, Vz,
                                         torch.cuda.current_stream(c.device).cuda_stream)
    _lib.check(code, "mvn_nearest_voxel")
    return out.long()


class VolumetricCELoss(nn.Module):
    """loss.py:52-80: mean over (frame, joint) of validity * -log(p_nearest + 1e-6)."""

    def forward(self, coord_volumes_batch, volumes_batch_pred, keypoints_gt, keypoints_binary_validity):
        B, J = volumes_batch_pred.shape[:2]
        idx = nearest_voxel(coord_volumes_batch, keypoints_gt)                        # (B, J)
        p = volumes_batch_pred.reshape(B, J, -1).gather(2, idx.unsqueeze(-1)).squeeze(-1)
        validity = keypoints_binary_validity.reshape(B, J, -1)[..., 0].to(p.dtype)   # validity[0] (loss.py:72)
        return (validity * -torch.log(p + 1e-6)).sum() / (B * J)
