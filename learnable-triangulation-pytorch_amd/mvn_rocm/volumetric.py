"""Coordinate volumes of the volumetric model on the GPU.

``build_coord_volumes`` replaces the per-frame Python loop of
``mvn/models/triangulation.py:280-341`` (about ten ATen launches per frame) by one
kernel (``mvn_coord_volumes``, csrc/coord_volumes.hip).  The small per-frame geometry —
cuboid position, rotation matrix (``mvn/utils/volumetric.py:87-100``) — is formed on the
host in float64 exactly as the reference's numpy does, then rounded to float32 where
torch rounds it; the V^3 grid, rotation and re-axing run on the device with the
reference's f32 op order (bit-exact, tests/test_gpu_parity.py).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._ops import _require_gpu


def rotation_matrix(axis, theta: float) -> np.ndarray:
    """Counter-clockwise rotation by theta about axis (the quaternion form of
    volumetric.py:87-100), float64."""
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.sqrt(np.dot(axis, axis))
    a = np.cos(theta / 2.0)
    b, c, d = -axis * np.sin(theta / 2.0)
    aa, bb, cc, dd = a * a, b * b, c * c, d * d
    bc, ad, ac, ab, bd, cd = b * c, a * d, a * c, a * b, b * d, c * d
    return np.array([[aa + bb - cc - dd, 2 * (bc + ad), 2 * (bd - ac)],
                     [2 * (bc - ad), aa + cc - bb - dd, 2 * (cd + ab)],
                     [2 * (bd + ac), 2 * (cd - ab), aa + dd - bb - cc]])


CUBOID_FLOATS = 18     # MVN_CUBOID_FLOATS: position[3], centre[3], step[3], rot[9] per frame


class Cuboids:
    """Per-frame cuboid geometry of the volumetric model (triangulation.py:280-341), on the GPU.

    ``params`` (B, 18) f32 = position, centre, step, rotation per frame, rounded to f32 as
    the reference's torch code rounds them.  ``coord_volumes()`` materialises the
    (B, V, V, V, 3) volume (``mvn_coord_volumes``); ``op.unproject_heatmaps`` and
    ``op.integrate_tensor_3d_with_coordinates`` also accept a ``Cuboids`` in place of the
    volume and then form the coordinates in-kernel (``mvn_*_cuboid``), bit-identically.
    """

    def __init__(self, params: torch.Tensor, volume_size: int, transfer_cmu_to_human36m: bool = False):
        if params.dim() != 2 or params.shape[1] != CUBOID_FLOATS or params.dtype != torch.float32:
            raise RuntimeError(f"cuboid params must be (B, {CUBOID_FLOATS}) float32, got {tuple(params.shape)}")
        self.params = params.contiguous()
        self.volume_size = int(volume_size)
        self.transfer = bool(transfer_cmu_to_human36m)

    @property
    def batch(self) -> int:
        return self.params.shape[0]

    @property
    def shape(self):
        """Shape of the coordinate volume these cuboids stand for."""
        V = self.volume_size
        return torch.Size((self.batch, V, V, V, 3))

    @property
    def device(self):
        return self.params.device

    def coord_volumes(self) -> torch.Tensor:
        """(B, V, V, V, 3) f32 coordinate volume (one kernel launch)."""
        _require_gpu(self.params)
        B, V = self.batch, self.volume_size
        out = torch.empty((B, V, V, V, 3), dtype=torch.float32, device=self.device)
        if out.numel() == 0:
            return out
        # mvn_coord_volumes takes the four fields as separate (B, k) arrays
        fields = [self.params[:, 0:3].contiguous(), self.params[:, 3:6].contiguous(),
                  self.params[:, 6:9].contiguous(), self.params[:, 9:18].contiguous()]
        code = _lib.load().mvn_coord_volumes(*(f.data_ptr() for f in fields), out.data_ptr(), B, V,
                                             int(self.transfer), torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(code, "mvn_coord_volumes")
        return out


def build_cuboids(base_points, cuboid_side: float, volume_size: int, theta=0.0, kind: str = "coco",
                  transfer_cmu_to_human36m: bool = False, device="cuda") -> Cuboids:
    """Per-frame cuboids of triangulation.py:280-341 (same arguments as build_coord_volumes)."""
    base = np.asarray(base_points.detach().cpu().numpy() if torch.is_tensor(base_points) else base_points,
                      dtype=np.float64).reshape(-1, 3)
    B, V = base.shape[0], int(volume_size)
    thetas = np.broadcast_to(np.asarray(theta, dtype=np.float64), (B,))
    if kind == "coco":
        axis = [0, 1, 0]
    elif kind == "mpii":
        axis = [0, 0, 1]
    else:
        raise ValueError(f"unknown kind {kind!r} (expected 'coco' or 'mpii')")
    sides = np.array([cuboid_side, cuboid_side, cuboid_side], dtype=np.float64)
    position = (base - sides / 2).astype(np.float32)                               # :300, then f32 (:313)
    step = np.broadcast_to((sides / (V - 1)).astype(np.float32), (B, 3)).copy()     # :313-315
    centre = base.astype(np.float32)                                                 # :330
    rot = (np.stack([rotation_matrix(axis, t) for t in thetas]) if B else np.zeros((0, 3, 3))).astype(np.float32)
    host = np.concatenate([position, centre, step, rot.reshape(B, 9)], axis=1)
    params = torch.from_numpy(np.ascontiguousarray(host)).to(torch.device(device))
    return Cuboids(params, V, transfer_cmu_to_human36m)


def build_coord_volumes(base_points, cuboid_side: float, volume_size: int, theta=0.0, kind: str = "coco",
                        transfer_cmu_to_human36m: bool = False, device="cuda"):
    """(B, V, V, V, 3) float32 coordinate volumes on ``device``.

    base_points: (B, 3) float64 array (the pelvis of each frame, triangulation.py:288-293);
    theta: scalar or (B,) rotation angles (0 in eval, uniform [0, 2pi) in training,
    triangulation.py:320-323); kind: 'coco' rotates about y, 'mpii' about z (:325-328).
    """
    return build_cuboids(base_points, cuboid_side, volume_size, theta, kind, transfer_cmu_to_human36m,
                         device).coord_volumes()
