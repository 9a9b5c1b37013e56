"""Seeded synthetic inputs for the hot path and the caller-side
geometry the models build around it.

Nothing here touches the reference; the same generators feed the bench, the GPU
parity tests and the golden-fixture script.  Every frame is generated from
(seed, global frame index) alone, so a rank of a sharded run can build exactly its
own frames on its own device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

IMAGE_SIZE = 384          # experiments/human36m/train/human36m_vol_softmax.yaml:6
HEATMAP_SIZE = 96         # PoseResNet output stride 4 (pose_resnet.py:205-226)
CUBOID_SIDE = 2500.0      # human36m_vol_softmax.yaml: cuboid_side
VOLUME_SIZE = 64          # human36m_vol_softmax.yaml: volume_size


@dataclass
class Camera:
    """Pinhole camera with the reference's intrinsics update rules (multiview.py:5-43)."""
    R: np.ndarray
    t: np.ndarray
    K: np.ndarray

    def update_after_resize(self, image_shape, new_image_shape):   # multiview.py:24-35
        height, width = image_shape
        new_width, new_height = new_image_shape
        sx, sy = new_width / width, new_height / height
        self.K = self.K.copy()
        self.K[0, 0] *= sx
        self.K[1, 1] *= sy
        self.K[0, 2] *= sx
        self.K[1, 2] *= sy

    @property
    def projection(self) -> np.ndarray:                            # multiview.py:37-43
        return self.K.dot(np.hstack([self.R, self.t]))


def _frame_rng(seed: int, frame: int) -> np.random.Generator:
    return np.random.default_rng([seed, frame])


def ring_cameras(n_views: int, rng: np.random.Generator, image_size: int = IMAGE_SIZE,
                 target=(0.0, 0.0, 900.0)) -> list:
    """N look-at cameras on a 5 m ring, height 1500 +- 200 mm, f = 800 px at 384^2 (z up)."""
    cams = []
    f = 800.0 * image_size / IMAGE_SIZE
    c = image_size / 2.0
    tgt = np.asarray(target, dtype=np.float64)
    for v in range(n_views):
        az = 2.0 * math.pi * v / n_views + rng.uniform(-0.2, 0.2)
        pos = np.array([5000.0 * math.cos(az), 5000.0 * math.sin(az), 1500.0 + rng.uniform(-200.0, 200.0)])
        fwd = tgt - pos
        fwd /= np.linalg.norm(fwd)
        right = np.cross(fwd, np.array([0.0, 0.0, 1.0]))
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        R = np.stack([right, down, fwd])                 # world -> camera
        t = (-R @ pos).reshape(3, 1)
        K = np.array([[f, 0.0, c], [0.0, f, c], [0.0, 0.0, 1.0]])
        cams.append(Camera(R, t, K))
    return cams


def projections(cams, image_size=IMAGE_SIZE, heatmap_size=HEATMAP_SIZE) -> np.ndarray:
    """(N, 3, 4) float64 projection matrices at heatmap resolution, via the
    reference's update_after_resize path (triangulation.py:272-278)."""
    out = []
    for cam in cams:
        c2 = Camera(cam.R, cam.t, cam.K.copy())
        c2.update_after_resize((image_size, image_size), (heatmap_size, heatmap_size))
        out.append(c2.projection)
    return np.stack(out)


def rotation_matrix(axis, theta: float) -> np.ndarray:
    """Counter-clockwise rotation about `axis` (quaternion form of volumetric.py:87-99)."""
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / math.sqrt(float(axis @ axis))
    a = math.cos(theta / 2.0)
    b, c, d = -axis * math.sin(theta / 2.0)
    return np.array([
        [a * a + b * b - c * c - d * d, 2 * (b * c + a * d), 2 * (b * d - a * c)],
        [2 * (b * c - a * d), a * a + c * c - b * b - d * d, 2 * (c * d + a * b)],
        [2 * (b * d + a * c), 2 * (c * d - a * b), a * a + d * d - b * b - c * c]])


def coord_volume(base_point: np.ndarray, theta: float, volume_size: int = VOLUME_SIZE,
                 cuboid_side: float = CUBOID_SIDE, kind: str = "coco", device="cpu",
                 transfer_cmu_to_human36m: bool = False) -> torch.Tensor:
    """(V, V, V, 3) float32 world coordinates of a cuboid around `base_point`, built with
    the op order of triangulation.py:295-339 (meshgrid 'ij', position + step * index,
    rotation about the base point, optional CMU -> H36M axis transfer)."""
    V = volume_size
    position = np.asarray(base_point, dtype=np.float64) - cuboid_side / 2.0
    step = cuboid_side / (V - 1)
    ar = torch.arange(V, device=device)
    grid = torch.stack(torch.meshgrid(ar, ar, ar, indexing="ij"), dim=-1).to(torch.float32).reshape(-1, 3)
    gc = torch.empty_like(grid)
    for k in range(3):
        gc[:, k] = float(position[k]) + step * grid[:, k]
    vol = gc.reshape(V, V, V, 3)
    center = torch.from_numpy(np.asarray(base_point, dtype=np.float64)).to(torch.float32).to(device)
    axis = [0, 1, 0] if kind == "coco" else [0, 0, 1]
    rot = torch.from_numpy(rotation_matrix(axis, theta)).to(torch.float32).to(device)
    vol = vol - center
    vol = rot.mm(vol.reshape(-1, 3).t()).t().reshape(V, V, V, 3)
    vol = vol + center
    if transfer_cmu_to_human36m:
        vol = vol.permute(0, 2, 1, 3)
        vol = vol.index_select(1, torch.arange(V - 1, -1, -1, device=device))
    return vol


@dataclass
class VolumetricBatch:
    features: torch.Tensor        # (B, N, C, H, W)
    proj: torch.Tensor            # (B, N, 3, 4) float32, heatmap resolution
    coords: torch.Tensor          # (B, V, V, V, 3) float32
    base_points: torch.Tensor     # (B, 3)
    base_points64: np.ndarray = None   # (B, 3) float64 (what the coordinate volumes are built from)
    thetas: np.ndarray = None          # (B,) rotation angles
    kind: str = "coco"

    def cuboids(self, device="cuda"):
        """The same coordinate volumes as per-frame cuboids (in-kernel coordinates,
        mvn_rocm.volumetric.Cuboids)."""
        from .volumetric import build_cuboids
        return build_cuboids(self.base_points64, CUBOID_SIDE, self.coords.shape[1], self.thetas, self.kind,
                             device=device)


def volumetric_batch(batch: int, n_views: int = 4, channels: int = 32, heatmap: int = HEATMAP_SIZE,
                     volume: int = VOLUME_SIZE, dtype=torch.float32, device="cpu", seed: int = 0,
                     first_frame: int = 0, rotate: bool = True, kind: str = "coco") -> VolumetricBatch:
    """Frames [first_frame, first_frame + batch) of the seeded synthetic workload."""
    feats, projs, coords, bases, bases64, thetas = [], [], [], [], [], []
    for f in range(first_frame, first_frame + batch):
        rng = _frame_rng(seed + 1, f)
        cams = ring_cameras(n_views, rng)
        projs.append(torch.from_numpy(projections(cams, heatmap_size=heatmap)).to(torch.float32))
        base = np.array([rng.uniform(-500, 500), rng.uniform(-500, 500), rng.uniform(800, 1000)])
        theta = rng.uniform(0.0, 2.0 * math.pi) if rotate else 0.0
        bases.append(torch.from_numpy(base).to(torch.float32))
        bases64.append(base)
        thetas.append(theta)
        coords.append(coord_volume(base, theta, volume, kind=kind, device=device))
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1_000_003 + f)
        feats.append(torch.randn((n_views, channels, heatmap, heatmap), generator=g, device=device))
    return VolumetricBatch(
        features=torch.stack(feats).to(dtype),
        proj=torch.stack(projs).to(device),
        coords=torch.stack(coords),
        base_points=torch.stack(bases).to(device),
        base_points64=np.stack(bases64), thetas=np.asarray(thetas, dtype=np.float64), kind=kind)


def blob_volumes(coords: torch.Tensor, n_joints: int = 17, seed: int = 0, first_frame: int = 0,
                 sigma_vox: float = 3.0, noise: float = 1.0, peak: float = 10.0) -> torch.Tensor:
    """(B, J, V, V, V) soft-argmax logits: a Gaussian blob of height `peak` at a random
    voxel per joint plus N(0, noise^2)."""
    B, Vx, Vy, Vz = coords.shape[:4]
    dev = coords.device
    out = torch.empty((B, n_joints, Vx, Vy, Vz), device=dev, dtype=torch.float32)
    ix = torch.arange(Vx, device=dev, dtype=torch.float32).view(Vx, 1, 1)
    iy = torch.arange(Vy, device=dev, dtype=torch.float32).view(1, Vy, 1)
    iz = torch.arange(Vz, device=dev, dtype=torch.float32).view(1, 1, Vz)
    for b in range(B):
        rng = _frame_rng(seed + 2, first_frame + b)
        g = torch.Generator(device=dev)
        g.manual_seed(seed * 7_000_003 + first_frame + b)
        for j in range(n_joints):
            cx, cy, cz = rng.integers(0, Vx), rng.integers(0, Vy), rng.integers(0, Vz)
            d2 = (ix - cx) ** 2 + (iy - cy) ** 2 + (iz - cz) ** 2
            out[b, j] = peak * torch.exp(-d2 / (2 * sigma_vox ** 2)) + noise * torch.randn(
                (Vx, Vy, Vz), generator=g, device=dev)
    return out


@dataclass
class AlgebraicBatch:
    proj: torch.Tensor            # (B, N, 3, 4) float32, image resolution
    points: torch.Tensor          # (B, N, J, 2) float32, pixels
    confidences: torch.Tensor     # (B, N, J) float32, normalised over views + 1e-5
    points_3d: torch.Tensor       # (B, J, 3) float64 ground truth


def algebraic_batch(batch: int = 1, n_views: int = 4, n_joints: int = 17, seed: int = 0,
                    first_frame: int = 0, noise_px: float = 2.0) -> AlgebraicBatch:
    """Config 1 of BASELINE.json: random 3D joints within +-900 mm of the pelvis,
    projected through N ring cameras at 384^2, + N(0, 2 px) noise, confidences
    U(0.1, 1) normalised over views + 1e-5 (triangulation.py:173-174)."""
    projs, pts, confs, gts = [], [], [], []
    for f in range(first_frame, first_frame + batch):
        rng = _frame_rng(seed + 3, f)
        cams = ring_cameras(n_views, rng)
        P = np.stack([c.projection for c in cams])                      # (N, 3, 4) float64
        X = np.array([0.0, 0.0, 900.0]) + rng.uniform(-900, 900, size=(n_joints, 3))
        Xh = np.concatenate([X, np.ones((n_joints, 1))], axis=1)
        uvw = np.einsum("nrk,jk->njr", P, Xh)
        uv = uvw[..., :2] / uvw[..., 2:] + rng.normal(0.0, noise_px, size=(n_views, n_joints, 2))
        c = rng.uniform(0.1, 1.0, size=(n_views, n_joints))
        projs.append(P)
        pts.append(uv)
        confs.append(c)
        gts.append(X)
    conf = torch.from_numpy(np.stack(confs)).to(torch.float32)
    conf = conf / conf.sum(dim=1, keepdim=True)
    conf = conf + 1e-5
    return AlgebraicBatch(
        proj=torch.from_numpy(np.stack(projs)).to(torch.float32),
        points=torch.from_numpy(np.stack(pts)).to(torch.float32),
        confidences=conf,
        points_3d=torch.from_numpy(np.stack(gts)))
