"""ORACLE — test infrastructure only.

Op-for-op torch-CPU restatement of the reference hot path.  It issues the same ATen
calls in the same order inside the same B x N (unproject) and B x J (DLT) Python
loops as the reference, so on CPU it produces the reference's bits (pinned by
tests/test_oracle.py against tests/golden/).  bench.py times it on the GPU box's host
cores as the CPU baseline (cpu_baseline.kind = "port"): the reference itself cannot
travel to the box.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _to_homogeneous(p):                       # multiview.py:57-58
    return torch.cat([p, torch.ones((p.shape[0], 1), dtype=p.dtype, device=p.device)], dim=1)


def _from_homogeneous(p):                     # multiview.py:74-75
    pt = p.transpose(1, 0)
    return (pt[:-1] / pt[-1]).transpose(1, 0)


def unproject_heatmaps(heatmaps, proj_matricies, coord_volumes, volume_aggregation_method="sum",
                       vol_confidences=None, align_corners=None):
    """mvn/utils/op.py:99-163.  align_corners=None keeps torch's default (False, with its
    warning) exactly like the reference call at op.py:134."""
    dev = heatmaps.device
    n_batch, n_views, n_ch = heatmaps.shape[:3]
    hm_shape = tuple(heatmaps.shape[3:])
    vol_shape = coord_volumes.shape[1:4]
    gs_kwargs = {} if align_corners is None else {"align_corners": bool(align_corners)}

    result = torch.zeros(n_batch, n_ch, *vol_shape, device=dev)                 # op.py:104
    for b in range(n_batch):                                                    # op.py:107
        pts_h = _to_homogeneous(coord_volumes[b].reshape((-1, 3)))
        per_view = torch.zeros(n_views, n_ch, *vol_shape, device=dev)           # op.py:111
        for v in range(n_views):                                                # op.py:113
            proj = pts_h @ proj_matricies[b, v].t()                             # op.py:117 -> multiview.py:96
            behind = proj[:, 2] <= 0.0                                          # op.py:121
            proj[proj[:, 2] == 0.0, 2] = 1.0                                    # op.py:123
            uv = _from_homogeneous(proj)                                        # op.py:124
            grid = torch.zeros_like(uv)                                         # op.py:127-130
            grid[:, 0] = 2 * (uv[:, 0] / hm_shape[0] - 0.5)
            grid[:, 1] = 2 * (uv[:, 1] / hm_shape[1] - 0.5)
            sampled = F.grid_sample(heatmaps[b, v].unsqueeze(0), grid.unsqueeze(1).unsqueeze(0), **gs_kwargs)
            sampled = sampled.view(n_ch, -1)                                    # op.py:137-138
            sampled[:, behind] = 0.0
            per_view[v] = sampled.view(n_ch, *vol_shape)                        # op.py:141-144

        m = volume_aggregation_method
        if m.startswith("conf"):                                                # op.py:147-148
            result[b] = (per_view * vol_confidences[b].view(n_views, n_ch, 1, 1, 1)).sum(0)
        elif m == "sum":
            result[b] = per_view.sum(0)
        elif m == "max":
            result[b] = per_view.max(0)[0]
        elif m == "softmax":                                                    # op.py:153-159
            w = F.softmax(per_view.clone().view(n_views, -1), dim=0).view(n_views, n_ch, *vol_shape)
            result[b] = (per_view * w).sum(0)
        else:
            raise ValueError("Unknown volume_aggregation_method: {}".format(m))
    return result


def integrate_tensor_3d_with_coordinates(volumes, coord_volumes, softmax=True):
    """mvn/utils/op.py:84-96."""
    n_batch, n_vol = volumes.shape[:2]
    spatial = volumes.shape[2:]
    flat = volumes.reshape((n_batch, n_vol, -1))
    flat = F.softmax(flat, dim=2) if softmax else F.relu(flat)
    vols = flat.reshape((n_batch, n_vol, *spatial))
    return torch.einsum("bnxyz, bxyzc -> bnc", vols, coord_volumes), vols


def integrate_tensor_2d(heatmaps, softmax=True):
    """mvn/utils/op.py:11-47: normalise each flattened map, project its mass onto the two
    axes, take the first moments (relu mode: divided by the mass)."""
    n_batch, n_maps, h, w = heatmaps.shape
    flat = heatmaps.reshape((n_batch, n_maps, -1))
    flat = F.softmax(flat, dim=2) if softmax else F.relu(flat)
    maps = flat.reshape((n_batch, n_maps, h, w))
    col_mass = maps.sum(dim=2)                      # over rows -> mass per column (x)
    row_mass = maps.sum(dim=3)                      # over columns -> mass per row (y)
    x = (col_mass * torch.arange(w).type(torch.float).to(maps.device)).sum(dim=2, keepdim=True)
    y = (row_mass * torch.arange(h).type(torch.float).to(maps.device)).sum(dim=2, keepdim=True)
    if not softmax:
        x = x / col_mass.sum(dim=2, keepdim=True)
        y = y / row_mass.sum(dim=2, keepdim=True)
    return torch.cat((x, y), dim=2).reshape((n_batch, n_maps, 2)), maps


def triangulate_batch_of_points(proj_matricies_batch, points_batch, confidences_batch=None):
    """mvn/utils/multiview.py:162-174 with the solver of :132-159 inlined."""
    n_batch, n_views, n_joints = points_batch.shape[:3]
    out = torch.zeros(n_batch, n_joints, 3, dtype=torch.float32, device=points_batch.device)
    for b in range(n_batch):
        P = proj_matricies_batch[b]
        for j in range(n_joints):
            pts = points_batch[b, :, j, :]
            if confidences_batch is not None:
                conf = confidences_batch[b, :, j]
            else:
                conf = torch.ones(n_views, dtype=torch.float32, device=pts.device)
            A = P[:, 2:3].expand(n_views, 2, 4) * pts.view(n_views, 2, 1)       # multiview.py:150
            A -= P[:, :2]                                                       # :151
            A *= conf.view(-1, 1, 1)                                            # :152
            _, _, V = torch.svd(A.view(-1, 4))                                  # :154
            X = -V[:, 3]                                                        # :156
            out[b, j] = _from_homogeneous(X.unsqueeze(0))[0]                    # :157
    return out


def build_coord_volumes(base_points, cuboid_side, volume_size, thetas, kind="coco", transfer_cmu=False,
                        rotate=None):
    """mvn/models/triangulation.py:280-341, the per-frame loop, op for op (torch CPU).
    ``rotate`` defaults to this module's restatement of volumetric.rotate_coord_volume
    (volumetric.py:103-114); the golden script passes the reference's own function."""
    import numpy as np
    rotate = rotate or rotate_coord_volume
    V = volume_size
    out = torch.zeros(len(base_points), V, V, V, 3)
    for b, base_point in enumerate(np.asarray(base_points, dtype=np.float64)):
        sides = np.array([cuboid_side, cuboid_side, cuboid_side])
        position = base_point - sides / 2
        xxx, yyy, zzz = torch.meshgrid(torch.arange(V), torch.arange(V), torch.arange(V), indexing="ij")
        grid = torch.stack([xxx, yyy, zzz], dim=-1).type(torch.float).reshape((-1, 3))
        grid_coord = torch.zeros_like(grid)
        for k in range(3):
            grid_coord[:, k] = position[k] + (sides[k] / (V - 1)) * grid[:, k]
        coord_volume = grid_coord.reshape(V, V, V, 3)
        axis = [0, 1, 0] if kind == "coco" else [0, 0, 1]
        center = torch.from_numpy(base_point).type(torch.float)
        coord_volume = coord_volume - center
        coord_volume = rotate(coord_volume, float(thetas[b]), axis)
        coord_volume = coord_volume + center
        if transfer_cmu:
            coord_volume = coord_volume.permute(0, 2, 1, 3)
            coord_volume = coord_volume.index_select(1, torch.arange(V - 1, -1, -1).long())
        out[b] = coord_volume
    return out


def rotate_coord_volume(coord_volume, theta, axis):
    """volumetric.py:103-114 (rotation matrix of :87-100 in float64, cast to f32, sgemm)."""
    import numpy as np
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.sqrt(np.dot(axis, axis))
    a = np.cos(theta / 2.0)
    b, c, d = -axis * np.sin(theta / 2.0)
    aa, bb, cc, dd = a * a, b * b, c * c, d * d
    bc, ad, ac, ab, bd, cd = b * c, a * d, a * c, a * b, b * d, c * d
    rot = np.array([[aa + bb - cc - dd, 2 * (bc + ad), 2 * (bd - ac)],
                    [2 * (bc - ad), aa + cc - bb - dd, 2 * (cd + ab)],
                    [2 * (bd + ac), 2 * (cd - ab), aa + dd - bb - cc]])
    rot = torch.from_numpy(rot).type(torch.float)
    shape = coord_volume.shape
    return rot.mm(coord_volume.reshape(-1, 3).t()).t().reshape(*shape)


def volumetric_ce_loss(coord_volumes_batch, volumes_batch_pred, keypoints_gt, keypoints_binary_validity):
    """mvn/models/loss.py:55-80: per frame a (J, V^3) distance volume, its argmin per joint,
    and the validity-weighted -log of the predicted probability there, summed in order."""
    import numpy as np
    loss, n_losses = 0.0, 0
    for b in range(volumes_batch_pred.shape[0]):
        dists = torch.sqrt(((coord_volumes_batch[b].unsqueeze(0)
                             - keypoints_gt[b].unsqueeze(1).unsqueeze(1).unsqueeze(1)) ** 2).sum(-1))
        idx = torch.argmin(dists.view(dists.shape[0], -1), dim=-1).detach().cpu().numpy()
        idx = np.stack(np.unravel_index(idx, volumes_batch_pred.shape[-3:]), axis=1)
        for j, (x, y, z) in enumerate(idx):
            loss += keypoints_binary_validity[b, j][0] * (-torch.log(volumes_batch_pred[b, j, x, y, z] + 1e-6))
            n_losses += 1
    return loss / n_losses
