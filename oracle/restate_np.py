"""ORACLE — test infrastructure only.

float64 restatements: the 2D soft-argmax (mvn/utils/op.py:11-47), the
confidence-weighted DLT (mvn/utils/multiview.py:132-174) and the 'sum' unprojection's
feature gradient (the exact sum of the forward's f32 tap products).
The design matrix is formed in float32 with the reference's three separately rounded
ops (multiview.py:150-152) and only the null-space solve is promoted to float64
(LAPACK gesdd via numpy).  This is the gate for the HIP DLT (<= 1e-6 relative): the
float32 reference SVD itself is ~2e-4 away from float64 on realistic cameras
(SURVEY.md §7, Appendix A), so no float32 ordering could meet 1e-4 against it.
"""
from __future__ import annotations

import numpy as np


def design_matrix(P: np.ndarray, pts: np.ndarray, conf) -> np.ndarray:
    """P (N,3,4), pts (N,2), conf (N,) or None -> A (2N,4) float32."""
    P = np.asarray(P, np.float32)
    pts = np.asarray(pts, np.float32)
    n = P.shape[0]
    c = np.ones(n, np.float32) if conf is None else np.asarray(conf, np.float32)
    A = np.broadcast_to(P[:, 2:3, :], (n, 2, 4)) * pts.reshape(n, 2, 1)   # :150
    A = A - P[:, :2, :]                                                   # :151
    A = A * c.reshape(-1, 1, 1)                                           # :152
    return A.reshape(-1, 4).astype(np.float32)


def triangulate_batch_of_points(proj, points, confidences=None) -> np.ndarray:
    """proj (B,N,3,4), points (B,N,J,2), confidences (B,N,J) -> (B,J,3) float64."""
    proj = np.asarray(proj)
    points = np.asarray(points)
    B, N, J = points.shape[:3]
    out = np.zeros((B, J, 3), np.float64)
    for b in range(B):
        for j in range(J):
            conf = None if confidences is None else np.asarray(confidences)[b, :, j]
            A = design_matrix(proj[b], points[b, :, j], conf).astype(np.float64)
            _, _, vh = np.linalg.svd(A, full_matrices=False)
            X = vh[-1]
            out[b, j] = X[:3] / X[3]
    return out


def integrate_tensor_2d(heatmaps, softmax=True):
    """mvn/utils/op.py:11-47 in float64: (B,J,H,W) -> ((B,J,2) (x, y), normalised maps)."""
    hm = np.asarray(heatmaps, np.float64)
    B, J, H, W = hm.shape
    flat = hm.reshape(B, J, -1)
    if softmax:
        e = np.exp(flat - flat.max(axis=2, keepdims=True))
        p = e / e.sum(axis=2, keepdims=True)
    else:
        p = np.maximum(flat, 0.0)
    p = p.reshape(B, J, H, W)
    mass = p.sum(axis=(2, 3))
    x = (p.sum(axis=2) * np.arange(W)).sum(axis=2)
    y = (p.sum(axis=3) * np.arange(H)).sum(axis=2)
    if not softmax:
        x, y = x / mass, y / mass
    return np.stack([x, y], axis=2), p


def coord_volumes(base_points, cuboid_side, volume_size, thetas, kind="coco", transfer_cmu=False):
    """mvn/models/triangulation.py:280-341 in numpy, reproducing the reference's f32 bits
    as the reference computes them on this container's CPU (MKL's K=3 sgemm accumulates
    rot.mm as an fma chain over k = 0, 1, 2; verified against tests/golden/coord_volumes.npz,
    which ran the reference's own rotate_coord_volume).  Host-independent, unlike a torch
    re-run, whose sgemm order follows the host's MKL code path."""
    f = np.float32

    def fma(a, b, c):
        return (np.float64(a) * np.float64(b) + np.float64(c)).astype(f)

    base_points = np.asarray(base_points, np.float64)
    V = int(volume_size)
    out = np.zeros((len(base_points), V, V, V, 3), f)
    i, j, k = np.meshgrid(np.arange(V), np.arange(V), np.arange(V), indexing="ij")
    g = (i, k, V - 1 - j) if transfer_cmu else (i, j, k)
    axis = np.array([0, 1, 0] if kind == "coco" else [0, 0, 1], np.float64)
    axis = axis / np.sqrt(np.dot(axis, axis))
    for b, base in enumerate(base_points):
        pos = (base - cuboid_side / 2.0).astype(f)
        st = f(cuboid_side / (V - 1))
        cen = base.astype(f)
        th = float(np.asarray(thetas, np.float64).reshape(-1)[b] if np.ndim(thetas) else thetas)
        a = np.cos(th / 2.0)
        bq, cq, dq = -axis * np.sin(th / 2.0)
        aa, bb, cc, dd = a * a, bq * bq, cq * cq, dq * dq
        bc, ad, ac, ab, bd, cd = bq * cq, a * dq, a * cq, a * bq, bq * dq, cq * dq
        R = np.array([[aa + bb - cc - dd, 2 * (bc + ad), 2 * (bd - ac)],
                      [2 * (bc - ad), aa + cc - bb - dd, 2 * (cd + ab)],
                      [2 * (bd + ac), 2 * (cd - ab), aa + dd - bb - cc]]).astype(f)
        d = [((pos[q] + (st * g[q].astype(f)).astype(f)).astype(f) - cen[q]).astype(f) for q in range(3)]
        out[b] = np.stack([(fma(R[r, 2], d[2], fma(R[r, 1], d[1], (R[r, 0] * d[0]).astype(f))) + cen[r]).astype(f)
                           for r in range(3)], -1)
    return out


def nearest_voxel(coords, keypoints):
    """(B,Vx,Vy,Vz,3), (B,J,3) -> (B,J) flat index of the nearest voxel (loss.py:63-66):
    f32 squared distance summed x, y, z in order, its IEEE square root, argmin with the
    first index on ties (distinct squared distances can round to one root).  NaN distances:
    numpy's argmin, like torch.argmin, returns the first NaN's index."""
    f = np.float32
    c = np.asarray(coords, f).reshape(len(coords), -1, 3)
    k = np.asarray(keypoints, f)
    d = c[:, None, :, :] - k[:, :, None, :]
    sq = (d * d).astype(f)
    d2 = ((sq[..., 0] + sq[..., 1]).astype(f) + sq[..., 2]).astype(f)
    return np.sqrt(d2).argmin(axis=2)


def _fma32(a, b, c):
    """f32 fma(a, b, c) through float64 (the product of two f32 is exact in float64)."""
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32)


def unproject_sum_feature_grad(feat_shape, proj, coords, grad_out, align_corners=False):
    """d(unproject_heatmaps(..., 'sum'))/d(heatmaps) (op.py:99-163, its autograd through
    grid_sampler_2d, op.py:134) as the EXACT float64 sum, per heatmap element, of the f32
    products grad_out * w of every voxel-view tap that reads it, w the forward's own f32
    bilinear weights: projection as the FMA chain of multiview.py:96, IEEE divisions
    (multiview.py:75, op.py:128-129), grid_sample's unnormalisation and corner weights
    (SURVEY.md §8a a1.1-a1.5).  This is what the deterministic backward computes before its
    final rounding; ATen's sequential float sum on the build container's CPU lies within a
    few 1e-7 of it."""
    f32 = np.float32
    B, N, C, H, W = feat_shape
    P = np.asarray(proj, np.float32)
    X = np.asarray(coords, np.float32).reshape(B, -1, 3)
    G = np.asarray(grad_out, np.float32).reshape(B, C, -1)
    acc = np.zeros((B, N, C, H, W), np.float64)
    for b in range(B):
        x, y, z = X[b, :, 0], X[b, :, 1], X[b, :, 2]
        for v in range(N):
            Pv = P[b, v]

            def row(r):
                t = (np.float64(x) * np.float64(Pv[r, 0])).astype(f32)
                t = _fma32(y, Pv[r, 1], t)
                t = _fma32(z, Pv[r, 2], t)
                return _fma32(f32(1), Pv[r, 3], t)
            uh, vh, wh = row(0), row(1), row(2)
            invalid = wh <= 0
            wh = np.where(wh == 0, f32(1), wh)
            gx = f32(2) * ((uh / wh).astype(f32) / f32(H) - f32(0.5))
            gy = f32(2) * ((vh / wh).astype(f32) / f32(W) - f32(0.5))
            if align_corners:
                ix = ((gx + f32(1)) * f32((W - 1) * 0.5)).astype(f32)
                iy = ((gy + f32(1)) * f32((H - 1) * 0.5)).astype(f32)
            else:
                ix = _fma32(gx + f32(1), f32(W * 0.5), f32(-0.5))
                iy = _fma32(gy + f32(1), f32(H * 0.5), f32(-0.5))
            x0, y0 = np.floor(ix), np.floor(iy)
            tx, ty = (ix - x0).astype(f32), (iy - y0).astype(f32)
            sx, sy = f32(1) - tx, f32(1) - ty
            for wt, dy, dx in ((sy * sx, 0, 0), (sy * tx, 0, 1), (ty * sx, 1, 0), (ty * tx, 1, 1)):
                xx, yy = x0.astype(np.int64) + dx, y0.astype(np.int64) + dy
                m = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H) & ~invalid
                for c in range(C):
                    np.add.at(acc[b, v, c], (yy[m], xx[m]),
                              (G[b, c][m] * wt[m].astype(f32)).astype(f32).astype(np.float64))
    return acc
