"""Host-side probe (design aid): the reference autograd backward of unproject_heatmaps (op.py:99-163,
ATen grid_sampler_2d backward on THIS host CPU) vs the exact sum of the f32 products g * w with the
forward's own bilinear weights — run on the GPU box host to see whether its ATen build rounds the
backward grid coordinate differently from the container where the goldens were captured.
    python tools/probe_bwd_host.py"""
import sys, numpy as np, torch
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/learnable-triangulation-pytorch_amd'); sys.path.insert(0,'/root/repo/tests')
from mvn_rocm import synth
from oracle import restate_torch
torch.set_num_threads(8)
vb = synth.volumetric_batch(2, n_views=4, channels=4, heatmap=32, volume=16, seed=8)
gout = torch.rand((2, 4, 16, 16, 16), generator=torch.Generator().manual_seed(6))
gout[1] *= 1e8
gout[0, 2] *= 1e-12
f = vb.features.clone().requires_grad_(True)
restate_torch.unproject_heatmaps(f, vb.proj, vb.coords, "sum").backward(gout)
ref = f.grad.numpy().astype(np.float64)
# exact f64 sum of f32 products g*w with the forward's f32 weights (what our kernel computes, pre-rounding)
B, N, C, H, W = vb.features.shape
f32 = np.float32
acc = np.zeros_like(ref)
P = vb.proj.numpy(); X = vb.coords.numpy().reshape(B, -1, 3)
G = gout.numpy().reshape(B, C, -1)
contrib = {}
for b in range(B):
    for v in range(N):
        x, y, z = X[b, :, 0], X[b, :, 1], X[b, :, 2]
        Pv = P[b, v]
        def row(r):  # fma chain
            t = (np.float64(x) * np.float64(Pv[r, 0])).astype(f32)
            t = (np.float64(y) * Pv[r, 1] + t).astype(f32)
            t = (np.float64(z) * Pv[r, 2] + t).astype(f32)
            return (np.float64(1) * Pv[r, 3] + t).astype(f32)
        uh, vh, wh = row(0), row(1), row(2)
        inv = wh <= 0
        wh = np.where(wh == 0, f32(1), wh)
        u = (uh / wh).astype(f32); vv = (vh / wh).astype(f32)
        gx = (f32(2) * ((u / f32(H)).astype(f32) - f32(0.5))).astype(f32)
        gy = (f32(2) * ((vv / f32(W)).astype(f32) - f32(0.5))).astype(f32)
        ix = (np.float64(gx + f32(1)) * np.float64(f32(W) * f32(0.5)) - 0.5).astype(f32)
        iy = (np.float64(gy + f32(1)) * np.float64(f32(H) * f32(0.5)) - 0.5).astype(f32)
        x0 = np.floor(ix); y0 = np.floor(iy)
        w_ = (ix - x0).astype(f32); n_ = (iy - y0).astype(f32)
        e_ = f32(1) - w_; s_ = f32(1) - n_
        for wt, dy, dx in ((s_*e_, 0, 0), (s_*w_, 0, 1), (n_*e_, 1, 0), (n_*w_, 1, 1)):
            xx = x0.astype(np.int64) + dx; yy = y0.astype(np.int64) + dy
            m = (xx >= 0) & (xx < W) & (yy >= 0) & (yy < H) & ~inv
            for c in range(C):
                prod = (G[b, c][m] * wt[m]).astype(f32).astype(np.float64)
                np.add.at(acc[b, v, c], (yy[m], xx[m]), prod)
nz = ref != 0
rel = np.abs(acc[nz] - ref[nz]) / np.abs(ref[nz])
print('max rel', rel.max(), 'count >1e-5', (rel > 1e-5).sum(), 'of', nz.sum())
i = np.argmax(np.where(nz, np.abs(acc - ref) / np.where(nz, np.abs(ref), 1), 0))
idx = np.unravel_index(i, ref.shape); print('worst', idx, 'ref', ref[idx], 'ours', acc[idx])
print('zero masks equal', np.array_equal(acc == 0, ref == 0))
