"""Offline model of the unprojection's LDS tap-read bank conflicts (design aid, CPU only).

For the bench geometry (synth.volumetric_batch), every 64-voxel wave of every tile and every
view: the LDS slot of each of the 4 bilinear taps under a given region layout, then the
cycles of one ds_read_b128 (gfx950: 4 lane groups of 16, one cycle per distinct slot per
16-byte bank quad, identical slots broadcast; MI355X_MICROARCH.md §LDS).
    python tools/lds_conflicts.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
from mvn_rocm import synth  # noqa: E402

GROUPS128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
             [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
GROUPS128 += [[l + 32 for l in g] for g in GROUPS128]


def geometry(B=2, H=96, W=96):
    vb = synth.volumetric_batch(B, seed=0)
    P = vb.proj.numpy().astype(np.float64)
    X = vb.coords.numpy().astype(np.float64)
    X = np.concatenate([X, np.ones(X.shape[:4] + (1,))], -1)
    uvw = np.einsum("bvrk,bxyzk->bvxyzr", P, X)
    w = np.where(uvw[..., 2] == 0, 1.0, uvw[..., 2])
    ix = (2 * (uvw[..., 0] / w / H - 0.5) + 1) * W / 2 - 0.5
    iy = (2 * (uvw[..., 1] / w / W - 0.5) + 1) * H / 2 - 0.5
    fx, fy = np.floor(ix).astype(np.int64), np.floor(iy).astype(np.int64)
    ok = (fx >= -1) & (fx < W) & (fy >= -1) & (fy < H) & (uvw[..., 2] > 0)
    return fx, fy, ok


def cycles_b128(slots):
    """slots: (64,) LDS slot (16-byte units) per lane -> cycles of one ds_read_b128."""
    tot = 0
    for g in GROUPS128:
        s = np.unique(slots[g])
        q = s % 16
        tot += np.bincount(q, minlength=16).max()
    return tot


def simulate(tile=(4, 8, 16), lane_of=None, layout="odd", swz=False, nwaves=4000, seed=0):
    fx, fy, ok = geometry()
    TX, TY, TZ = tile
    B, NV, Vx, Vy, Vz = fx.shape
    rng = np.random.default_rng(seed)
    tot, ideal, n = 0, 0, 0
    tiles = [(b, x, y, z) for b in range(B) for x in range(0, Vx, TX) for y in range(0, Vy, TY) for z in range(0, Vz, TZ)]
    for (b, x0, y0, z0) in [tiles[i] for i in rng.choice(len(tiles), min(len(tiles), nwaves // 8), replace=False)]:
        # voxel of thread t in the tile (kernel order: z fastest, then y, then x)
        t = np.arange(TX * TY * TZ)
        X, Y, Z = x0 + t // (TZ * TY), y0 + (t // TZ) % TY, z0 + t % TZ
        base = 0
        for v in range(NV):
            m = ok[b, v, X, Y, Z]
            if not m.any():
                continue
            gx, gy = fx[b, v, X, Y, Z], fy[b, v, X, Y, Z]
            bx0, by0 = gx[m].min(), gy[m].min()
            bw = gx[m].max() - bx0 + 2
            bh = gy[m].max() - by0 + 2
            pitch = {"odd": bw | 1, "raw": bw, "m4": bw + (4 - bw % 16) % 16 if False else bw + ((4 - bw) % 16)}[layout]
            for wv in range(len(t) // 64):
                sel = slice(wv * 64, wv * 64 + 64)
                r, c = gy[sel] - by0, gx[sel] - bx0
                for dr, dc in ((0, 0), (0, 1), (1, 0), (1, 1)):
                    rr, cc = r + dr, c + dc
                    slot = base + rr * pitch + cc
                    if swz:
                        slot = slot ^ ((rr & 3) << 2)
                    slot = np.where(m[sel], slot, 10 ** 6)
                    tot += cycles_b128(slot)
                    ideal += 4
                    n += 1
            base += pitch * bh
    return tot / n, ideal / n


if __name__ == "__main__":
    for layout in ("odd", "raw"):
        for swz in (False, True):
            c, i = simulate(layout=layout, swz=swz, nwaves=1600)
            print(f"layout={layout:4s} swizzle={swz!s:5s}  cycles/ds_read_b128 {c:.2f} (ideal {i:.0f})")
