"""Per-view row-pitch rules for the four-view kernel's LDS bank conflicts, against the best pitch per
view (search over 16 residues): the model behind DESIGN.md 4.1 (r14).  CPU only, uses the
geometry and ds_read_b128 cycle model of tools/lds_conflicts.py.  python tools/lds_pitch_rules.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lds_conflicts as L  # noqa: E402


def patch_vt(TZ=16):
    """unproject_x4's lane -> voxel-in-wave mapping (MVN_X4_PATCH_LANES: 2 x 8 patches)."""
    out = []
    for lane in range(64):
        m = lane & 31
        g1 = (4 <= m < 12) or (16 <= m < 20) or m >= 28
        i = (m - 4 if m < 12 else m - 8 if m < 20 else m - 16) if g1 else (m if m < 4 else m - 8 if m < 16 else m - 12)
        g = 2 * (lane >> 5) + (1 if g1 else 0)
        ZH = TZ // 8
        yw = 2 * (g // ZH) + (i >> 3)
        z = 8 * (g % ZH) + (i & 7)
        out.append(yw * TZ + z)
    return np.array(out)


fx, fy, ok = L.geometry()
TX, TY, TZ = 4, 8, 16
B, NV, Vx, Vy, Vz = fx.shape
rng = np.random.default_rng(1)
tiles = [(b, x, y, z) for b in range(B) for x in range(0, Vx, TX) for y in range(0, Vy, TY) for z in range(0, Vz, TZ)]
pv = patch_vt(TZ)
rules = {}
def add(name, c, n):
    a = rules.setdefault(name, [0, 0]); a[0] += c; a[1] += n
for (b, x0, y0, z0) in [tiles[i] for i in rng.choice(len(tiles), 100, replace=False)]:
    t = np.arange(TX * TY * TZ)
    X, Y, Z = x0 + t // (TZ * TY), y0 + (t // TZ) % TY, z0 + t % TZ
    for v in range(NV):
        m = ok[b, v, X, Y, Z]
        if not m.any(): continue
        gx, gy = fx[b, v, X, Y, Z], fy[b, v, X, Y, Z]
        bx0, by0 = gx[m].min(), gy[m].min()
        bw = gx[m].max() - bx0 + 2
        # projected steps of the tile: z (8 voxels) and y (1 voxel) from the tile's corner voxels
        fxz = fx[b, v, x0, y0, min(z0 + 15, Vz - 1)] - fx[b, v, x0, y0, z0]; fyz = fy[b, v, x0, y0, min(z0 + 15, Vz - 1)] - fy[b, v, x0, y0, z0]
        def cost(pitch):
            c = 0; n = 0
            for wv in range(len(t) // 64):
                idx = wv * 64 + pv
                r, cc = gy[idx] - by0, gx[idx] - bx0
                for dr, dc in ((0, 0), (0, 1), (1, 0), (1, 1)):
                    slot = (r + dr) * pitch + cc + dc
                    slot = np.where(m[idx], slot, 10 ** 6)
                    c += L.cycles_b128(slot); n += 1
            return c, n
        c, n = cost(bw | 1); add("odd", c, n)
        costs = [cost(p)[0] for p in range(bw, bw + 16)]
        add("best", min(costs), n)
        # rule: pitch so that a 1-row step lands 8 slots (half a bank sweep) away from the z-line direction
        for k in range(16):
            p = bw + ((k - bw) % 16)
            add(f"mod{k}", cost(p)[0], n)
        # direction rule: if z projects mostly vertically (|fyz| > |fxz|), choose pitch = 8 mod 16 + 1 else odd
        p = bw + ((9 - bw) % 16) if abs(fyz) > abs(fxz) else bw | 1
        add("dir", cost(p)[0], n)
        sgn = 1 if fxz * fyz >= 0 else -1
        p = bw + (((2 if sgn > 0 else 14) - bw) % 16)
        add("diag", cost(p)[0], n)
for k, (c, n) in sorted(rules.items(), key=lambda kv: kv[1][0] / kv[1][1]): print(f"{k:6s} {c / n:.3f}")
