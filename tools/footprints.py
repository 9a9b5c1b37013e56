"""Footprint statistics of the four-view unprojection's voxel tiles at the bench geometry
(CPU only, design aid): LDS slots per tile (sum over views of the odd-pitch box area), the
chunk count (4-pixel staging chunks) against the threads of a block, and the tiles that do
not fit one LDS pass ("slow" tiles, deferred to the unpipelined path).
    python tools/footprints.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import lds_conflicts  # noqa: E402


def tile_stats(fx, fy, ok, tile, threads, kbuf, mc=2):
    B, NV, V = fx.shape[0], fx.shape[1], fx.shape[2]
    TX, TY, TZ = tile
    lim = kbuf - 66
    slots, chunks, slow = [], [], 0
    for b in range(B):
        for x0 in range(0, V, TX):
            for y0 in range(0, V, TY):
                for z0 in range(0, V, TZ):
                    tot = totc = sn = cn = 0
                    npass, big = 1, False
                    for v in range(NV):
                        sl = (b, v, slice(x0, x0 + TX), slice(y0, y0 + TY), slice(z0, z0 + TZ))
                        m = ok[sl]
                        if not m.any():
                            continue
                        gx, gy = fx[sl][m], fy[sl][m]
                        bw, bh = gx.max() - gx.min() + 2, gy.max() - gy.min() + 2
                        area = (bw | 1) * bh
                        xa = gx.min() & ~3
                        nch = ((gx.min() + bw - xa + 3) >> 2) * bh
                        big |= area > lim or nch > mc * threads
                        if sn + area > lim or cn + nch > mc * threads:
                            npass, sn, cn = npass + 1, 0, 0
                        sn, cn, tot, totc = sn + area, cn + nch, tot + area, totc + nch
                    slots.append(tot)
                    chunks.append(totc)
                    slow += big or npass > 1
    return np.array(slots), np.array(chunks), slow


def main():
    fx, fy, ok = lds_conflicts.geometry(B=4)
    for tile, threads, kbuf in (((4, 8, 16), 512, 2000), ((4, 8, 8), 256, 1000)):
        s, c, slow = tile_stats(fx, fy, ok, tile, threads, kbuf)
        print(f"tile {tile} ({threads} threads, {kbuf} slots): slots mean {s.mean():.0f} p99 {np.percentile(s, 99):.0f} "
              f"max {s.max()}; chunks mean {c.mean():.0f} max {c.max()}, > threads {100 * (c > threads).mean():.1f} %; "
              f"slow tiles {100 * slow / len(s):.2f} %")


if __name__ == "__main__":
    main()
