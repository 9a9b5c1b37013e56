"""Fixed vs per-channel-group cost of the fast bf16 unprojection: config-3
geometry (4 views, 96^2 maps, 64^3, 32 frames) at C = 4, 8, 16, 32 channels, softmax and sum;
a linear fit t(C) = fixed + per_group * C/4 splits the kernel into its per-voxel prologue
(projection, footprints, staging setup) and its channel loop.

    python tools/fast_channel_sweep.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for agg in ("softmax", "sum"):
        rows = []
        for C in (4, 8, 16, 32):
            vb = synth.volumetric_batch(32, channels=C, dtype=torch.bfloat16, device=dev, seed=0)
            f = lambda: op.unproject_heatmaps(vb.features, vb.proj, vb.coords, agg, precision="fast")  # noqa: E731
            f()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    f()
                e.record()
                torch.cuda.synchronize()
                best = min(best, s.elapsed_time(e) / 20 * 1e3)
            rows.append((C, best))
            print(f"{agg:8s} C={C:3d}  {best:8.1f} us", flush=True)
        c = np.array([r[0] / 4 for r in rows]); t = np.array([r[1] for r in rows])
        k, f0 = np.polyfit(c, t, 1)
        print(f"{agg:8s} fit: fixed {f0:.1f} us + {k:.1f} us per 4-channel group "
              f"(C=32: fixed share {f0 / (f0 + 8 * k):.2f})", flush=True)


if __name__ == "__main__":
    main()
