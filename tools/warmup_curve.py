"""Per-step unprojection time (HIP events) over the first steps of a fresh process, for the
bench's op-layer step: how long until the kernel reaches its steady time, and whether
pre-touching the buffers or an idle GPU warm-up changes that.
    python tools/warmup_curve.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from mvn_rocm import op  # noqa: E402


def curve(wl, n):
    evs = []
    t0 = time.perf_counter()
    for _ in range(n):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        v = op.unproject_heatmaps(wl.feat, wl.proj, wl.coords, "softmax")
        e[1].record()
        op.integrate_tensor_3d_with_coordinates(v[:, :17], wl.coords, True)
        evs.append(e)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return [a.elapsed_time(b) * 1e3 for a, b in evs], wall


def main():
    dev = torch.device("cuda:0")
    wl = bench.Workload(bench._configs()["2"], 0, 1, dev)
    torch.cuda.synchronize()
    ts, wall = curve(wl, 200)
    print("steps 0..199 (10-step means):", " ".join(f"{sum(ts[i:i + 10]) / 10:.0f}" for i in range(0, 200, 10)),
          f" wall {wall * 1e3:.1f} ms", flush=True)
    time.sleep(2.0)
    ts, wall = curve(wl, 100)
    print("after 2 s idle, steps 0..99:", " ".join(f"{sum(ts[i:i + 10]) / 10:.0f}" for i in range(0, 100, 10)), flush=True)


if __name__ == "__main__":
    main()
