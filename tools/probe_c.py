"""Unprojection time vs channel count (fixed cost vs per-channel-group cost), x4 kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402


def time_it(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = torch.device("cuda:0")
for B, dt in ((8, torch.float32), (32, torch.bfloat16)):
    for C in (4, 8, 16, 32, 64):
        vb = synth.volumetric_batch(B, channels=C, dtype=dt, device=dev, seed=0)
        for agg in ("softmax", "sum"):
            ms = min(time_it(lambda: op.unproject_heatmaps(vb.features, vb.proj, vb.coords, agg)) for _ in range(3))
            print(f"B={B:3d} {str(dt):15s} C={C:3d} {agg:8s} {ms * 1e3:8.1f} us", flush=True)
