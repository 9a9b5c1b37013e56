"""Time the unprojection backward at config 2's shape (8 frames, 4 views x 32 ch x 96^2 ->
64^3, f32): float-atomic accumulation against the default per-call-scaled fixed point, and
check that two fixed-point runs are bit-identical.
    python tools/time_backward.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _backward, synth  # noqa: E402

dev = torch.device("cuda:0")
vb = synth.volumetric_batch(8, device=dev, seed=0)
g = torch.randn(8, 32, 64, 64, 64, device=dev)


def run(agg):
    return _backward.unproject_bwd(vb.features, vb.proj, vb.coords, None, g, agg, False, False)[0]


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


for name, agg in (("sum", 0), ("softmax", 2)):
    _backward.UNPROJECT_BACKWARD = "float_atomic"
    t_atomic = timed(lambda: run(agg))
    _backward.UNPROJECT_BACKWARD = "fixed"
    t_det = timed(lambda: run(agg))
    x, y = run(agg), run(agg)
    print(f"{name:8s} backward, 8 frames: float atomics {t_atomic:.3f} ms, fixed point {t_det:.3f} ms "
          f"({t_det / t_atomic:.2f}x); two fixed-point runs bit-identical: {torch.equal(x, y)}", flush=True)
