"""Workload for rocprofv3: a few launches of each hot-path kernel at the bench configs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
precision = sys.argv[3] if len(sys.argv) > 3 else "exact"     # the unprojection's arithmetic
dev = torch.device("cuda:0")
B, dt, nv = {"2": (8, torch.float32, 4), "3": (32, torch.bfloat16, 4), "4": (16, torch.float32, 8)}[cfg]
vb = synth.volumetric_batch(B, n_views=nv, dtype=dt, device=dev, seed=0)
for _ in range(iters):
    vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax", precision=precision)
    op.integrate_tensor_3d_with_coordinates(vol[:, :17], vb.coords)
torch.cuda.synchronize()
print("done", cfg, iters, precision)
