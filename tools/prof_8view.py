"""Workload for rocprofv3: the 8-view unprojection (config 4, 16 frames, f32, softmax)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402

dev = torch.device("cuda:0")
vb = synth.volumetric_batch(16, n_views=8, device=dev, seed=0)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
torch.cuda.synchronize()
print("done")
