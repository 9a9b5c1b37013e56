"""Error of the fast bf16 softmax unprojection (f32 out) against the C oracle on the same bf16
bits, over seeds and volume shapes (cubic vs ragged), with the sample-magnitude statistics the
error analysis in DESIGN.md §4.1a uses.
    python tools/fast_bf16_error_probe.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402
from oracle import capi  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for shape in ((24, 24, 24), (13, 21, 10)):
        for seed in range(41, 47):
            for method in ("sum", "softmax"):
                vb = synth.volumetric_batch(2, channels=8, heatmap=64, volume=24, seed=seed, dtype=torch.bfloat16)
                c = vb.coords[:, :shape[0], :shape[1], :shape[2]].contiguous()
                bits = vb.features.view(torch.int16).numpy().view(np.uint16)
                ref = capi.unproject(bits, vb.proj.numpy(), c.numpy(), method, feat_bf16_bits=True)
                out = op.unproject_heatmaps(vb.features.to(dev), vb.proj.to(dev), c.to(dev), method,
                                            out_dtype=torch.float32, precision="fast").cpu().numpy()
                d = np.abs(out.astype(np.float64) - ref)
                print(f"{str(shape):14s} seed {seed} {method:8s} max|d|/max|ref| {d.max() / np.abs(ref).max():.5f}  "
                      f"max|ref| {np.abs(ref).max():.3f}  max|feat| {vb.features.float().abs().max():.2f}", flush=True)


if __name__ == "__main__":
    main()
