"""Config 5 (64 frames: channels-last bf16 unprojection -> V2V front block) run whole, or in
frame groups whose channels-last intermediate stays in the 256 MiB MALL between the two
launches (G frames x 16.8 MB).  Same outputs; wall time per 64 frames after settling.
    python tools/cfg5_groups.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import synth, v2v  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = 64
    vb = synth.volumetric_batch(B, n_views=4, channels=32, heatmap=96, volume=64, dtype=torch.bfloat16, device=dev, seed=0)
    g = torch.Generator().manual_seed(0)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=dev)
    out = torch.empty((B, 16, 64, 64, 64), dtype=torch.bfloat16, device=dev)

    def step(G):
        for i in range(0, B, G):
            cl = v2v.unproject_channels_last(vb.features[i:i + G], vb.proj[i:i + G], vb.coords[i:i + G], "softmax")
            out[i:i + G] = v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16)

    ref = None
    for rnd in range(2):
        for G in (64, 32, 16, 8, 4, 2):
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.5:
                step(G)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                step(G)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 10
            if ref is None:
                ref = out.clone()
            same = torch.equal(out, ref)
            print(f"round {rnd} groups of {G:2d} frames: {ms:7.3f} ms per 64 frames -> {B / ms * 1e3:8.0f} frames/s"
                  f"  intermediate {G * 16.8:6.0f} MB  same: {same}", flush=True)


if __name__ == "__main__":
    main()
