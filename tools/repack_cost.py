"""What a channels-last repack of the feature maps would cost (VERDICT r5 item 2's bound):
NCHW -> (B, N, C/G, H, W, G) for the 8-view f32 config (G = 2, the 8-view kernel's slot) and
the 4-view bf16 config (G = 4), as torch's permute-copy on the device (a streaming
transpose: read + write of the maps), timed with HIP events.
    python tools/repack_cost.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for label, B, N, dt, G in (("cfg4 f32 8 views, 16 frames", 16, 8, torch.float32, 2),
                               ("cfg3 bf16 4 views, 32 frames", 32, 4, torch.bfloat16, 4)):
        f = torch.randn((B, N, 32, 96, 96), device=dev).to(dt)
        out = torch.empty((B, N, 32 // G, 96, 96, G), device=dev, dtype=dt)
        src = f.view(B, N, 32 // G, G, 96, 96).permute(0, 1, 2, 4, 5, 3)
        for _ in range(20):
            out.copy_(src)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            out.copy_(src)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        nb = 2 * f.numel() * f.element_size()
        print(f"{label}: repack {us:.1f} us ({nb / us / 1e3:.0f} GB/s of read + write)", flush=True)


if __name__ == "__main__":
    main()
