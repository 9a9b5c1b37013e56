"""Time the config-5 pipeline pieces: unproject (softmax, channels-last bf16) and the V2V
front block (mvn_v2v_front), B frames of 4 views x 32 ch x 96^2 -> 64^3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import synth, v2v  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
vb = synth.volumetric_batch(B, dtype=torch.bfloat16, device=dev, seed=0)
g = torch.Generator().manual_seed(0)
w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
packed, scale, shift = v2v.fold_basic3d_block(w, torch.zeros(16), torch.ones(16), torch.zeros(16), torch.zeros(16),
                                              torch.ones(16), device=dev)


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


cl = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords)
t_u = timed(lambda: v2v.unproject_channels_last(vb.features, vb.proj, vb.coords))
t_c = timed(lambda: v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16))
flop = 2 * 32 * 16 * 343 * 64 ** 3 * B
print(f"B={B}: unproject(cl, bf16) {t_u:.3f} ms, v2v_front {t_c:.3f} ms = {flop / t_c / 1e9:.1f} TFLOP/s "
      f"({flop / t_c / 1e9 / 2500 * 100:.1f}% of 2.5 PF bf16 dense); pipeline {B / (t_u + t_c) * 1e3:.0f} frames/s")
