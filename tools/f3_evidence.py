"""SURVEY §8f rank 3 (unproject -> V2V front, config 5): does the place the intermediate
volume is read from matter?  The front block's conv is timed on the same 8-frame group
(4 views x 32 ch x 96^2 -> 64^3, channels-last bf16, 134 MB) three ways:
  mall    — right after the group's unprojection wrote it (the intermediate fits the 256 MiB
            Infinity Cache: the one-call pipeline's situation);
  evicted — the same, with 1 GiB of unrelated copies between producer and consumer (the
            intermediate must come back from HBM: the two-launch whole-batch situation);
  batch   — one conv over the whole 64-frame batch written by one unprojection (1.07 GB).
Also the unprojection alone, and the one-call pipeline (mvn_unproject_v2v_front) over 64
frames against the two whole-batch launches.
    python tools/f3_evidence.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import synth, v2v  # noqa: E402

dev = torch.device("cuda:0")
B, G = 64, 8
vb = synth.volumetric_batch(B, dtype=torch.bfloat16, device=dev, seed=0)
g = torch.Generator().manual_seed(0)
w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                              torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                              device=dev)
src = torch.empty(1 << 28, device=dev)          # 1 GiB eviction stream
dst = torch.empty_like(src)


def ev():
    return torch.cuda.Event(enable_timing=True)


def settle(seconds=1.0):
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        v2v.v2v_front(v2v.unproject_channels_last(vb.features[:G], vb.proj[:G], vb.coords[:G]), packed, scale, shift,
                      torch.bfloat16)
    torch.cuda.synchronize()


def group_conv_ms(evict, rounds=5):
    """mean conv time per 8-frame group, the group's intermediate just written"""
    ts = []
    for _ in range(rounds):
        for s in range(0, B, G):
            cl = v2v.unproject_channels_last(vb.features[s:s + G], vb.proj[s:s + G], vb.coords[s:s + G])
            if evict:
                dst.copy_(src)
            a, b = ev(), ev()
            a.record()
            v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16)
            b.record()
            ts.append((a, b))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ts) / len(ts)


def timed(fn, it=5):
    fn()
    torch.cuda.synchronize()
    a, b = ev(), ev()
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


settle()
mall = group_conv_ms(False)
evicted = group_conv_ms(True)
mall2 = group_conv_ms(False)
cl_all = v2v.unproject_channels_last(vb.features, vb.proj, vb.coords)
batch = timed(lambda: v2v.v2v_front(cl_all, packed, scale, shift, torch.bfloat16))
unp = timed(lambda: v2v.unproject_channels_last(vb.features, vb.proj, vb.coords))
two = timed(lambda: v2v.v2v_front(v2v.unproject_channels_last(vb.features, vb.proj, vb.coords), packed, scale, shift,
                                  torch.bfloat16))
one = timed(lambda: v2v.unproject_v2v_front(vb.features, vb.proj, vb.coords, packed, scale, shift, "softmax",
                                            torch.bfloat16))
print(f"conv per 8-frame group: intermediate in MALL {mall:.3f} / {mall2:.3f} ms, evicted to HBM {evicted:.3f} ms "
      f"({(evicted / ((mall + mall2) / 2) - 1) * 100:+.1f} %)")
print(f"conv over 64 frames from a 1.07 GB HBM intermediate: {batch:.3f} ms = {batch / (B // G):.3f} ms per 8 frames")
print(f"unprojection (channels-last bf16) 64 frames: {unp:.3f} ms; conv share of the two-launch step "
      f"{batch / (batch + unp) * 100:.1f} %")
print(f"64 frames: two whole-batch launches {two:.3f} ms ({B / two * 1e3:.0f} frames/s), one-call pipeline "
      f"{one:.3f} ms ({B / one * 1e3:.0f} frames/s)")
