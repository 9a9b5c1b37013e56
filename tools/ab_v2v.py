"""A/B timing of mvn_v2v_front across several builds (kernel variants) in one process,
interleaved rounds, at config 5's shape (B frames of a 64^3 x 32 bf16 volume).

    python tools/ab_v2v.py [--batch B] libA.so libB.so ...   (build: tools/build_variant.sh name v2v_front -D...)
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib  # noqa: E402
from mvn_rocm.v2v import fold_basic3d_block  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    res, args = _lib.SIGNATURES["mvn_v2v_front"]
    lib.mvn_v2v_front.restype, lib.mvn_v2v_front.argtypes = res, args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    libs = [(os.path.basename(p), load(p)) for p in a.libs]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    B, V = a.batch, 64
    g = torch.Generator().manual_seed(0)
    w = torch.randn(16, 32, 7, 7, 7, generator=g) * 0.02
    packed, scale, shift = fold_basic3d_block(w, torch.randn(16, generator=g), torch.rand(16, generator=g) + 0.5,
                                              torch.randn(16, generator=g), torch.randn(16, generator=g),
                                              torch.rand(16, generator=g) + 0.5, device=dev)
    x = torch.randn(B, V, V, V, 32, generator=g).to(torch.bfloat16).to(dev)
    outs, times = {}, {n: [] for n, _ in libs}
    for name, lib in libs:
        o = torch.empty(B, 16, V, V, V, device=dev)
        assert lib.mvn_v2v_front(x.data_ptr(), packed.data_ptr(), scale.data_ptr(), shift.data_ptr(), o.data_ptr(),
                                 0, B, V, stream) == 0
        outs[name] = o
    flop = 2.0 * B * V ** 3 * 16 * 32 * 343
    for _ in range(a.rounds):
        for name, lib in libs:
            o = outs[name]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.mvn_v2v_front(x.data_ptr(), packed.data_ptr(), scale.data_ptr(), shift.data_ptr(), o.data_ptr(),
                                  0, B, V, stream)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 5)
    ref = outs[libs[0][0]]
    for name, _ in libs:
        t = min(times[name])
        d = (outs[name] - ref).abs().max().item()
        print(f"{name:28s} {t:7.3f} ms  {flop / t / 1e9:7.1f} TFLOP/s  max|diff| vs first {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
