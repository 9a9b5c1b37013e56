"""Measured arithmetic floor of the 4-view unprojection (tools/micro/unproject_floor.hip)
next to the production kernel, at config 2 (f32, B=8) and config 3 (B=32) shapes.

    python tools/micro/unproject_floor.py        (GPU box; build with build_floor.sh first)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402

MODES = {0: "proj+taps+softmax", 1: "proj+taps+sum", 2: "projection only", 3: "taps+softmax (no proj)",
         4: "FAST proj+dot2+softmax", 5: "FAST proj+dot2+sum", 6: "FAST projection only"}


def timed(fn, iters=20, rounds=3):
    best = 1e30
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best * 1e3


def main():
    fl = ctypes.CDLL(os.path.join(ROOT, "tools", "bin", "unproject_floor.so"))
    fl.floor_run.restype = ctypes.c_int
    fl.floor_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [ctypes.c_void_p]
    lib = _lib.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    seed = torch.randn(256 * 4, device=dev)
    for B, dt, label in ((8, torch.float32, "cfg2 f32 B=8"), (32, torch.bfloat16, "cfg3 bf16 B=32")):
        vb = synth.volumetric_batch(B, n_views=4, dtype=dt, device=dev, seed=0)
        nvox = 64 ** 3
        out = torch.empty(B * nvox, device=dev)
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (4 * 32 * 96 * 96 + 32 * nvox) + 12 * nvox + 48 * 4)
        for mode, name in MODES.items():
            def f(mode=mode):
                r = fl.floor_run(mode, vb.proj.data_ptr(), vb.coords.data_ptr(), seed.data_ptr(), out.data_ptr(),
                                 B, nvox, 96, 96, 32, stream)
                assert r == 0, r
            us = timed(f)
            print(f"{label:15s} floor {name:24s} {us:8.1f} us  (HBM floor {nbytes / 8e6:6.1f} us; "
                  f"a kernel at this time would be {nbytes / us / 8e6:5.3f} of 8 TB/s)", flush=True)
        code = 1 if dt == torch.bfloat16 else 0
        vol = torch.empty((B, 32, 64, 64, 64), dtype=dt, device=dev)
        for agg, an in ((2, "softmax"), (0, "sum")):
            for prec, pn in ((0, "exact"), (1, "FAST")):
                def g(agg=agg, prec=prec):
                    r = lib.mvn_unproject_precision(vb.features.data_ptr(), code, vb.proj.data_ptr(),
                                                    vb.coords.data_ptr(), None, 0, None, vol.data_ptr(), code, 0, B, 4,
                                                    32, 96, 96, 64, 64, 64, agg, 0, prec, stream)
                    assert r == 0, r
                us = timed(g)
                print(f"{label:15s} production unproject_x4 {pn:5s} {an:8s} {us:8.1f} us  "
                      f"({nbytes / us / 8e6:5.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
