"""Unprojection time against the channel count at the bench geometry (4 views, 96^2 maps ->
64^3, f32 B=8 and bf16 B=32; design aid): T(C) = a + b * C separates the per-block cost that
does not depend on the channels (coordinates, projection, footprints, regions, descriptors,
first group's latency) from the per-channel-group cost, at the kernel level (overlap included).
    python tools/scan_channels.py [lib.so]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "learnable-triangulation-pytorch_amd", "mvn_rocm",
                                                                "libmvn_hip.so")
    lib = ctypes.CDLL(os.path.abspath(path))
    res, args = _lib.SIGNATURES["mvn_unproject"]
    lib.mvn_unproject.restype, lib.mvn_unproject.argtypes = res, args
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for B, dt, label in ((8, torch.float32, "cfg2 geometry f32 B=8"), (32, torch.bfloat16, "cfg3 geometry bf16 B=32")):
        code = 1 if dt == torch.bfloat16 else 0
        rows = []
        for C in (4, 8, 16, 32, 64):
            vb = synth.volumetric_batch(B, n_views=4, channels=C, dtype=dt, device=dev, seed=0)
            out = torch.empty((B, C, 64, 64, 64), dtype=dt, device=dev)
            for agg in (2, 0):
                def call():
                    r = lib.mvn_unproject(vb.features.data_ptr(), code, vb.proj.data_ptr(), vb.coords.data_ptr(), None,
                                          out.data_ptr(), code, B, 4, C, 96, 96, 64, 64, 64, agg, 0, stream)
                    assert r == 0, r
                best = float("inf")
                for _ in range(3):
                    call()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(20):
                        call()
                    e.record()
                    torch.cuda.synchronize()
                    best = min(best, s.elapsed_time(e) / 20 * 1e3)
                rows.append((C, agg, best))
            del out, vb
        for agg, name in ((2, "softmax"), (0, "sum")):
            cs = np.array([c for c, a, _ in rows if a == agg], dtype=float)
            ts = np.array([t for _, a, t in rows if a == agg])
            b1, a0 = np.polyfit(cs, ts, 1)
            print(f"{label} {name:8s} " + "  ".join(f"C={int(c)}: {t:7.1f} us" for c, t in zip(cs, ts)) +
                  f"   fit T = {a0:.1f} + {b1:.2f} * C us (at C = 32 the fixed part is {100 * a0 / (a0 + 32 * b1):.0f} %)",
                  flush=True)


if __name__ == "__main__":
    main()
