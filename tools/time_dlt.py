"""A/B latency of mvn_dlt across builds of libmvn_hip.so (BASELINE config 1: batch 1, 4 views x 17
joints; and a batch of 64), HIP events around 200 back-to-back calls, interleaved rounds; results
compared with the first build.
    python tools/time_dlt.py libA.so libB.so ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    res, args = _lib.SIGNATURES["mvn_dlt"]
    lib.mvn_dlt.restype, lib.mvn_dlt.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for B in (1, 64):
        ab = synth.algebraic_batch(B, 4, 17, seed=0)
        P, pts, conf = ab.proj.to(dev), ab.points.to(dev), ab.confidences.to(dev)
        outs, res = {}, {}
        for rnd in range(3):
            for name, lib in libs:
                out = outs.setdefault(name, torch.empty((B, 17, 3), device=dev))
                call = lambda: lib.mvn_dlt(P.data_ptr(), pts.data_ptr(), conf.data_ptr(), out.data_ptr(), B, 4, 17, st)  # noqa: E731
                for _ in range(10):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(200):
                    call()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(name, []).append(e0.elapsed_time(e1) / 200 * 1e3)
        first = libs[0][0]
        for name, v in res.items():
            d = ((outs[name] - outs[first]).abs().max() / outs[first].abs().max()).item()
            print(f"B={B:3d} {name:14s} {min(v):7.2f} us/call  max-rel vs {first}: {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
