"""A/B of mvn_softargmax2d across builds of libmvn_hip.so: config 1's 4 views x 17 joints of 96^2
heatmaps (x100 multiplier, softmax) and a 64-frame batch; HIP events around 200 calls, best of 3;
outputs compared with the first build.
    python tools/time_softargmax2d.py libA.so libB.so ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    res, args = _lib.SIGNATURES["mvn_softargmax2d"]
    lib.mvn_softargmax2d.restype, lib.mvn_softargmax2d.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    for B, sm in ((4, 1), (4, 0), (256, 1)):
        hm = torch.randn((B, 17, 96, 96), generator=torch.Generator().manual_seed(1)).to(dev)
        outs, res = {}, {}
        for rnd in range(3):
            for name, lib in libs:
                xy = torch.empty((B, 17, 2), device=dev)
                maps = torch.empty_like(hm)
                call = lambda: lib.mvn_softargmax2d(hm.data_ptr(), 0, 100.0, sm, xy.data_ptr(), maps.data_ptr(), 0,  # noqa: E731
                                                    B, 17, 96, 96, st)
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
                outs[name] = (xy.clone(), maps.clone())
        first = libs[0][0]
        for name, v in res.items():
            dxy = ((outs[name][0] - outs[first][0]).abs().max() / outs[first][0].abs().max()).item()
            dm = ((outs[name][1] - outs[first][1]).abs().max() / outs[first][1].abs().max()).item()
            print(f"maps {B}x17 softmax={sm} {name:14s} {min(v):7.2f} us/call  max-rel vs {first}: xy {dxy:.3g} maps {dm:.3g}",
                  flush=True)


if __name__ == "__main__":
    main()
