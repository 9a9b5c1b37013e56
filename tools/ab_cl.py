"""A/B of the channels-last bf16 unprojection (config 5's producer: 64 frames, softmax,
NDHWC bf16 out) across builds of libmvn_hip.so, interleaved, outputs compared bitwise.
    python tools/ab_cl.py libA.so libB.so ..."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402


def main():
    libs = []
    for p in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.abspath(p))
        res, args = _lib.SIGNATURES["mvn_unproject_ex"]
        lib.mvn_unproject_ex.restype, lib.mvn_unproject_ex.argtypes = res, args
        libs.append((os.path.basename(p), lib))
    dev = torch.device("cuda:0")
    B = 64
    vb = synth.volumetric_batch(B, dtype=torch.bfloat16, device=dev, seed=0)
    out = torch.empty((B, 64, 64, 64, 32), dtype=torch.bfloat16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    ref, res = {}, {}
    for rnd in range(3):
        for name, lib in libs:
            def call():
                r = lib.mvn_unproject_ex(vb.features.data_ptr(), 1, vb.proj.data_ptr(), vb.coords.data_ptr(), None,
                                         out.data_ptr(), 1, 1, B, 4, 32, 96, 96, 64, 64, 64, 2, 0, st)
                assert r == 0, r
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                call()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                call()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(s.elapsed_time(e) / 10)
            if rnd == 0:
                ref[name] = out.clone()
    base = libs[0][0]
    for name, v in res.items():
        print(f"cfg5 cl bf16 B=64  {name:12s} {min(v) * 1e3:8.1f} us  same-as-{base}: "
              f"{torch.equal(ref[name].view(torch.int16), ref[base].view(torch.int16))}", flush=True)


if __name__ == "__main__":
    main()
