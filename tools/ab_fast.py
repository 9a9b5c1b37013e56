"""A/B of builds of libmvn_hip.so in the fast arithmetic (mvn_unproject_precision, DESIGN.md
§4.1a) at config 3 (bf16, 32 frames) and config 2, interleaved rounds in one process; outputs
compared bitwise against the first build.

    python tools/ab_fast.py path/to/libA.so path/to/libB.so ...
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    res, args = _lib.SIGNATURES["mvn_unproject_precision"]
    lib.mvn_unproject_precision.restype, lib.mvn_unproject_precision.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for B, dt, label in ((32, torch.bfloat16, "cfg3 bf16 B=32"), (8, torch.float32, "cfg2 f32 B=8")):
        vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (4 * 32 * 96 * 96 + 32 * 64 ** 3) + 12 * 64 ** 3 + 4 * 12 * 4)
        code = 1 if dt == torch.bfloat16 else 0
        outs, res = {}, {}

        def call(lib, out, agg):
            r = lib.mvn_unproject_precision(vb.features.data_ptr(), code, vb.proj.data_ptr(), vb.coords.data_ptr(),
                                            None, 0, None, out.data_ptr(), code, 0, B, 4, 32, 96, 96, 64, 64, 64,
                                            agg, 0, 1, stream)
            assert r == 0, r

        for _ in range(3):
            for name, lib in libs:
                for agg, an in ((2, "softmax"), (0, "sum")):
                    out = outs.setdefault((name, an), torch.empty((B, 32, 64, 64, 64), dtype=dt, device=dev))
                    call(lib, out, agg)
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(20):
                        call(lib, out, agg)
                    e.record()
                    torch.cuda.synchronize()
                    res.setdefault((name, an), []).append(s.elapsed_time(e) / 20)
        first = libs[0][0]
        for (name, an), v in res.items():
            ms = min(v)
            same = torch.equal(outs[(name, an)].view(torch.int16 if E == 2 else torch.int32),
                               outs[(first, an)].view(torch.int16 if E == 2 else torch.int32))
            print(f"{label:15s} {name:22s} {an:8s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e9:.3f} of 8 TB/s  "
                  f"same-as-{first}: {same}", flush=True)


if __name__ == "__main__":
    main()
