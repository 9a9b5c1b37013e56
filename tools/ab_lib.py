"""A/B timing of mvn_unproject across several builds of libmvn_hip.so (kernel variants),
in one process, interleaved rounds; outputs are checked bitwise against the first build.

    python tools/ab_lib.py path/to/libA.so path/to/libB.so ...
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
    res, args = _lib.SIGNATURES["mvn_unproject"]
    lib.mvn_unproject.restype, lib.mvn_unproject.argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    for name, lib in libs:
        if hasattr(lib, "mvn_debug_unproject_occupancy"):
            print(f"{name}: x4 blocks per CU f32 {lib.mvn_debug_unproject_occupancy(0)} "
                  f"bf16 {lib.mvn_debug_unproject_occupancy(1)}", flush=True)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    cases = [(8, 4, torch.float32, "cfg2 f32 B=8"), (32, 4, torch.bfloat16, "cfg3 bf16 B=32")]
    if os.environ.get("AB_CFG4"):
        cases.append((16, 8, torch.float32, "cfg4 f32 N=8 B=16"))
    if os.environ.get("AB_ONLY"):        # e.g. AB_ONLY=cfg4
        cases = [c for c in cases if c[3].startswith(os.environ["AB_ONLY"])]
    for B, NV, dt, label in cases:
        vb = synth.volumetric_batch(B, n_views=NV, dtype=dt, device=dev, seed=0)
        feat, proj, coords = vb.features, vb.proj, vb.coords
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (NV * 32 * 96 * 96 + 32 * 64 ** 3) + 12 * 64 ** 3 + 4 * 12 * NV)
        code = 1 if dt == torch.bfloat16 else 0
        outs = {}
        res = {}

        def call(lib, out, agg):
            r = lib.mvn_unproject(feat.data_ptr(), code, proj.data_ptr(), coords.data_ptr(), None, out.data_ptr(),
                                  code, B, NV, 32, 96, 96, 64, 64, 64, agg, 0, stream)
            assert r == 0, r

        for rnd in range(3):
            for name, lib in libs:
                for agg, aname in ((2, "softmax"), (0, "sum")):
                    out = outs.setdefault((name, aname), torch.empty((B, 32, 64, 64, 64), dtype=dt, device=dev))
                    call(lib, out, agg)
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(20):
                        call(lib, out, agg)
                    e.record()
                    torch.cuda.synchronize()
                    res.setdefault((name, aname), []).append(s.elapsed_time(e) / 20)
        first = libs[0][0]
        for (name, aname), v in res.items():
            ms = min(v)
            same = torch.equal(outs[(name, aname)], outs[(first, aname)])
            print(f"{label:15s} {name:24s} {aname:8s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.0f} GB/s "
                  f"({nbytes / ms / 1e6 / 80:5.1f}% of 8 TB/s)  same-as-{first}: {same}", flush=True)


if __name__ == "__main__":
    main()
