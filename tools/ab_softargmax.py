"""A/B timing of mvn_softargmax3d across builds of libmvn_hip.so, on the bench's input: channels
[0:17] of a (B, 32, 64^3) unprojected volume (strided slice), volume output in the input dtype.
    python tools/ab_softargmax.py libA.so libB.so ..."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, op, synth  # noqa: E402


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    for n in ("mvn_softargmax3d", "mvn_softargmax3d_workspace_bytes"):
        res, args = _lib.SIGNATURES[n]
        getattr(lib, n).restype, getattr(lib, n).argtypes = res, args
    return lib


def main():
    libs = [(os.path.basename(p), load(p)) for p in sys.argv[1:]]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for B, dt, label in ((8, torch.float32, "cfg2 f32 B=8"), (32, torch.bfloat16, "cfg3 bf16 B=32")):
        vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
        vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
        V3 = 64 ** 3
        code = 1 if dt == torch.bfloat16 else 0
        E = 2 if code else 4
        nbytes = B * (2 * 17 * V3 * E + 12 * V3)
        res, outs = {}, {}
        for rnd in range(3):
            for name, lib in libs:
                ws = torch.empty(lib.mvn_softargmax3d_workspace_bytes(B, 17, 64, 64, 64), dtype=torch.uint8, device=dev)
                xyz = torch.empty((B, 17, 3), device=dev)
                out = torch.empty((B, 17, 64, 64, 64), dtype=dt, device=dev)

                def call():
                    r = lib.mvn_softargmax3d(vol.data_ptr(), code, 32 * V3, V3, vb.coords.data_ptr(), 1.0, 1,
                                             xyz.data_ptr(), out.data_ptr(), code, ws.data_ptr(), ws.numel(),
                                             B, 17, 64, 64, 64, stream)
                    assert r == 0, r
                call()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    call()
                e.record()
                torch.cuda.synchronize()
                res.setdefault(name, []).append(s.elapsed_time(e) / 20)
                outs[name] = (xyz.clone(), out.clone())
        first = libs[0][0]
        for name, v in res.items():
            ms = min(v)
            dx = (outs[name][0] - outs[first][0]).abs().max().item()
            same = torch.equal(outs[name][1], outs[first][1])
            print(f"{label:15s} {name:16s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.0f} GB/s alg  "
                  f"xyz max|d| vs {first}: {dx:.3g}  volume bitwise: {same}", flush=True)


if __name__ == "__main__":
    main()
