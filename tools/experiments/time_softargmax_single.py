# ARCHIVED with tools/experiments/softargmax_single.hip (not kept, profiles/r17_ab_softargmax_single.txt);
# needs that kernel built in place of csrc/softargmax.hip plus its debug hook in the C ABI.
"""Time the 3D soft-argmax paths in one process: the single-pass kernel (default dispatch) vs the
three launches (mvn_debug_set_softargmax(1)), on the bench's operand — channels [0:17] of a
(B, 32, 64^3) unprojected volume (strided), output in the input dtype.  HIP events, best of 3
rounds of 20 calls.  Algorithmic bytes: volume read + normalised volume written +
coordinates read.
    python tools/time_softargmax.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, op, synth  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for B, dt, label in ((8, torch.float32, "cfg2 f32 B=8"), (32, torch.bfloat16, "cfg3 bf16 B=32")):
        vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
        vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")[:, :17]
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (2 * 17 * 64 ** 3 * E + 12 * 64 ** 3)
        res, outs = {}, {}
        for rnd in range(3):
            for name, mode in (("single", 0), ("three", 1), ("nosync", 2), ("nowait", 3)):
                kn = _lib.softargmax_knobs()
                kn.mode = mode
                with kn:
                    call = lambda: op.integrate_tensor_3d_with_coordinates(vol, vb.coords)
                    call()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(20):
                        r = call()
                    e.record()
                    torch.cuda.synchronize()
                res.setdefault(name, []).append(s.elapsed_time(e) / 20)
                outs[name] = r
        for name, v in res.items():
            ms = min(v)
            dx = (outs[name][0] - outs["three"][0]).abs().max().item()
            print(f"{label:15s} {name:7s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.0f} GB/s alg  "
                  f"xyz max|d| vs three: {dx:.3g}", flush=True)


if __name__ == "__main__":
    main()
