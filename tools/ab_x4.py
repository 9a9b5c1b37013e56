"""A/B of the four-view kernel (unproject_x4) against the generic tiled kernel, in one
process, interleaved rounds, via the C ABI's test knob; outputs compared bitwise.
    python tools/ab_x4.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, op, synth  # noqa: E402


def time_it(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    for B, N, dt, label in ((8, 4, torch.float32, "cfg2 f32 B=8"), (32, 4, torch.bfloat16, "cfg3 bf16 B=32"),
                            (16, 8, torch.float32, "cfg4 8v f32 B=16")):
        vb = synth.volumetric_batch(B, n_views=N, dtype=dt, device=dev, seed=0)
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (N * 32 * 96 * 96 + 32 * 64 ** 3) + 12 * 64 ** 3 + 4 * 12 * N)
        res, outs = {}, {}
        for rnd in range(3):
            for kern, generic in (("x4", False), ("tiled", True)):
                with _lib.unproject_knobs(generic=generic):
                    for agg in ("softmax", "sum", "max"):
                        fn = lambda: op.unproject_heatmaps(vb.features, vb.proj, vb.coords, agg)  # noqa: E731
                        res.setdefault((kern, agg), []).append(time_it(fn, iters))
                        if rnd == 0:
                            outs[(kern, agg)] = fn()
        for (kern, agg), v in sorted(res.items()):
            ms = min(v)
            same = torch.equal(outs[(kern, agg)].view(torch.int16 if E == 2 else torch.int32),
                               outs[("tiled", agg)].view(torch.int16 if E == 2 else torch.int32))
            print(f"{label:16s} {kern:6s} {agg:8s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:8.1f} GB/s "
                  f"({nbytes / ms / 1e6 / 8000:5.3f} of 8 TB/s)  bitwise == tiled: {same}", flush=True)


if __name__ == "__main__":
    main()
