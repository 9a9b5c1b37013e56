"""A/B of the unprojection's two arithmetics (precision='exact' / 'fast') at
the bench configs, interleaved rounds in one process: kernel time (HIP events, best of
rounds), algorithmic GB/s, and the fast volume's deviation from the exact one.

    python tools/ab_precision.py [iters] [cfg ...]      cfg in 2 3 4 (default all)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402


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


CFGS = {"2": (8, 4, torch.float32), "3": (32, 4, torch.bfloat16), "4": (16, 8, torch.float32)}


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    which = sys.argv[2:] or ["2", "3", "4"]
    dev = torch.device("cuda:0")
    for cfg in which:
        B, N, dt = CFGS[cfg]
        vb = synth.volumetric_batch(B, n_views=N, dtype=dt, device=dev, seed=0)
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (N * 32 * 96 * 96 + 32 * 64 ** 3) + 12 * 64 ** 3 + 4 * 12 * N)
        res, outs = {}, {}
        for _ in range(3):
            for prec in ("exact", "fast"):
                for agg in ("softmax", "sum"):
                    def fn():
                        outs[(prec, agg)] = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, agg, precision=prec)
                    res.setdefault((prec, agg), []).append(time_it(fn, iters))
        for (prec, agg), v in sorted(res.items()):
            ms = min(v)
            a, b = outs[(prec, agg)].float(), outs[("exact", agg)].float()
            rel = float((a - b).abs().max() / b.abs().max())
            print(f"cfg{cfg} B={B:3d} N={N} {str(dt)[6:]:9s} {prec:5s} {agg:8s} {ms * 1e3:8.1f} us "
                  f"{nbytes / ms / 1e6:7.0f} GB/s ({nbytes / ms / 1e6 / 8000:.3f} of 8 TB/s)  max-rel vs exact {rel:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
