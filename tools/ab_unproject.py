"""A/B timing of the unprojection kernels (tiled vs simple) on the bench configs, in one
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402


def time_it(fn, iters=20):
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
    dev = torch.device("cuda:0")
    for B, dt, label in ((8, torch.float32, "cfg2 f32 B=8"), (32, torch.bfloat16, "cfg3 bf16 B=32")):
        vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
        E = 2 if dt == torch.bfloat16 else 4
        nbytes = B * (E * (4 * 32 * 96 * 96 + 32 * 64 ** 3) + 12 * 64 ** 3 + 4 * 48)
        res = {}
        for rnd in range(3):
            for kern in ("tiled", "simple"):
                os.environ["MVN_UNPROJECT_KERNEL"] = kern
                for agg in ("softmax", "sum"):
                    ms = time_it(lambda: op.unproject_heatmaps(vb.features, vb.proj, vb.coords, agg))
                    res.setdefault((kern, agg), []).append(ms)
        os.environ["MVN_UNPROJECT_KERNEL"] = "tiled"
        a = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "sum")
        os.environ["MVN_UNPROJECT_KERNEL"] = "simple"
        b = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "sum")
        same = torch.equal(a, b)
        for (kern, agg), v in sorted(res.items()):
            ms = min(v)
            print(f"{label:16s} {kern:7s} {agg:8s} {ms:8.3f} ms  {nbytes / ms / 1e6:8.1f} GB/s  "
                  f"({nbytes / ms / 1e6 / 8000 * 100:5.1f}% of 8 TB/s)  {B / ms * 1e3:9.0f} frames/s")
        print(f"{label}: tiled == simple (sum, bitwise): {same}")


if __name__ == "__main__":
    main()
