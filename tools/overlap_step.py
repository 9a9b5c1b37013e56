"""Whole bench step (unproject softmax -> soft-argmax over channels [0:17]) run three ways,
interleaved in one process, outputs compared bitwise:
  seq      one unproject over the batch, then one soft-argmax (bench.py's step)
  grp<G>   frame groups of G, unproject(g) -> soft-argmax(g) on one stream (MALL locality)
  ovl<G>   frame groups of G on two streams: soft-argmax(g) on a second stream after an
           event, concurrent with unproject(g+1) (the unprojection is LDS/VALU-latency bound
           and leaves HBM idle; the soft-argmax is HBM bound)
    python tools/overlap_step.py [--steps K]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402


def main():
    steps = 50
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    lib = _lib.load()
    dev = torch.device("cuda:0")
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()
    V, J, C = 64, 17, 32
    V3 = V ** 3
    for B, dt, groups in ((8, torch.float32, (1, 2, 4)), (32, torch.bfloat16, (4, 8, 16))):
        N = 4
        vb = synth.volumetric_batch(B, n_views=N, dtype=dt, device=dev, seed=0)
        code = 1 if dt == torch.bfloat16 else 0
        E = 2 if dt == torch.bfloat16 else 4
        vol = torch.empty((B, C, V, V, V), dtype=dt, device=dev)
        xyz = torch.empty((B, J, 3), device=dev)
        vout = torch.empty((B, J, V, V, V), dtype=dt, device=dev)
        ws = torch.empty(lib.mvn_softargmax3d_workspace_bytes(B, J, V, V, V), dtype=torch.uint8, device=dev)
        wss = [torch.empty(lib.mvn_softargmax3d_workspace_bytes(B, J, V, V, V), dtype=torch.uint8, device=dev)
               for _ in range(2)]

        def unproject(f0, nf, st):
            r = lib.mvn_unproject(vb.features.data_ptr() + f0 * N * C * 96 * 96 * E, code,
                                  vb.proj.data_ptr() + f0 * N * 48, vb.coords.data_ptr() + f0 * V3 * 12, None,
                                  vol.data_ptr() + f0 * C * V3 * E, code, nf, N, C, 96, 96, V, V, V, 2, 0,
                                  st.cuda_stream)
            assert r == 0, r

        def softargmax(f0, nf, st, w):
            r = lib.mvn_softargmax3d(vol.data_ptr() + f0 * C * V3 * E, code, C * V3, V3,
                                     vb.coords.data_ptr() + f0 * V3 * 12, 1.0, 1, xyz.data_ptr() + f0 * J * 12,
                                     vout.data_ptr() + f0 * J * V3 * E, code, w.data_ptr(), w.numel(), nf, J, V, V, V,
                                     st.cuda_stream)
            assert r == 0, r

        def step(mode, G):
            if mode == "seq":
                unproject(0, B, s0)
                softargmax(0, B, s0, ws)
            elif mode == "grp":
                for f0 in range(0, B, G):
                    unproject(f0, G, s0)
                    softargmax(f0, G, s0, ws)
            else:
                k = 0
                for f0 in range(0, B, G):
                    unproject(f0, G, s0)
                    ev = torch.cuda.Event()
                    ev.record(s0)
                    s1.wait_event(ev)
                    softargmax(f0, G, s1, wss[k & 1])
                    k += 1
                ev = torch.cuda.Event()
                ev.record(s1)
                s0.wait_event(ev)

        modes = [("seq", B)] + [(m, g) for g in groups for m in ("grp", "ovl")]
        res, ref = {}, {}
        for rnd in range(3):
            for mode, G in modes:
                name = mode if mode == "seq" else f"{mode}{G}"
                for _ in range(20):
                    step(mode, G)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s0)
                for _ in range(steps):
                    step(mode, G)
                b.record(s0)
                torch.cuda.synchronize()
                res.setdefault(name, []).append(a.elapsed_time(b) / steps)
                if rnd == 0:
                    ref[name] = (xyz.clone(), vout.clone())
        for name, v in res.items():
            ms = min(v)
            same = torch.equal(ref[name][0], ref["seq"][0]) and torch.equal(ref[name][1], ref["seq"][1])
            print(f"B={B:3d} {str(dt):15s} {name:7s} step {ms * 1e3:7.1f} us -> {B / ms * 1e3:8.0f} frames/s  "
                  f"same-as-seq: {same}", flush=True)


if __name__ == "__main__":
    main()
