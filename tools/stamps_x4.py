"""Per-phase timeline of the four-view unprojection's blocks (diagnostic, design aid): a build
of csrc/unproject_x4.hip patched with s_memtime stamps written by thread 0 of every block
(g_stamps[block * 10 + phase], fetched with mvn_diag_stamps) runs configs 2 and 3; prints the
median cycles of each phase over the blocks and the block lifetime.
    python tools/stamps_x4.py path/to/stamp-build.so
Phases: 0 entry, 1 coordinates + projection, 2 footprint butterfly + barrier + combine,
3 regions, 4 chunk descriptors, 5 first group's loads issued, 6 tap slots, 7 first commit +
barrier, 9 end of the channel loop (8 unused)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402

NAMES = {1: "coords + projection", 2: "box butterfly + barrier", 3: "regions", 4: "chunk descriptors",
         5: "first loads issued", 6: "tap slots", 7: "first commit + barrier", 9: "channel loop (8 groups)"}


def main():
    lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
    res, args = _lib.SIGNATURES["mvn_unproject"]
    lib.mvn_unproject.restype, lib.mvn_unproject.argtypes = res, args
    lib.mvn_diag_stamps.restype, lib.mvn_diag_stamps.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    for B, dt, label, nblk in ((8, torch.float32, "cfg2 f32 B=8 (tile 4x8x16)", 8 * 512),
                               (32, torch.bfloat16, "cfg3 bf16 B=32 (tile 4x8x8)", 32 * 1024)):
        vb = synth.volumetric_batch(B, n_views=4, dtype=dt, device=dev, seed=0)
        code = 1 if dt == torch.bfloat16 else 0
        out = torch.empty((B, 32, 64, 64, 64), dtype=dt, device=dev)
        for _ in range(30):
            r = lib.mvn_unproject(vb.features.data_ptr(), code, vb.proj.data_ptr(), vb.coords.data_ptr(), None,
                                  out.data_ptr(), code, B, 4, 32, 96, 96, 64, 64, 64, 2, 0, stream)
            assert r == 0, r
        torch.cuda.synchronize()
        buf = np.zeros(nblk * 10, dtype=np.uint64)
        assert lib.mvn_diag_stamps(buf.ctypes.data, buf.nbytes) == 0
        st = buf.reshape(nblk, 10).astype(np.int64)
        ok = st[:, 9] > 0
        st = st[ok]
        life = st[:, 9] - st[:, 0]
        print(f"{label}: {ok.sum()} one-pass blocks; block lifetime median {np.median(life):.0f} cycles "
              f"(p10 {np.percentile(life, 10):.0f}, p90 {np.percentile(life, 90):.0f}); kernel span "
              f"{st[:, 9].max() - st[:, 0].min():.0f}")
        prev = 0
        for i in (1, 2, 3, 4, 5, 6, 7, 9):
            d = st[:, i] - st[:, prev]
            print(f"   {NAMES[i]:28s} median {np.median(d):8.0f}  mean {d.mean():8.0f}  ({100 * np.median(d) / np.median(life):4.1f} %)")
            prev = i


if __name__ == "__main__":
    main()
