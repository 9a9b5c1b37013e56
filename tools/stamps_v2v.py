"""Per-phase timeline of the V2V front conv's tiles (diagnostic, design aid): a build of
csrc/v2v_front.hip patched with s_memtime stamps written by thread 0 of every block per tile
(g_vst[(block * 16 + tile) * 8 + phase], fetched with mvn_diag_vstamps) runs config 5's conv
(64 frames); prints median cycles per phase over all tiles.
    python tools/stamps_v2v.py path/to/stamp-build.so
Phases: 0 tile start (after the slices barrier), 1 first pass's fragments loaded,
2 the 12 common passes, 3 pass 48 (own x-row), 4 partial-sum exchange + barrier,
5 own sum + barrier, 6 next slices into LDS, 7 epilogue stores."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib  # noqa: E402
from mvn_rocm.v2v import fold_basic3d_block  # noqa: E402

NAMES = ["", "first pass fragments", "12 common passes", "pass 48 (own row)", "exchange + barrier",
         "own sum + barrier", "next slices to LDS", "epilogue stores"]


def main():
    lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
    res, args = _lib.SIGNATURES["mvn_v2v_front"]
    lib.mvn_v2v_front.restype, lib.mvn_v2v_front.argtypes = res, args
    lib.mvn_diag_vstamps.restype, lib.mvn_diag_vstamps.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    B, V = 64, 64
    g = torch.Generator().manual_seed(0)
    w = torch.randn(16, 32, 7, 7, 7, generator=g) * 0.02
    packed, scale, shift = fold_basic3d_block(w, torch.randn(16, generator=g), torch.rand(16, generator=g) + 0.5,
                                              torch.randn(16, generator=g), torch.randn(16, generator=g),
                                              torch.rand(16, generator=g) + 0.5, device=dev)
    x = torch.randn(B, V, V, V, 32, generator=g).to(torch.bfloat16).to(dev)
    o = torch.empty(B, 16, V, V, V, device=dev)
    for _ in range(6):
        assert lib.mvn_v2v_front(x.data_ptr(), packed.data_ptr(), scale.data_ptr(), shift.data_ptr(), o.data_ptr(),
                                 0, B, V, stream) == 0
    torch.cuda.synchronize()
    nblk = B * (V // 4) * (V // 16)
    buf = np.zeros(nblk * 16 * 8, dtype=np.uint64)
    assert lib.mvn_diag_vstamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(nblk, 16, 8).astype(np.int64)
    tile = st[:, :, 7] - st[:, :, 0]
    gap = st[:, 1:, 0] - st[:, :-1, 7]          # end of one tile's epilogue -> next tile's start barrier
    print(f"conv 64 frames: {nblk} blocks x 16 tiles; tile median {np.median(tile):.0f} cycles "
          f"(p10 {np.percentile(tile, 10):.0f}, p90 {np.percentile(tile, 90):.0f}); "
          f"loop back to the next tile's barrier median {np.median(gap):.0f}")
    for i in range(1, 8):
        d = st[:, :, i] - st[:, :, i - 1]
        print(f"   {NAMES[i]:24s} median {np.median(d):8.0f}  mean {d.mean():8.0f}  ({100 * np.median(d) / np.median(tile):4.1f} %)")
    print(f"   MFMA work per tile per wave: 12 x 112 + 28 = 1,372 MFMAs x 16 cycles = 21,952 cycles")


if __name__ == "__main__":
    main()
