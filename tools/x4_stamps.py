"""Per-block phase durations of the four-view unprojection from a diagnostic build
(tools/build_x4_variant.sh stamps -DMVN_X4_STAMPS=1).  python tools/x4_stamps.py tools/bin/stamps.so"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import _lib, synth  # noqa: E402

lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
res, args = _lib.SIGNATURES["mvn_unproject"]
lib.mvn_unproject.restype, lib.mvn_unproject.argtypes = res, args
lib.mvn_x4_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream
names = ["coords+corners+proj", "boxes", "regions", "chunks+issue", "slots+commit+barrier", "main loop"]
for B, dt, label in ((8, torch.float32, "cfg2 f32"), (32, torch.bfloat16, "cfg3 bf16")):
    vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
    code = 1 if dt == torch.bfloat16 else 0
    out = torch.empty((B, 32, 64, 64, 64), dtype=dt, device=dev)
    for agg in (2, 0):
        for _ in range(3):
            assert lib.mvn_unproject(vb.features.data_ptr(), code, vb.proj.data_ptr(), vb.coords.data_ptr(), None,
                                     out.data_ptr(), code, B, 4, 32, 96, 96, 64, 64, 64, agg, 0, stream) == 0
        torch.cuda.synchronize()
        nb = B * (64 ** 3 // (512 if code == 0 else 256))       # tile 4x8x16 (f32) / 4x8x8 (bf16)
        st = np.zeros(nb * 16, np.uint64)
        assert lib.mvn_x4_stamps(st.ctypes.data, st.nbytes) == 0
        st = st.reshape(nb, 16).astype(np.int64)
        d = np.diff(st[:, 1:8], axis=1)               # memtime phases (cycles)
        tot = st[:, 7] - st[:, 1]
        print(f"{label} agg={agg}: blocks {nb}, block lifetime median {np.median(tot):.0f} cyc, mean {tot.mean():.0f}")
        for i, n in enumerate(names):
            print(f"    {n:14s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  p90 {np.percentile(d[:, i], 90):8.0f}")
        print(f"    (chunk descriptors alone: median {np.median(st[:, 12] - st[:, 4]):8.0f}; first issue {np.median(st[:, 5] - st[:, 12]):8.0f})")
        for k, n in enumerate(("consume", "commit (vmcnt + ds_write)", "barrier", "issue")):
            print(f"    loop:{n:26s} median {np.median(st[:, 8 + k]):8.0f}")
        rt = (st[:, 0] - st[:, 0].min()) / 100.0      # s_memrealtime: 100 MHz -> us
        end = rt + tot / 2100.0                        # lifetime at ~2.1 GHz
        span = end.max()
        print(f"    block starts span {rt.max():.1f} us; per-block lifetime at ~2.1 GHz = {np.median(tot) / 2100:.2f} us")
        print(f"    estimated kernel span {span:.1f} us; last block start at {rt.max() / span:.3f} of it; "
              f"blocks ending after 90 % of the span: {(end > 0.9 * span).sum()}; "
              f"time with < half the block slots busy ~ {(span - np.percentile(end, 75)):.1f} us")
