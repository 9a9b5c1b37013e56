"""Time the tiled unprojection with parts ablated (MVN_UNPROJECT_ABLATE bits: 1 stores,
2 staging loads, 4 LDS tap reads) — attribution only, outputs are wrong when ablated."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
import torch  # noqa: E402

from mvn_rocm import op, synth  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_unproject import time_it  # noqa: E402

dev = torch.device("cuda:0")
for B, dt in ((8, torch.float32), (32, torch.bfloat16)):
    vb = synth.volumetric_batch(B, dtype=dt, device=dev, seed=0)
    res = {}
    for rnd in range(3):
        for ab in (0, 1, 2, 4, 3, 5, 6, 7):
            os.environ["MVN_UNPROJECT_ABLATE"] = str(ab)
            res.setdefault(ab, []).append(time_it(lambda: op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")))
    os.environ["MVN_UNPROJECT_ABLATE"] = "0"
    names = {0: "full", 1: "-stores", 2: "-loads", 4: "-ldsreads", 3: "-stores-loads", 5: "-stores-lds",
             6: "-loads-lds", 7: "-all(geometry+valu)"}
    for ab, v in res.items():
        print(f"{str(dt):15s} B={B:3d} {names[ab]:22s} {min(v) * 1e3:8.1f} us")
