"""Per-kernel HIP-event times of the config-2 step in three forms, same process, same data:
bench.Workload.step (op layer, outputs allocated per step), the op layer with preallocated
outputs, and direct C-ABI calls with preallocated outputs.
    python tools/step_modes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from mvn_rocm import _lib, op  # noqa: E402


def timed(fn, n=30):
    evs = []
    for _ in range(5):
        fn(None)
    torch.cuda.synchronize()
    for _ in range(n):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        fn(ev)
        evs.append(ev)
    torch.cuda.synchronize()
    return (sum(e[0].elapsed_time(e[1]) for e in evs) / n * 1e3, sum(e[1].elapsed_time(e[2]) for e in evs) / n * 1e3)


def main():
    dev = torch.device("cuda:0")
    cfg = bench._configs()["2"]
    wl = bench.Workload(cfg, 0, 1, dev)
    B, V3 = 8, 64 ** 3
    lib = _lib.load()
    vol = torch.empty((B, 32, 64, 64, 64), device=dev)
    xyz = torch.empty((B, 17, 3), device=dev)
    vout = torch.empty((B, 17, 64, 64, 64), device=dev)
    ws = torch.empty(lib.mvn_softargmax3d_workspace_bytes(B, 17, 64, 64, 64), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def eager(ev):
        if ev: ev[0].record()
        v = op.unproject_heatmaps(wl.feat, wl.proj, wl.coords, "softmax")
        if ev: ev[1].record()
        op.integrate_tensor_3d_with_coordinates(v[:, :17], wl.coords, True)
        if ev: ev[2].record()

    def direct(ev):
        if ev: ev[0].record()
        lib.mvn_unproject(wl.feat.data_ptr(), 0, wl.proj.data_ptr(), wl.coords.data_ptr(), None, vol.data_ptr(), 0,
                          B, 4, 32, 96, 96, 64, 64, 64, 2, 0, st)
        if ev: ev[1].record()
        lib.mvn_softargmax3d(vol.data_ptr(), 0, 32 * V3, V3, wl.coords.data_ptr(), 1.0, 1, xyz.data_ptr(),
                             vout.data_ptr(), 0, ws.data_ptr(), ws.numel(), B, 17, 64, 64, 64, st)
        if ev: ev[2].record()

    for rnd in range(3):
        for name, fn in (("op layer (bench)", eager), ("direct C ABI", direct)):
            u, s = timed(fn)
            print(f"round {rnd} {name:18s} unproject {u:7.1f} us  softargmax {s:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
