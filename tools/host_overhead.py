"""Host-side cost of one bench step (op layer: validation, custom-op dispatch, allocation,
ctypes) against its GPU time, per layer of the dispatch, and the same step replayed from a
captured HIP graph.  Also the driver's own shape: 20 timed steps after 5 warmup steps.
    python tools/host_overhead.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def enqueue_us(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def main():
    from mvn_rocm import _lib, _ops, op
    dev = torch.device("cuda:0")
    lib = _lib.load()
    for name in ("2", "3"):
        cfg = bench._configs()[name]
        wl = bench.Workload(cfg, 0, 1, dev)
        J = cfg["joints"]
        B, N, C, H, W = wl.feat.shape
        V = wl.coords.shape[1]
        out = torch.empty((B, C, V, V, V), dtype=wl.feat.dtype, device=dev)
        dt = _ops._DTYPE_CODE[wl.feat.dtype]
        stream = torch.cuda.current_stream().cuda_stream
        fp, pp, cp, op_ = wl.feat.data_ptr(), wl.proj.data_ptr(), wl.coords.data_ptr(), out.data_ptr()
        raw = lambda: lib.mvn_unproject(fp, dt, pp, cp, None, op_, dt, B, N, C, H, W, V, V, V, 2, 0, stream)  # noqa: E731
        vol = op.unproject_heatmaps(wl.feat, wl.proj, wl.coords, "softmax")
        rows = [
            ("ctypes mvn_unproject", raw),
            ("torch.ops.mvn_rocm.unproject", lambda: _ops.unproject(wl.feat, wl.proj, wl.coords, None, 2, False, dt)),
            ("op.unproject_heatmaps", lambda: op.unproject_heatmaps(wl.feat, wl.proj, wl.coords, "softmax")),
            ("op.integrate_tensor_3d_with_coordinates",
             lambda: op.integrate_tensor_3d_with_coordinates(vol[:, :J], wl.coords, True)),
            ("bench step (untimed)", lambda: wl.step(False)),
        ]
        for label, fn in rows:
            e, w = enqueue_us(fn)
            print(f"cfg{name}: {label:42s} enqueue {e:7.1f} us/call, wall {w:7.1f} us/call", flush=True)
        # the driver's shape: 5 warmup + 20 timed steps, wall vs the event-timed kernels
        wl.reserve_events(20)
        for _ in range(5):
            wl.step(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            wl.step(True)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 20 * 1e3
        u, s = wl.kernel_ms()
        print(f"cfg{name}: 20 timed steps: {wall:.4f} ms/step wall, kernels {u:.4f} + {s:.4f} = {u + s:.4f} ms "
              f"({(wall - u - s) / wall * 100:.1f} % outside)", flush=True)
        s_ = torch.cuda.Stream()
        s_.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_):
            for _ in range(3):
                wl.step(False)
        torch.cuda.current_stream().wait_stream(s_)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            res = wl.step(False)
        e, w = enqueue_us(g.replay)
        print(f"cfg{name}: {'graph replay of the step':42s} enqueue {e:7.1f} us/call, wall {w:7.1f} us/call", flush=True)
        del g, res, out, vol


if __name__ == "__main__":
    main()
