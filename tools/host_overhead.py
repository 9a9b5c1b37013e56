"""Host-side cost of one bench step (op layer: validation, custom-op dispatch, allocation,
ctypes) against its GPU time, and the same step replayed from a captured HIP graph.
    python tools/host_overhead.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for name in ("2", "3"):
        cfg = bench._configs()[name]
        wl = bench.Workload(cfg, 0, 1, dev)
        for _ in range(10):
            wl.step(False)
        torch.cuda.synchronize()
        n = 50
        t0 = time.perf_counter()
        for _ in range(n):
            wl.step(False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"cfg{name}: enqueue {(t1 - t0) / n * 1e6:7.1f} us/step, wall {(t2 - t0) / n * 1e6:7.1f} us/step (eager)",
              flush=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                wl.step(False)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = wl.step(False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"cfg{name}: enqueue {(t1 - t0) / n * 1e6:7.1f} us/step, wall {(t2 - t0) / n * 1e6:7.1f} us/step (graph)",
              flush=True)
        del g, out


if __name__ == "__main__":
    main()
