"""Benchmark of the volumetric triangulation hot path on MI355X.

Metric (BASELINE.json): multiview frames/sec (4-view x 64^3 unproject + soft-argmax).
One "step" = one pass of the hot path over one batch of synthetic frames resident in
HBM:  unproject_heatmaps(softmax aggregation) -> integrate_tensor_3d_with_coordinates
over channels [0:17] of the unprojected volume (the stand-in for V2V)
-> (N > 1) one all-gather of the (B/N, 17, 3) joints over RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4] [--no-cpu-baseline]

With the default --config 2 the line also carries `secondary` (config 3, bf16, 32 frames)
and `config5` (unproject written channels-last + the V2V front Conv3d block on bf16 MFMA,
64 frames, with its own MFMA roofline); --no-secondary drops both.

N > 1 is launched by torch.distributed.run (one process per GPU); every rank builds its
own frames from (seed, global frame index) — weak scaling, fixed frames per GPU.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mvn_rocm import dist as mdist, op, synth  # noqa: E402

METRIC = "multiview frames/sec (4-view x 64^3 unproject+soft-argmax), 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# BASELINE.json configs (per GPU): name -> (views, channels, heatmap, volume, joints, frames/GPU, dtype)
CONFIGS = {
    "2": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=8, dtype=torch.float32,
              label="cfg2: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg) + 17-joint soft-argmax, fp32"),
    "3": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=32, dtype=torch.bfloat16,
              label="cfg3: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg) + 17-joint soft-argmax, bf16"),
    "4": dict(views=8, channels=32, heatmap=96, volume=64, joints=17, frames=16, dtype=torch.float32,
              label="cfg4: 8 views (CMU-style) x 32 ch x 96^2 -> 64^3 unproject + soft-argmax, fp32"),
    "5": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=64, dtype=torch.bfloat16,
              label="cfg5: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg, channels-last bf16) + V2V front "
                    "Basic3DBlock(32,16,7) conv3d+BN+ReLU on bf16 MFMA"),
}
MFMA_BF16_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 (no sparsity)
V2V_FLOP_PER_FRAME = 2 * 32 * 16 * 343 * 64 ** 3


def unproject_bytes(c, E):
    """Algorithmic bytes of one frame's unprojection: features read once,
    volume written once, coordinates read once (f32), projections read."""
    V3 = c["volume"] ** 3
    return E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3) + 4 * 3 * V3 + 4 * 12 * c["views"]


def frame_bytes(c, E):
    """Whole-path algorithmic bytes per frame (SURVEY.md §8d / BASELINE.md §4)."""
    V3 = c["volume"] ** 3
    return (E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3 + 2 * c["joints"] * V3)
            + 4 * (2 * 3 * V3) + 4 * (12 * c["views"] + 3 * c["joints"]))


def measured_traffic(cfg_name):
    """HBM bytes per unprojection launch from the newest committed PMC summary
    (profiles/rNN_traffic.json, written by tools/profile_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes over the same kernel and config), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    for k, d in data.get(f"cfg{cfg_name}", {}).items():
        if k.startswith("unproject_tiled<2,") and "hbm_bytes_per_launch" in d:
            return d["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    return None, None


def kernel_name(c):
    t = "float" if c["dtype"] == torch.float32 else "bf16"
    return f"unproject_tiled<softmax, {t}, {t}, {4 if c['views'] <= 4 else 8} views>"


def dtype_name(dt):
    return {torch.float32: "f32", torch.bfloat16: "bf16"}[dt]


def unproject_bytes_cuboid(c, E):
    """Algorithmic bytes of one frame's unprojection with in-kernel coordinates: features
    read once, volume written once, cuboid (18 f32) and projections read."""
    V3 = c["volume"] ** 3
    return E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3) + 4 * 18 + 4 * 12 * c["views"]


def frame_bytes_cuboid(c, E):
    V3 = c["volume"] ** 3
    return (E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3 + 2 * c["joints"] * V3)
            + 4 * 2 * 18 + 4 * (12 * c["views"] + 3 * c["joints"]))


class Workload:
    def __init__(self, cfg, rank, world, device, seed=0, cuboid=False):
        self.cfg, self.rank, self.world, self.device = cfg, rank, world, device
        B = cfg["frames"]
        vb = synth.volumetric_batch(B, n_views=cfg["views"], channels=cfg["channels"], heatmap=cfg["heatmap"],
                                    volume=cfg["volume"], dtype=cfg["dtype"], device=device, seed=seed,
                                    first_frame=rank * B)
        self.feat, self.proj, self.coords = vb.features, vb.proj, vb.coords
        if cuboid:      # coordinates formed inside both kernels (mvn_*_cuboid), never materialised
            self.coords = vb.cuboids(device)
        self.ev = []

    def step(self, timed=False):
        J = self.cfg["joints"]
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        vol = op.unproject_heatmaps(self.feat, self.proj, self.coords, "softmax")
        if timed:
            e1.record()
            self.ev.append((e0, e1))
        xyz, sm = op.integrate_tensor_3d_with_coordinates(vol[:, :J], self.coords, True)
        if self.world > 1:      # the path's one exchange: joints of every rank, RCCL over xGMI
            xyz = mdist.gather_joints(xyz, self.cfg["frames"] * self.world)
        return xyz, sm

    def unproject_ms(self):
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) for a, b in self.ev]
        return sum(t) / len(t)


def run_config(name, args, rank, world, device, cuboid=False, cfg=None):
    cfg = cfg if cfg is not None else CONFIGS[name]
    wl = Workload(cfg, rank, world, device, cuboid=cuboid)
    for _ in range(args.warmup):
        wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wl.step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    E = 2 if cfg["dtype"] == torch.bfloat16 else 4
    frames_total = cfg["frames"] * world * args.steps
    unproj_ms = wl.unproject_ms()
    launch_bytes = (unproject_bytes_cuboid if cuboid else unproject_bytes)(cfg, E) * cfg["frames"]
    achieved = launch_bytes / (unproj_ms * 1e-3) / 1e9
    return dict(
        cfg=cfg, elapsed=elapsed, fps=frames_total / elapsed, ms_per_step=elapsed / args.steps * 1e3,
        unproject_ms=unproj_ms, launch_bytes=launch_bytes, achieved_gbps=achieved,
        path_gbps=(frame_bytes_cuboid if cuboid else frame_bytes)(cfg, E) * frames_total / elapsed / 1e9)


def run_config5(args, rank, world, device, cuboid=False):
    """Config 5: unproject (softmax, written channels-last bf16) + V2V front block on MFMA;
    roofline of the front block against the bf16 dense MFMA peak."""
    from mvn_rocm import v2v
    cfg = CONFIGS["5"]
    B = cfg["frames"]
    vb = synth.volumetric_batch(B, n_views=cfg["views"], channels=cfg["channels"], heatmap=cfg["heatmap"],
                                volume=cfg["volume"], dtype=cfg["dtype"], device=device, seed=0, first_frame=rank * B)
    g = torch.Generator().manual_seed(0)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=device)
    ev = []
    coords = vb.cuboids(device) if cuboid else vb.coords

    def step(timed=False):
        cl = v2v.unproject_channels_last(vb.features, vb.proj, coords, "softmax")
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        y = v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16)
        if timed:
            e1.record()
            ev.append((e0, e1))
        return y

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    conv_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    tflops = V2V_FLOP_PER_FRAME * B / (conv_ms * 1e-3) / 1e12
    return dict(workload=cfg["label"], value=B * world * args.steps / elapsed, unit="frames/s",
                ms_per_step=elapsed / args.steps * 1e3, frames_per_gpu=B, dtype="bf16",
                roofline={"kernel": "v2v_front<bf16> (Conv3d 32->16 k7 + BN + ReLU)", "bound": "mfma",
                          "achieved": tflops, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / MFMA_BF16_PEAK_TFLOPS, "launch_ms": conv_ms,
                          "flop_per_launch": V2V_FLOP_PER_FRAME * B})


def cpu_baseline(seconds=15.0):
    """The reference algorithm restated op-for-op in torch-CPU (oracle/restate_torch.py),
    timed on this host on one frame of config 2 at a time (bounded sample)."""
    from oracle import restate_torch
    import warnings
    warnings.filterwarnings("ignore")
    vb = synth.volumetric_batch(1, seed=0)
    cfg = CONFIGS["2"]
    n, t0 = 0, time.perf_counter()
    while True:
        vol = restate_torch.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
        restate_torch.integrate_tensor_3d_with_coordinates(vol[:, :cfg["joints"]], vb.coords, True)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return dict(value=n / el, unit="frames/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{n} frame(s) of config 2 (4x32x96^2 -> 64^3, softmax agg, 17-joint soft-argmax, fp32) "
                       f"through oracle/restate_torch.py in {el:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="2", choices=[k for k in sorted(CONFIGS) if k != "5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-in-kernel-coords", action="store_true",
                    help="skip the in-kernel-coordinates run (keeps rocprof kernel means per variant clean)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    main_res = run_config(args.config, args, rank, world, device)
    secondary = None
    if not args.no_secondary and args.config == "2":
        s = run_config("3", args, rank, world, device)
        secondary = dict(workload=s["cfg"]["label"], value=s["fps"], unit="frames/s", ms_per_step=s["ms_per_step"],
                         frames_per_gpu=s["cfg"]["frames"], unproject_ms=s["unproject_ms"],
                         unproject_achieved_gbps=s["achieved_gbps"],
                         unproject_frac=s["achieved_gbps"] / HBM_PEAK_GBPS,
                         path_algorithmic_gbps=s["path_gbps"], path_frac=s["path_gbps"] / HBM_PEAK_GBPS)
    in_kernel_coords = None
    if not args.no_secondary and not args.no_in_kernel_coords:
        # the same workload with the coordinate volume formed inside both kernels from the
        # per-frame cuboids instead of read from HBM
        k = run_config(args.config, args, rank, world, device, cuboid=True)
        in_kernel_coords = dict(workload=k["cfg"]["label"] + ", coordinates formed in-kernel from per-frame cuboids",
                                value=k["fps"], unit="frames/s", ms_per_step=k["ms_per_step"],
                                unproject_ms=k["unproject_ms"], unproject_algorithmic_bytes_per_launch=k["launch_bytes"],
                                unproject_achieved_gbps=k["achieved_gbps"],
                                unproject_frac=k["achieved_gbps"] / HBM_PEAK_GBPS,
                                path_algorithmic_gbps=k["path_gbps"])
    cfg4 = None
    if not args.no_secondary and args.config == "2":
        # BASELINE config 4: 8 views, a global batch of 128 frames sharded over the ranks
        # (strong scaling: 128 / world frames per GPU), joints all-gathered over RCCL
        c4 = dict(CONFIGS["4"], frames=max(1, 128 // world))
        r4 = run_config("4", args, rank, world, device, cfg=c4)
        cfg4 = dict(workload=c4["label"] + ", global batch 128 sharded over the ranks", value=r4["fps"],
                    unit="frames/s", scaling="strong", global_batch=c4["frames"] * world, frames_per_gpu=c4["frames"],
                    ms_per_step=r4["ms_per_step"], unproject_ms=r4["unproject_ms"],
                    unproject_achieved_gbps=r4["achieved_gbps"], unproject_frac=r4["achieved_gbps"] / HBM_PEAK_GBPS,
                    path_algorithmic_gbps=r4["path_gbps"])
    cfg5 = None
    if not args.no_secondary and args.config == "2":
        cfg5 = run_config5(args, rank, world, device)
        if not args.no_in_kernel_coords:
            k5 = run_config5(args, rank, world, device, cuboid=True)
            cfg5["in_kernel_coords"] = dict(value=k5["value"], unit="frames/s", ms_per_step=k5["ms_per_step"])
    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline()

    if rank == 0:
        r, c = main_res, main_res["cfg"]
        traffic, traffic_src = measured_traffic(args.config)
        line = {
            "metric": METRIC,
            "value": r["fps"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype_name(c["dtype"]),
            "data": "synthetic (seeded ring cameras, N(0,1) features, rotated 2.5 m cuboids; SURVEY.md §8d)",
            "config": {"workload": c["label"], "global_batch": c["frames"] * world, "frames_per_gpu": c["frames"],
                       "views": c["views"], "channels": c["channels"], "heatmap": c["heatmap"],
                       "volume": c["volume"], "joints": c["joints"], "parallelism": f"dp{world}",
                       "collective": "all_gather joints (RCCL)" if world > 1 else None},
            "roofline": {"kernel": kernel_name(c), "bound": "hbm",
                         "achieved": r["achieved_gbps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": r["achieved_gbps"] / HBM_PEAK_GBPS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "launch_ms": r["unproject_ms"], "algorithmic_bytes_per_launch": r["launch_bytes"]},
            "path_algorithmic_gbps": r["path_gbps"],
            "cpu_baseline": base,
            "secondary": secondary,
            "in_kernel_coords": in_kernel_coords,
            "config4": cfg4,
            "config5": cfg5,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
