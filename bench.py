"""Benchmark of the volumetric triangulation hot path on MI355X.

Metric (BASELINE.json): multiview frames/sec (4-view x 64^3 unproject + soft-argmax).
One "step" = one pass of the hot path over one batch of synthetic frames resident in
HBM:  unproject_heatmaps(softmax aggregation) -> integrate_tensor_3d_with_coordinates
over channels [0:17] of the unprojected volume (the stand-in for V2V)
-> (N > 1) one all-gather of the (B/N, 17, 3) joints over RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4] [--no-cpu-baseline]
                    [--no-secondary] [--dry-run]

Process model (the reference's DDP model, /root/reference/train.py:370-382): one process
per GPU.  Launched by torch.distributed.run (WORLD_SIZE set) every process is one rank.
Launched as `python bench.py --gpus N` with no WORLD_SIZE, this process spawns the N rank
processes itself (fresh interpreters with a torchrun-style environment, before anything
here touches the GPU), waits for them and exits with their status.  Every rank builds
its own frames from (seed, global frame index); the headline config is weak scaling
(8 frames per GPU), config 4 is strong scaling (a global batch of 128 split over the
ranks).  Rank 0 prints ONE JSON line.

--dry-run runs the whole multi-process protocol on the CPU (gloo): rank bring-up,
barriers, max-over-ranks timing and the joints all-gather, with a stand-in step that
needs no GPU (tests/test_bench.py).  --dist-backend gloo --share-device runs the real GPU
step on several ranks sharing cuda:0 with host-side collectives (RCCL refuses two ranks on
one device): the multi-rank path on a one-GPU box (tests/test_gpu_bench_multirank.py).

Every config also reports `telemetry` (sclk, mclk, socket power, hotspot temperature, GFX
activity and power-limit residency sampled during an untimed burst of the same step right
after its timed region) and the line carries `gpu` (UUID, ASIC serial, power cap).

With the default --config 2 the line also carries `secondary` (config 3, bf16, 32 frames,
with its own roofline block), `config1` (the algebraic path: DLT at batch 1, 4 views x 17
joints, and the 2D soft-argmax -> DLT chain), `config4` and `config5` (unproject written
channels-last + the V2V front Conv3d block on bf16 MFMA, 64 frames, MFMA roofline);
--no-secondary drops them.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "learnable-triangulation-pytorch_amd"))
sys.path.insert(0, ROOT)

METRIC = "multiview frames/sec (4-view x 64^3 unproject+soft-argmax), 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 (no sparsity)
V2V_FLOP_PER_FRAME = 2 * 32 * 16 * 343 * 64 ** 3


def _configs():
    import torch
    # BASELINE.json configs (per GPU): views, channels, heatmap, volume, joints, frames/GPU, dtype
    return {
        "2": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=8, dtype=torch.float32,
                  label="cfg2: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg) + 17-joint soft-argmax, fp32"),
        "3": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=32, dtype=torch.bfloat16,
                  label="cfg3: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg) + 17-joint soft-argmax, bf16"),
        "4": dict(views=8, channels=32, heatmap=96, volume=64, joints=17, frames=16, dtype=torch.float32,
                  label="cfg4: 8 views (CMU-style) x 32 ch x 96^2 -> 64^3 unproject + soft-argmax, fp32"),
        "5": dict(views=4, channels=32, heatmap=96, volume=64, joints=17, frames=64, dtype=torch.bfloat16,
                  label="cfg5: 4 views x 32 ch x 96^2 -> 64^3 unproject(softmax agg, channels-last bf16) + V2V "
                        "front Basic3DBlock(32,16,7) conv3d+BN+ReLU on bf16 MFMA"),
    }


# ----------------------------------------------------------------------------- process model
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Spawn n rank processes of this script (torchrun-style environment, rendezvous on
    127.0.0.1) and return the first non-zero exit status, or 0.  Called before anything in
    this process touches the GPU; the ranks are fresh child processes, never an exec."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every rank: whichever fails first (not only rank 0) ends the others, which would
    # otherwise block in a barrier or collective that never completes
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if live:
            time.sleep(0.05)
    return rc


class Clock:
    """Barrier + device sync around the timed region; max over ranks."""

    def __init__(self, world, device, dry, host_collectives=False):
        self.world, self.device, self.dry = world, device, dry
        self.host = host_collectives       # gloo process group: collectives on host tensors

    def sync(self):
        import torch
        if not self.dry:
            torch.cuda.synchronize()

    def fence(self):
        import torch.distributed as dist
        self.sync()
        if self.world > 1:
            dist.barrier()
        self.sync()

    def max_over_ranks(self, seconds):
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return seconds
        t = torch.tensor([seconds], device="cpu" if self.host else self.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


def settle_steps(step, args, clock):
    """Untimed clock settling before the warmup: the GPU comes out of idle (process start,
    host-side data generation) at a low clock and takes ~25 ms of back-to-back launches to
    reach its loaded clock (config-2 unprojection 214 -> 172 us over the first 90 steps,
    tools/warmup_curve.py; MI355X_MICROARCH.md 'DVFS give-back' measures after >= 2 s of
    launches).  Runs ~args.settle seconds of steps, the same count on every rank (a step
    may hold a collective)."""
    if args.settle <= 0 or clock.dry:
        return 0
    for _ in range(3):          # first launches (code loading) are not representative
        step(False)
    clock.sync()
    t0 = time.perf_counter()
    for _ in range(5):
        step(False)
    clock.sync()
    per = max((time.perf_counter() - t0) / 5, 1e-5)
    n = int(clock.max_over_ranks(min(args.settle / per, 100000.0)))
    for _ in range(n):
        step(False)
    return n + 8


def timed_loop(step, args, clock):
    settle_steps(step, args, clock)
    for _ in range(args.warmup):
        step(False)
    clock.fence()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    clock.fence()
    return clock.max_over_ranks(time.perf_counter() - t0)


# ----------------------------------------------------------------------------- GPU telemetry
def _smi(fn, *a):
    try:
        return fn(*a)
    except Exception:       # telemetry must never fail the bench
        return None


def gpu_identity(device):
    """Which MI355X the line was measured on (so that lines from different boxes can be
    compared): ASIC serial / UUID and the board's power cap, from amdsmi."""
    import torch
    try:
        import amdsmi
        h = torch.cuda._get_amdsmi_handler(device)
    except Exception:
        return None
    asic = _smi(amdsmi.amdsmi_get_gpu_asic_info, h) or {}
    cap = _smi(amdsmi.amdsmi_get_power_cap_info, h) or {}
    return {"uuid": _smi(amdsmi.amdsmi_get_gpu_device_uuid, h), "asic_serial": asic.get("asic_serial"),
            "market_name": asic.get("market_name"), "power_cap_w": (cap.get("power_cap") or 0) / 1e6 or None}


def telemetry(device, step, seconds=0.15, samples=6):
    """Clocks, power and temperature the GPU holds under this config's load: an untimed burst
    of the same step (~`seconds` of GPU work, right after the timed region, so the same
    thermal and power state) is enqueued and amdsmi is sampled while it runs.  Medians of
    `samples` reads: sclk / mclk (MHz), socket power (W), hotspot temperature (C), GFX
    activity (%), and the throttle status word (0 = no throttling)."""
    import statistics
    import torch
    try:
        import amdsmi
        h = torch.cuda._get_amdsmi_handler(device)
    except Exception:
        return None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):         # GPU time per step (one synchronised step would count the sync)
        step(False)
    torch.cuda.synchronize()
    per = max((time.perf_counter() - t0) / 10, 1e-5)
    for _ in range(max(4, int(seconds / per))):
        step(False)
    reads = {"sclk_mhz": [], "mclk_mhz": [], "power_w": [], "temp_hotspot_c": [], "gfx_activity_pct": [],
             "throttle_status": []}

    def num(d, *keys):              # the first numeric field ("N/A" strings are skipped)
        for k in keys:
            if isinstance(d.get(k), (int, float)):
                return d[k]
        return None
    m0 = _smi(amdsmi.amdsmi_get_gpu_metrics_info, h) or {}
    for _ in range(samples):
        time.sleep(seconds / (2 * samples))
        g = _smi(amdsmi.amdsmi_get_clock_info, h, amdsmi.AmdSmiClkType.GFX) or {}
        m = _smi(amdsmi.amdsmi_get_clock_info, h, amdsmi.AmdSmiClkType.MEM) or {}
        pw = _smi(amdsmi.amdsmi_get_power_info, h) or {}
        mt = _smi(amdsmi.amdsmi_get_gpu_metrics_info, h) or {}
        for k, v in (("sclk_mhz", num(g, "clk", "cur_clk")), ("mclk_mhz", num(m, "clk", "cur_clk")),
                     ("power_w", num(pw, "current_socket_power", "socket_power", "average_socket_power")),
                     ("temp_hotspot_c", num(mt, "temperature_hotspot")), ("gfx_activity_pct", num(mt, "average_gfx_activity")),
                     ("throttle_status", num(mt, "throttle_status"))):
            if isinstance(v, (int, float)):
                reads[k].append(v)
    m1 = _smi(amdsmi.amdsmi_get_gpu_metrics_info, h) or {}
    torch.cuda.synchronize()
    out = {k: (statistics.median(v) if v else None) for k, v in reads.items()}
    out["samples"] = samples
    # share of the sampling window the SMU spent at the package power limit (PPT residency
    # accumulator over the firmware's accumulation counter; 0 = never power-limited)
    dp, da = (num(m1, "ppt_residency_acc") or 0) - (num(m0, "ppt_residency_acc") or 0), \
        (num(m1, "accumulation_counter") or 0) - (num(m0, "accumulation_counter") or 0)
    out["ppt_limited_frac"] = round(dp / da, 4) if da > 0 else None
    return out


def rank_identity(device, rank, local, dry):
    """Who this rank is and which device it computed on: (rank, local rank, host, pid) and the
    device's UUID (amdsmi, else torch's), PCI address and name.  Gathered from every rank, the
    list shows that an N-rank RCCL line ran on N distinct GPUs."""
    ident = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "pid": os.getpid()}
    if dry:
        ident.update(device="cpu", device_uuid=None)
        return ident
    import torch
    p = torch.cuda.get_device_properties(device)
    g = gpu_identity(device) or {}
    ident.update(device=str(device), device_uuid=g.get("uuid") or str(getattr(p, "uuid", "")) or None,
                 pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", name=p.name)
    return ident


def gather_objects(obj, world):
    """[obj of rank 0, ..., obj of rank world-1] on every rank (one all_gather_object)."""
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def dist_record(ident, world, backend):
    """The line's `dist` block: backend, every rank's identity, and the number of distinct
    devices they computed on (== world under RCCL, which refuses two ranks on one GPU)."""
    ranks = gather_objects(ident, world)
    devs = {(r["host"], r.get("device_uuid") or r.get("pci") or r["device"]) for r in ranks}
    return {"backend": backend, "world": world, "ranks": ranks, "distinct_devices": len(devs)}


# ----------------------------------------------------------------------------- algorithmic bytes
def unproject_bytes(c, E, cuboid=False):
    """Algorithmic bytes of one frame's unprojection: features read once,
    volume written once, coordinates read once (f32; 18 floats of cuboid when formed
    in-kernel), projections read."""
    V3 = c["volume"] ** 3
    coords = 4 * 18 if cuboid else 4 * 3 * V3
    return E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3) + coords + 4 * 12 * c["views"]


def frame_bytes(c, E, cuboid=False):
    """Whole-path algorithmic bytes per frame (SURVEY.md §8d / BASELINE.md §4)."""
    V3 = c["volume"] ** 3
    coords = 4 * 2 * 18 if cuboid else 4 * (2 * 3 * V3)
    return (E * (c["views"] * c["channels"] * c["heatmap"] ** 2 + c["channels"] * V3 + 2 * c["joints"] * V3)
            + coords + 4 * (12 * c["views"] + 3 * c["joints"]))


def measured_traffic(cfg_name, precision="exact"):
    """HBM bytes per unprojection launch from the newest committed PMC summary
    (profiles/rNN_traffic.json: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the
    same kernel and config), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_traffic.json")))
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    for k, d in data.get(f"cfg{cfg_name}", {}).items():
        if not (k.startswith(("unproject_x4<2,", "unproject_tiled<2,")) and "hbm_bytes_per_launch" in d):
            continue
        # unproject_x4<AGG, TIn, TOut, K, CL, FAST>: the last template argument is the arithmetic
        # (profiles before round 6 name 5 arguments: exact)
        args = k[k.index("<") + 1:k.rindex(">")].split(",")
        fast = k.startswith("unproject_x4") and len(args) >= 6 and args[5].strip() == "1"
        if fast == (precision == "fast"):
            return d["hbm_bytes_per_launch"], os.path.relpath(files[-1], ROOT)
    return None, None


def kernel_name(c, precision="exact"):
    import torch
    t = "float" if c["dtype"] == torch.float32 else "bf16"
    p = "" if precision == "exact" else (", fast: bf16 pixel-pair slots, v_dot2" if t == "bf16" and c["views"] == 4
                                        else ", fast")
    if c["views"] == 4:      # the chunk-staged kernel (csrc/unproject_x4.hip), tile per dtype
        return f"unproject_x4<softmax, {t}, {t}, tile {'4x8x16' if t == 'float' else '8x8x8'}{p}>"
    return f"unproject_x4<softmax, {t}, {t}, 8 views, 2-channel slots, tile 4x8x8{p}>"


def dtype_name(dt):
    import torch
    return {torch.float32: "f32", torch.bfloat16: "bf16"}[dt]


_COPY_GBPS = None


def copy_bandwidth(device):
    """Measured device-to-device copy bandwidth (SURVEY.md §8d asks for the fraction of it
    next to the spec peak): a 1 GiB f32 buffer copied back to back, bytes read + written
    per second, best of 3 x 20 copies after ~0.3 s of settling."""
    global _COPY_GBPS
    if _COPY_GBPS is None:
        import torch
        n = (1 << 30) // 4
        src = torch.empty(n, device=device).normal_()
        dst = torch.empty_like(src)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:     # (synchronised: enqueueing alone queued ~1.5 s of copies)
            for _ in range(4):
                dst.copy_(src)
            torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                dst.copy_(src)
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) / 20)
        _COPY_GBPS = 2 * n * 4 / (best * 1e-3) / 1e9
        del src, dst
    return _COPY_GBPS


def _ratio(a, b):
    return None if a is None else a / b


def roofline(c, r, cfg_name, device=None):
    prec = r.get("precision", "exact")
    traffic, src = measured_traffic(cfg_name, prec)
    out = {"kernel": kernel_name(c, prec), "precision": prec, "bound": "hbm", "achieved": r["achieved_gbps"], "peak": HBM_PEAK_GBPS,
           "unit": "GB/s", "frac": _ratio(r["achieved_gbps"], HBM_PEAK_GBPS), "traffic": traffic, "traffic_source": src,
           "launch_ms": r["unproject_ms"], "algorithmic_bytes_per_launch": r["launch_bytes"]}
    if device is not None:
        cp = copy_bandwidth(device)
        out.update(measured_copy_gbps=cp, frac_of_measured_copy=_ratio(r["achieved_gbps"], cp))
    return out


# ----------------------------------------------------------------------------- workloads
class Workload:
    """One rank's frames of a config, resident on the device, and the timed step."""

    def __init__(self, cfg, rank, world, device, seed=0, cuboid=False, first_frame=None, global_batch=None,
                 precision="exact"):
        import torch
        from mvn_rocm import synth
        self.cfg, self.world, self.device = cfg, world, device
        self.precision = precision      # the unprojection's arithmetic
        B = cfg["frames"]
        # ragged strong-scaling shards (config 4 over N not dividing 128): the caller passes the
        # true global batch, or ranks would pad the joints all-gather to different sizes
        self.global_batch = B * world if global_batch is None else global_batch
        first = rank * B if first_frame is None else first_frame
        vb = synth.volumetric_batch(B, n_views=cfg["views"], channels=cfg["channels"], heatmap=cfg["heatmap"],
                                    volume=cfg["volume"], dtype=cfg["dtype"], device=device, seed=seed,
                                    first_frame=first)
        self.feat, self.proj, self.coords = vb.features, vb.proj, vb.coords
        if cuboid:      # coordinates formed inside both kernels (mvn_*_cuboid), never materialised
            self.coords = vb.cuboids(device)
        self.ev = []
        self._pool = []
        self.last = None
        self.gathered = None
        self.starts = None      # first frame of every rank's shard (set by the caller)

    def reserve_events(self, n, stride=4):
        """Pre-create the timing events of n timed steps, so that no Event is constructed
        inside the timed region (only recorded).  Every `stride`-th timed step (steps stride-1,
        2 stride-1, ...) records three events — before and after its unprojection and after its
        soft-argmax; 0 = no events (no kernel times).  Recording costs GPU time: with events on
        every step config 2's step took 233.9-234.5 us against 225.7-226.4 us without
        (profiles/r21_timing_events_ab.txt), so the kernels are timed on a sample of the steps
        spread over the whole timed region."""
        import torch
        if 0 < n < stride:          # short timed regions: at least the last step
            stride = n
        self.stride, self.nstep = stride, 0
        n = 0 if stride <= 0 else n // stride
        self._pool = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(n)]
        # torch creates the HIP event lazily, at its first record(): record each once now, or the
        # timed region pays 3 hipEventCreate per step (~180 us over the driver's 20 steps, r17)
        for trio in self._pool:
            for e in trio:
                e.record()
        torch.cuda.synchronize()
        self.ev = []

    def step(self, timed=False, gather=True):
        from mvn_rocm import dist as mdist, op
        J = self.cfg["joints"]
        if timed:
            # the last step of every stride (the first timed step follows the fence's idle GPU)
            sample = self.stride > 0 and self.nstep % self.stride == self.stride - 1
            self.nstep += 1
            timed = sample
        if timed:
            e0, e1, e2 = self._pool[len(self.ev)]
            e0.record()
        vol = op.unproject_heatmaps(self.feat, self.proj, self.coords, "softmax", precision=self.precision)
        if timed:
            e1.record()
        xyz, sm = op.integrate_tensor_3d_with_coordinates(vol[:, :J], self.coords, True)
        if timed:
            e2.record()
            self.ev.append((e0, e1, e2))
        self.last = (vol, xyz)
        if self.world > 1 and gather:   # the path's one exchange: joints of every rank, RCCL over xGMI
            xyz = mdist.gather_joints(xyz, self.global_batch)
            self.gathered = xyz
        return xyz, sm

    def kernel_ms(self):
        """(unprojection, soft-argmax) mean ms over the sampled timed steps."""
        import torch
        torch.cuda.synchronize()
        n = len(self.ev)
        if n == 0:
            return None, None
        return (sum(a.elapsed_time(b) for a, b, _ in self.ev) / n, sum(b.elapsed_time(c) for _, b, c in self.ev) / n)


def run_config(name, args, rank, world, device, clock, cuboid=False, cfg=None, first_frame=None, starts=None,
               global_batch=None, precision=None):
    import torch
    cfg = cfg if cfg is not None else _configs()[name]
    precision = precision or args.precision
    wl = Workload(cfg, rank, world, device, cuboid=cuboid, first_frame=first_frame, global_batch=global_batch,
                  precision=precision)
    wl.starts = starts if starts is not None else [r * cfg["frames"] for r in range(world)]
    wl.reserve_events(args.steps, args.event_stride)
    elapsed = timed_loop(lambda t: wl.step(t), args, clock)
    E = 2 if cfg["dtype"] == torch.bfloat16 else 4
    frames_total = wl.global_batch * args.steps
    unproj_ms, sa_ms = wl.kernel_ms()
    # every rank samples its own GPU (the line carries the per-rank list at world > 1); the burst
    # runs each rank's local step only — a rank-dependent count of collectives would deadlock
    tel = telemetry(device, lambda t: wl.step(t, gather=False))
    launch_bytes = unproject_bytes(cfg, E, cuboid) * cfg["frames"]
    return dict(cfg=cfg, workload=wl, precision=precision, elapsed=elapsed, fps=frames_total / elapsed,
                ms_per_step=elapsed / args.steps * 1e3,
                unproject_ms=unproj_ms, softargmax_ms=sa_ms, launch_bytes=launch_bytes,
                achieved_gbps=(launch_bytes / (unproj_ms * 1e-3) / 1e9) if unproj_ms else None,
                path_gbps=frame_bytes(cfg, E, cuboid) * frames_total / elapsed / 1e9, telemetry=tel)


def run_config5(args, rank, world, device, clock, cuboid=False):
    """Config 5: unproject (softmax, written channels-last bf16) + V2V front block on MFMA;
    roofline of the front block against the bf16 dense MFMA peak."""
    import torch
    from mvn_rocm import synth, v2v
    cfg = _configs()["5"]
    B = cfg["frames"]
    vb = synth.volumetric_batch(B, n_views=cfg["views"], channels=cfg["channels"], heatmap=cfg["heatmap"],
                                volume=cfg["volume"], dtype=cfg["dtype"], device=device, seed=0, first_frame=rank * B)
    g = torch.Generator().manual_seed(0)
    w = torch.randn((16, 32, 7, 7, 7), generator=g) * 0.02
    packed, scale, shift = v2v.fold_basic3d_block(w, torch.randn(16, generator=g) * 0.1, torch.rand(16, generator=g) + 0.5,
                                                  torch.randn(16, generator=g) * 0.1, torch.zeros(16), torch.ones(16),
                                                  device=device)
    ev = []
    last = []
    coords = vb.cuboids(device) if cuboid else vb.coords
    # timing events created (first record) before the timed region, as Workload.reserve_events
    pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in pool:
        a.record()
        b.record()
    torch.cuda.synchronize()

    def step(timed=False):
        cl = v2v.unproject_channels_last(vb.features, vb.proj, coords, "softmax")
        if timed:
            e0, e1 = pool[len(ev)]
            e0.record()
        y = v2v.v2v_front(cl, packed, scale, shift, torch.bfloat16)
        if timed:
            e1.record()
            ev.append((e0, e1))
        last[:] = [cl, y]
        return y

    elapsed = timed_loop(step, args, clock)
    conv_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    tflops = V2V_FLOP_PER_FRAME * B / (conv_ms * 1e-3) / 1e12
    # the same work through the one-call pipeline (mvn_unproject_v2v_front: frame groups of 8
    # through a 134 MB workspace instead of the 1.07 GB whole-batch intermediate)
    one = timed_loop(lambda t: v2v.unproject_v2v_front(vb.features, vb.proj, coords, packed, scale, shift, "softmax",
                                                       torch.bfloat16), args, clock)
    # telemetry after BOTH timed loops: its burst of extra GPU work (this config runs at the
    # package power limit) would otherwise heat the chip between them
    tel = telemetry(device, step)
    pin = None if cuboid else dict(feat=vb.features, proj=vb.proj, coords=vb.coords, last=tuple(last),
                                   w_bf16=w.bfloat16().float(), scale=scale, shift=shift)
    return dict(parity_inputs=pin, workload=cfg["label"], value=B * world * args.steps / elapsed, unit="frames/s",
                one_call={"value": B * world * args.steps / one, "ms_per_step": one / args.steps * 1e3,
                          "api": "mvn_unproject_v2v_front (groups of 8 frames, MALL-resident intermediate)"},
                ms_per_step=elapsed / args.steps * 1e3, frames_per_gpu=B, dtype="bf16", telemetry=tel,
                roofline={"kernel": "v2v_front<bf16> (Conv3d 32->16 k7 + BN + ReLU)", "bound": "mfma",
                          "achieved": tflops, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / MFMA_BF16_PEAK_TFLOPS, "launch_ms": conv_ms,
                          "flop_per_launch": V2V_FLOP_PER_FRAME * B,
                          # the dense peak is quoted at 2.4 GHz; bf16 MFMA loads hold a lower
                          # clock (MI355X_MICROARCH.md 'DVFS give-back'): the fraction of the
                          # peak at the sclk this config held (telemetry), an MFMA-pipe figure
                          "frac_at_held_clock": (tflops / (MFMA_BF16_PEAK_TFLOPS * tel["sclk_mhz"] / 2400.0)
                                                 if tel and tel.get("sclk_mhz") else None)})


def run_config1(args, device):
    """BASELINE config 1, the algebraic path at batch 1 (4 views x 17 joints): the DLT alone
    (triangulate_batch_of_points, multiview.py:162-174) and the model's chain from heatmaps
    (triangulation.py:164-191): 2D soft-argmax of heatmaps * 100 -> confidence
    normalisation -> upscale to image pixels -> DLT.  Device time from HIP events around
    100 back-to-back calls; wall time per call includes the host launch."""
    import torch
    from mvn_rocm import multiview, op, synth
    ab = synth.algebraic_batch(1, 4, 17, seed=0)
    P, pts, conf = ab.proj.to(device), ab.points.to(device), ab.confidences.to(device)
    hm = torch.randn((4, 17, 96, 96), generator=torch.Generator().manual_seed(1)).to(device)
    raw_conf = torch.rand((1, 4, 17), generator=torch.Generator().manual_seed(2)).to(device) + 0.1

    def dlt():
        return multiview.triangulate_batch_of_points(P, pts, conf)

    def chain():
        xy, _ = op.integrate_tensor_2d(hm, True, multiplier=100.0, return_heatmaps=False)
        xy = xy.view(1, 4, 17, 2) * 4.0                      # 384 / 96, both axes
        c = raw_conf / raw_conf.sum(dim=1, keepdim=True) + 1e-5
        return multiview.triangulate_batch_of_points(P, xy, c)

    res = {}
    for name, fn in (("dlt", dlt), ("chain", chain)):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = max(100, args.steps)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = (e0.elapsed_time(e1) / n * 1e3, (time.perf_counter() - t0) / n * 1e6)
    return dict(workload="cfg1: algebraic DLT (triangulate_batch_of_points), 4 views x 17 joints, batch 1, f32 in, "
                         "f64 null-vector solve",
                dlt_device_us=res["dlt"][0], dlt_wall_us=res["dlt"][1], value=1e6 / res["dlt"][1],
                unit="frames/s (batch 1, host-launch inclusive)",
                chain_workload="integrate_tensor_2d(heatmaps x100, 4x17x96^2) -> conf norm -> upscale -> DLT",
                chain_device_us=res["chain"][0], chain_wall_us=res["chain"][1])


# ----------------------------------------------------------------------------- CPU baseline
def _host_cores():
    """(physical cores, logical CPUs) of the host from lscpu, or (None, os.cpu_count())."""
    try:
        out = subprocess.run(["lscpu", "-p=CORE,SOCKET"], capture_output=True, text=True, timeout=10).stdout
        cores = {ln for ln in out.splitlines() if ln and not ln.startswith("#")}
        return (len(cores) or None), os.cpu_count()
    except (OSError, subprocess.SubprocessError):
        return None, os.cpu_count()


def cpu_baseline(budget_s=8.0):
    """The reference algorithm restated op-for-op in torch-CPU (oracle/restate_torch.py,
    pinned bit-exact to the reference by tests/test_oracle.py), timed on this host at the
    config-2 batch of 8 frames: with every thread torch uses here, and with one thread;
    plus config 1 (DLT, batch 1).  Bounded sample: whole batches until `budget_s` per leg."""
    import warnings

    import torch
    from mvn_rocm import synth
    from oracle import restate_torch
    warnings.filterwarnings("ignore")
    cfg = _configs()["2"]
    vb = synth.volumetric_batch(cfg["frames"], seed=0)

    def batches(budget):
        n, t0 = 0, time.perf_counter()
        while True:
            vol = restate_torch.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
            restate_torch.integrate_tensor_3d_with_coordinates(vol[:, :cfg["joints"]], vb.coords, True)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return n, el

    threads = torch.get_num_threads()
    n_all, el_all = batches(budget_s)
    torch.set_num_threads(1)
    n_one, el_one = batches(0.0)                     # one batch (~8x the all-thread time)
    ab = synth.algebraic_batch(1, 4, 17, seed=0)
    nd, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        restate_torch.triangulate_batch_of_points(ab.proj, ab.points, ab.confidences)
        nd += 1
    dlt_ms = (time.perf_counter() - t0) / nd * 1e3
    torch.set_num_threads(threads)
    phys, logical = _host_cores()
    B = cfg["frames"]
    return dict(value=n_all * B / el_all, unit="frames/s", cores=threads, kind="port",
                sample=f"{n_all} batch(es) of {B} frames of config 2 (4x32x96^2 -> 64^3, softmax agg, 17-joint "
                       f"soft-argmax, fp32) through oracle/restate_torch.py (op-for-op restatement of "
                       f"op.py:84-163, bit-exact with the reference) in {el_all:.1f} s, {threads} threads",
                threads_1=dict(value=n_one * B / el_one, unit="frames/s", cores=1,
                               sample=f"{n_one} batch(es) of {B} frames in {el_one:.1f} s, 1 thread"),
                host_physical_cores=phys, host_logical_cpus=logical,
                threads_policy=(f"{threads} threads = this job's CPU share on the GPU box (the pool sets "
                                f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', '?')} per GPU and asks jobs "
                                f"not to exceed it); SURVEY.md §8d's os.cpu_count() ({logical}) counts the whole "
                                f"shared host, which this job may not occupy"),
                config1_dlt_ms_per_frame=dlt_ms,
                config1_sample=f"{nd} calls of restate_torch.triangulate_batch_of_points (multiview.py:132-174), "
                               f"batch 1, 4 views x 17 joints, {threads} threads")


def _rel(a, b):
    import numpy as np
    return float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def _within_one_bf16_ulp(got, ref, slack):
    """Every value of a bf16 result within one bf16 ulp of the f32 reference (+ `slack` x
    max|ref| absolute, where the f32 value cancels towards 0)."""
    import numpy as np
    ref = ref.astype(np.float64)
    _, e = np.frexp(ref)
    ulp = np.where(ref == 0, 0.0, np.ldexp(1.0, e - 8))
    return bool((np.abs(got.astype(np.float64) - ref) <= ulp + slack * np.abs(ref).max()).all())


def _frames(n):
    """Frames of an n-frame launch the parity check recomputes: the first and the last (the
    last frame's addresses are the launch's largest; at config 4's 128 frames its output
    lies past 2^32 bytes)."""
    return sorted({0, n - 1})


def _np_feat(t):
    import numpy as np
    import torch
    t = t.cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def _within_fast_bar(got, ref):
    """The fast mode's bar for a bf16 volume of the bench's softmax step:
    one bf16 ulp of the f32 oracle + 2^-7 x max|ref| (bf16 bilinear weights, which the view
    softmax puts in the exponent; tests/test_gpu_fast.py's softmax bar)."""
    return _within_one_bf16_ulp(got, ref, 2.0 ** -7)


def parity_unproject(feat, proj, coords, vol, J, frames, xyz=None, layout="ncdhw", precision="exact"):
    """Frames `frames` of a timed unprojection (softmax agg) against the C oracle
    (oracle/mvn_oracle.c, pinned to the reference's goldens) on the same inputs.
      unproject_max_rel    GPU volume vs oracle unproject_heatmaps (op.py:99-163):
                           max|d| / max|ref| over the frame's C x V^3 values
      joints_max_rel       GPU joints vs the oracle soft-argmax (op.py:84-96) of the GPU's own
                           channels [0:J] (the same input the GPU's soft-argmax saw)
      chain_joints_max_rel GPU joints vs the oracle chain unproject -> soft-argmax end to end
    bf16 maps: the oracle runs in f32 on the same bf16 bits; a bf16 volume is checked to be
    within one bf16 ulp of it.  Worst value over the frames."""
    import numpy as np
    import torch
    from oracle import capi
    out = dict(frames_checked=list(frames), unproject_max_rel=0.0)
    bf16 = feat.dtype == torch.bfloat16
    for f in frames:
        fe = _np_feat(feat[f:f + 1])
        pr, co = proj[f:f + 1].cpu().numpy(), coords[f:f + 1].cpu().numpy()
        ref_vol = capi.unproject(fe, pr, co, "softmax", feat_bf16_bits=bf16)
        got = vol[f:f + 1]
        if layout == "ndhwc":
            got = got.permute(0, 4, 1, 2, 3)
        got_vol = got.float().cpu().numpy()
        out["unproject_max_rel"] = max(out["unproject_max_rel"], _rel(got_vol, ref_vol))
        if vol.dtype == torch.bfloat16 and precision == "exact":
            ok = _within_one_bf16_ulp(got_vol, ref_vol, 1e-5)
            out["unproject_within_one_bf16_ulp"] = out.get("unproject_within_one_bf16_ulp", True) and ok
        elif vol.dtype == torch.bfloat16:
            ok = _within_fast_bar(got_vol, ref_vol)
            out["unproject_within_fast_bar"] = out.get("unproject_within_fast_bar", True) and ok
        if xyz is not None:
            got_xyz = xyz[f:f + 1].cpu().numpy().astype(np.float64)
            own_xyz, _ = capi.softargmax3d(np.ascontiguousarray(got_vol[:, :J]), co, True, 1.0)
            ref_xyz, _ = capi.softargmax3d(np.ascontiguousarray(ref_vol[:, :J]), co, True, 1.0)
            out["joints_max_rel"] = max(out.get("joints_max_rel", 0.0), _rel(got_xyz, own_xyz))
            out["chain_joints_max_rel"] = max(out.get("chain_joints_max_rel", 0.0), _rel(got_xyz, ref_xyz))
    return out


def parity_check(res):
    """Parity of a timed workload itself (SURVEY.md §5 'Metrics': the line carries the parity
    error): the first and the last frame of the last timed step, recomputed by the C oracle
    on the same inputs (parity_unproject).  The oracle is the checker only: this runs after
    the timed regions and nothing it computes enters a timed number."""
    wl = res["workload"]
    vol, xyz = wl.last
    t0 = time.perf_counter()
    out = parity_unproject(wl.feat, wl.proj, wl.coords, vol, wl.cfg["joints"], _frames(vol.shape[0]), xyz,
                           precision=wl.precision)
    bars = ("unproject <= 1e-5 (f32 out) / one bf16 ulp (bf16 out); joints <= 1e-4 (north_star)"
            if wl.precision == "exact" else
            "fast mode: unproject <= 1e-4 (f32 maps, north_star's bound) / one bf16 ulp + 2^-7 max|ref| (bf16 maps, softmax); "
            "chain joints <= 1e-4 (north_star)")
    return dict(out, precision=wl.precision, bars=bars, oracle="oracle/mvn_oracle.c via oracle/capi.py",
                oracle_s=time.perf_counter() - t0)


def parity_check5(r5):
    """Config 5's timed outputs, first and last frame: the channels-last bf16 unprojection
    against the C oracle (within one bf16 ulp), and the V2V front block (bf16 out) against
    torch's CPU conv3d on the same bf16 operands (the GPU's own unprojection and the
    bf16-rounded weights, f32 math) + the folded BatchNorm + ReLU (v2v.py:7-17): within one
    bf16 ulp + 1e-4 x max|ref|."""
    import torch
    import torch.nn.functional as F
    p = r5["parity_inputs"]
    cl, y = p["last"]
    frames = _frames(cl.shape[0])
    t0 = time.perf_counter()
    out = parity_unproject(p["feat"], p["proj"], p["coords"], cl, 0, frames, layout="ndhwc")
    w, sc, sh = p["w_bf16"], p["scale"].cpu().view(1, -1, 1, 1, 1), p["shift"].cpu().view(1, -1, 1, 1, 1)
    conv_rel, conv_ok = 0.0, True
    for f in frames:
        x = cl[f:f + 1].permute(0, 4, 1, 2, 3).float().cpu()
        ref = torch.relu(F.conv3d(x, w, None, padding=3) * sc + sh).numpy()
        got = y[f:f + 1].float().cpu().numpy()
        conv_rel = max(conv_rel, _rel(got, ref))
        conv_ok = conv_ok and _within_one_bf16_ulp(got, ref, 1e-4)
    return dict(out, v2v_front_max_rel=conv_rel, v2v_front_within_one_bf16_ulp_plus_1e4=conv_ok,
                bars="unproject one bf16 ulp; v2v front one bf16 ulp + 1e-4 x max|ref| vs torch-CPU conv3d",
                oracle="oracle/mvn_oracle.c via oracle/capi.py; torch.nn.functional.conv3d (CPU, f32)",
                oracle_s=time.perf_counter() - t0)


def verify_gather(res):
    """world > 1: the gathered joints of the last timed step (RCCL all-gather) against the
    first frame of every rank's shard recomputed on rank 0 from (seed, global frame index):
    bit for bit (frames are independent in every kernel, so a frame's joints do not depend on
    the batch it ran in).  Run after every timed region."""
    import torch
    from mvn_rocm import op, synth
    wl = res["workload"]
    c, got = wl.cfg, wl.gathered
    if got is None:
        return None
    checked, ok = [], True
    for start in wl.starts:
        vb = synth.volumetric_batch(1, n_views=c["views"], channels=c["channels"], heatmap=c["heatmap"],
                                    volume=c["volume"], dtype=c["dtype"], device=wl.device, seed=0, first_frame=start)
        vol = op.unproject_heatmaps(vb.features, vb.proj, vb.coords, "softmax")
        xyz, _ = op.integrate_tensor_3d_with_coordinates(vol[:, :c["joints"]], vb.coords, True)
        ok = ok and bool(torch.equal(xyz[0], got[start]))
        checked.append(start)
    return dict(gather_verified=ok, frames_recomputed=checked)


# ----------------------------------------------------------------------------- dry run (CPU)
def dry_run(args, rank, world):
    """The multi-rank protocol of the bench on the CPU (gloo): every rank builds its own
    frames from (seed, global frame index), a stand-in step (the mean of each frame's
    coordinate volume as 17 'joints') and the joints all-gather; rank 0 checks the gathered
    joints against all frames built locally.  Two legs, as the GPU line: config 2's weak
    scaling (8 frames per rank) and config 4's strong scaling (a global batch of 128 split
    over the ranks, ragged when the world does not divide it).  The line carries the same
    `dist` block (backend, every rank's identity) as a GPU line."""
    import torch
    import torch.distributed as dist
    from mvn_rocm import dist as mdist, synth
    B = 8
    G = B * world

    def joints(first, count):
        vb = synth.volumetric_batch(count, n_views=4, channels=1, heatmap=8, volume=4, seed=0, first_frame=first)
        return vb.coords.reshape(count, -1, 3).mean(1, keepdim=True).expand(count, 17, 3).contiguous()

    local = joints(rank * B, B)
    clock = Clock(world, torch.device("cpu"), True)

    def step(_timed):
        return mdist.gather_joints(local, G) if world > 1 else local

    elapsed = timed_loop(step, args, clock)
    got = step(False)
    ok = bool(torch.equal(got, joints(0, G))) if rank == 0 else None

    # config 4's shape: 128 frames split over the ranks
    G4 = 128
    start, count = mdist.shard(G4, world, rank)
    local4 = joints(start, count)

    def step4(_timed):
        return mdist.gather_joints(local4, G4) if world > 1 else local4

    el4 = timed_loop(step4, args, clock)
    got4 = step4(False)
    shards = gather_objects([start, count], world)
    ok4 = None
    if rank == 0:
        ok4 = bool(torch.equal(got4, joints(0, G4)))
        # and every shard's first frame recomputed alone (verify_gather's check)
        ok4 = ok4 and all(bool(torch.equal(got4[s0], joints(s0, 1)[0])) for s0, _ in shards)
    ident = rank_identity(None, rank, int(os.environ.get("LOCAL_RANK", rank)), True)
    drec = dist_record(ident, world, dist.get_backend() if world > 1 else None)
    return dict(metric=METRIC, value=G * args.steps / elapsed, unit="frames/s", n_gpus=world, steps=args.steps,
                warmup=args.warmup, ms_per_step=elapsed / args.steps * 1e3, higher_is_better=True, scaling="weak",
                vs_baseline=None, dtype="f32", data="dry run: CPU/gloo protocol check, stand-in step (no HIP)",
                dry_run=True, gather_verified=ok, dist=drec,
                config={"workload": "dry run of the config-2 sharding", "global_batch": G, "frames_per_gpu": B,
                        "parallelism": f"dp{world}", "collective": "all_gather joints (gloo)" if world > 1 else None},
                config4={"workload": "dry run of the config-4 sharding (128 frames split over the ranks)",
                         "global_batch": G4, "value": G4 * args.steps / el4, "scaling": "strong",
                         "shards": shards, "gather": {"gather_verified": ok4,
                                                      "frames_recomputed": [s0 for s0, _ in shards]}})


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle", type=float, default=1.0,
                    help="seconds of untimed steps before the warmup, per config (GPU clock ramp from idle)")
    ap.add_argument("--config", default="2", choices=["2", "3", "4"])
    ap.add_argument("--precision", default="exact", choices=["exact", "fast"],
                    help="the unprojection arithmetic of the headline and its secondary configs (DESIGN.md §4.1a); "
                         "the other arithmetic is reported beside them")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--event-stride", type=int, default=4,
                    help="kernel times from HIP events on every K-th timed step (events cost GPU time; "
                         "1 = every step, 0 = none)")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-in-kernel-coords", action="store_true",
                    help="skip the in-kernel-coordinates run (keeps rocprof kernel means per variant clean)")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo protocol check, no GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="(tests) gloo runs the multi-rank protocol with host-side collectives, e.g. several "
                         "ranks sharing one GPU (RCCL refuses two ranks on one device)")
    ap.add_argument("--share-device", action="store_true",
                    help="(tests, with --dist-backend gloo) every rank computes on cuda:0")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1,
                    help="(tests) this rank of a dry run exits with an error before its first barrier")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        if rank == args.dry_run_fail_rank:
            raise SystemExit(f"rank {rank}: failing on request (--dry-run-fail-rank)")
        line = dry_run(args, rank, world)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    if args.share_device and args.dist_backend != "gloo":
        raise SystemExit("--share-device needs --dist-backend gloo (RCCL refuses two ranks on one GPU)")
    device = torch.device("cuda", 0 if args.share_device else local)
    torch.cuda.set_device(device)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    clock = Clock(world, device, False, host_collectives=args.dist_backend == "gloo")
    coll = (f"all_gather joints ({'RCCL' if args.dist_backend == 'nccl' else 'gloo, host tensors'})"
            if world > 1 else None)
    configs = _configs()
    extras = not args.no_secondary and args.config == "2"

    main_res = run_config(args.config, args, rank, world, device, clock)
    secondary = config1 = in_kernel_coords = cfg4 = cfg5 = sec_res = None
    if extras:
        s = sec_res = run_config("3", args, rank, world, device, clock)
        secondary = dict(workload=s["cfg"]["label"], value=s["fps"], unit="frames/s", ms_per_step=s["ms_per_step"],
                         frames_per_gpu=s["cfg"]["frames"], dtype="bf16", unproject_ms=s["unproject_ms"],
                         softargmax_ms=s["softargmax_ms"], roofline=roofline(s["cfg"], s, "3", device),
                         path_algorithmic_gbps=s["path_gbps"], path_frac=s["path_gbps"] / HBM_PEAK_GBPS,
                         telemetry=s["telemetry"])
    other = other_res = None
    if extras:
        # the other unprojection arithmetic on configs 2 and 3, same protocol
        alt = "fast" if args.precision == "exact" else "exact"
        other_res = {"2": run_config("2", args, rank, world, device, clock, precision=alt),
                     "3": run_config("3", args, rank, world, device, clock, precision=alt)}
        other = {"precision": alt}
        for cn, o in other_res.items():
            other[f"config{cn}"] = dict(workload=o["cfg"]["label"], value=o["fps"], unit="frames/s",
                                        ms_per_step=o["ms_per_step"], unproject_ms=o["unproject_ms"],
                                        softargmax_ms=o["softargmax_ms"], roofline=roofline(o["cfg"], o, cn, device),
                                        path_algorithmic_gbps=o["path_gbps"],
                                        path_frac=o["path_gbps"] / HBM_PEAK_GBPS, telemetry=o["telemetry"])
    if not args.no_secondary and not args.no_in_kernel_coords:
        # the same workload with the coordinate volume formed inside both kernels from the
        # per-frame cuboids instead of read from HBM
        k = run_config(args.config, args, rank, world, device, clock, cuboid=True)
        in_kernel_coords = dict(workload=k["cfg"]["label"] + ", coordinates formed in-kernel from per-frame cuboids",
                                value=k["fps"], unit="frames/s", ms_per_step=k["ms_per_step"],
                                unproject_ms=k["unproject_ms"], unproject_algorithmic_bytes_per_launch=k["launch_bytes"],
                                unproject_achieved_gbps=k["achieved_gbps"],
                                unproject_frac=_ratio(k["achieved_gbps"], HBM_PEAK_GBPS),
                                path_algorithmic_gbps=k["path_gbps"])
    if extras:
        # BASELINE config 4: 8 views, a global batch of 128 frames split over the ranks
        # (strong scaling), joints all-gathered over RCCL inside the timed step
        from mvn_rocm import dist as mdist
        start, count = mdist.shard(128, world, rank)
        c4 = dict(configs["4"], frames=count)
        r4 = run_config("4", args, rank, world, device, clock, cfg=c4, first_frame=start,
                        starts=[mdist.shard(128, world, q)[0] for q in range(world)], global_batch=128)
        cfg4 = dict(workload=c4["label"] + ", global batch 128 split over the ranks", value=128 * args.steps / r4["elapsed"],
                    unit="frames/s", scaling="strong", global_batch=128, frames_per_gpu=count,
                    ms_per_step=r4["ms_per_step"], unproject_ms=r4["unproject_ms"],
                    unproject_achieved_gbps=r4["achieved_gbps"], unproject_frac=_ratio(r4["achieved_gbps"], HBM_PEAK_GBPS),
                    collective=coll, telemetry=r4["telemetry"])
        cfg5 = run_config5(args, rank, world, device, clock)
        if not args.no_in_kernel_coords:
            k5 = run_config5(args, rank, world, device, clock, cuboid=True)
            cfg5["in_kernel_coords"] = dict(value=k5["value"], unit="frames/s", ms_per_step=k5["ms_per_step"])
        if rank == 0:
            config1 = run_config1(args, device)
    base = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU leg: the reference algorithm timed on the host, and the timed workloads'
        # outputs checked against the oracle (never inside a timed region)
        base = cpu_baseline()
        parity = parity_check(main_res)
        if secondary is not None:
            secondary["parity"] = parity_check(sec_res)
        if cfg4 is not None:
            cfg4["parity"] = parity_check(r4)
        if cfg5 is not None and cfg5.get("parity_inputs") is not None:
            cfg5["parity"] = parity_check5(cfg5)
        if other is not None:
            for cn, o in other_res.items():
                other[f"config{cn}"]["parity"] = parity_check(o)
    if cfg5 is not None:
        cfg5.pop("parity_inputs", None)
    gather = None
    if rank == 0 and world > 1:
        gather = verify_gather(main_res)
        if cfg4 is not None:
            cfg4["gather"] = verify_gather(r4)
        # rank 0's own shard of the timed outputs against the oracle (the checker, after
        # every timed region), so that a multi-GPU line carries parity too
        if not args.no_cpu_baseline:
            parity = parity_check(main_res)
            if cfg4 is not None:
                cfg4["parity"] = parity_check(r4)
    # the self-proving multi-rank record: backend, every rank's device, per-rank telemetry
    drec = dist_record(rank_identity(device, rank, local, False), world,
                       (dist.get_backend() if world > 1 else None))
    tel_ranks = gather_objects(main_res["telemetry"], world) if world > 1 else None
    tel4_ranks = gather_objects(r4["telemetry"], world) if (world > 1 and cfg4 is not None) else None
    if cfg4 is not None:
        cfg4["telemetry_per_rank"] = tel4_ranks

    if rank == 0:
        r, c = main_res, main_res["cfg"]
        line = {
            "metric": METRIC,
            "value": r["fps"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_s": args.settle,
            "ms_per_step": r["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype_name(c["dtype"]),
            "data": "synthetic (seeded ring cameras, N(0,1) features, rotated 2.5 m cuboids; SURVEY.md §8d)",
            "config": {"workload": c["label"], "global_batch": c["frames"] * world, "frames_per_gpu": c["frames"],
                       "views": c["views"], "channels": c["channels"], "heatmap": c["heatmap"],
                       "volume": c["volume"], "joints": c["joints"], "parallelism": f"dp{world}",
                       "collective": coll, **({"device_shared": True} if args.share_device else {})},
            "roofline": roofline(c, r, args.config, device),
            "softargmax_ms": r["softargmax_ms"],
            "path_algorithmic_gbps": r["path_gbps"],
            "path_frac": r["path_gbps"] / HBM_PEAK_GBPS,
            "telemetry": r["telemetry"],
            "telemetry_per_rank": tel_ranks,
            "gpu": gpu_identity(device),
            "dist": drec,
            "cpu_baseline": base,
            "parity": parity,
            "gather": gather,
            "precision": args.precision,
            "secondary": secondary,
            "other_precision": other,
            "config1": config1,
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
