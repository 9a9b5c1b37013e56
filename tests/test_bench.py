"""bench.py's process model on the CPU: `--gpus N` with no WORLD_SIZE spawns N rank
processes itself (torchrun-style environment), and the dry run exercises the ranks'
barriers, max-over-ranks timing and the joints all-gather over gloo."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", (1, 2, 3))
def test_bench_spawns_the_ranks(gpus):
    line = _bench("--gpus", str(gpus), "--dry-run", "--steps", "3", "--warmup", "1")
    assert line["n_gpus"] == gpus
    assert line["config"]["global_batch"] == 8 * gpus and line["config"]["parallelism"] == f"dp{gpus}"
    assert line["gather_verified"] is True       # gathered joints == every frame built on rank 0
    assert line["steps"] == 3 and line["warmup"] == 1 and line["value"] > 0


@pytest.mark.parametrize("gpus", (5, 8))
def test_bench_dry_run_config4_shards_and_dist_record(gpus):
    """the multi-rank line proves itself — backend, every rank's identity,
    one entry per rank — and config 4's 128 frames split over a ragged (5) or even (8) world
    are gathered in frame order, every shard's first frame recomputed on rank 0."""
    line = _bench("--gpus", str(gpus), "--dry-run", "--steps", "2", "--warmup", "1", timeout=420)
    d = line["dist"]
    assert d["backend"] == "gloo" and d["world"] == gpus
    assert [r["rank"] for r in d["ranks"]] == list(range(gpus))
    assert [r["local_rank"] for r in d["ranks"]] == list(range(gpus))
    assert len({r["pid"] for r in d["ranks"]}) == gpus
    c4 = line["config4"]
    assert c4["global_batch"] == 128 and c4["scaling"] == "strong"
    counts = [c for _, c in c4["shards"]]
    assert sum(counts) == 128 and max(counts) - min(counts) <= 1
    assert [s for s, _ in c4["shards"]] == [sum(counts[:r]) for r in range(gpus)]
    assert c4["gather"]["gather_verified"] is True
    assert c4["gather"]["frames_recomputed"] == [s for s, _ in c4["shards"]]
    assert line["gather_verified"] is True


def test_bench_a_failing_rank_ends_the_job():
    """Rank 1 dies before the first barrier (--dry-run-fail-rank): the launcher sees it while
    rank 0 is still blocked in the barrier, terminates rank 0 and exits non-zero — instead of
    waiting on rank 0 forever."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--dry-run-fail-rank", "1"], capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def _verify_worker(rank, world, port, out_path):
    """One rank of a world-2 gloo job: its shard's joints (stand-in ops: the C oracle) are
    all-gathered, then rank 0 runs bench.verify_gather — the check a multi-GPU bench line
    carries as `gather` — against the true gather and against one with a corrupted frame."""
    import numpy as np
    import torch
    import torch.distributed as dist
    for p in (ROOT, os.path.join(ROOT, "learnable-triangulation-pytorch_amd")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from mvn_rocm import dist as mdist, op, synth
    from oracle import capi

    def unproject(feat, proj, coords, agg):          # stand-ins on the CPU: the C oracle
        return torch.from_numpy(capi.unproject(feat.numpy(), proj.numpy(), coords.numpy(), agg))

    def softargmax(vol, coords, softmax=True):
        xyz, sm = capi.softargmax3d(np.ascontiguousarray(vol.numpy()), coords.numpy(), softmax, 1.0)
        return torch.from_numpy(xyz), torch.from_numpy(sm)

    op.unproject_heatmaps, op.integrate_tensor_3d_with_coordinates = unproject, softargmax
    cfg = dict(frames=3, views=3, channels=4, heatmap=16, volume=8, joints=3, dtype=torch.float32)
    G = 5
    start, count = mdist.shard(G, world, rank)
    vb = synth.volumetric_batch(count, n_views=3, channels=4, heatmap=16, volume=8, seed=0, first_frame=start)
    xyz, _ = softargmax(unproject(vb.features, vb.proj, vb.coords, "softmax")[:, :3], vb.coords)
    gathered = mdist.gather_joints(xyz.contiguous(), G)

    class WL:
        pass
    wl = WL()
    wl.cfg, wl.device, wl.gathered = cfg, torch.device("cpu"), gathered
    wl.starts = [mdist.shard(G, world, q)[0] for q in range(world)]
    if rank == 0:
        good = bench.verify_gather({"workload": wl})
        wl.gathered = gathered.clone()
        wl.gathered[wl.starts[-1], 0, 0] += 1.0
        bad = bench.verify_gather({"workload": wl})
        with open(out_path, "w") as f:
            json.dump([good, bad], f)
    dist.barrier()
    dist.destroy_process_group()


def test_verify_gather_world2(tmp_path):
    """bench.verify_gather: at world 2 over gloo, rank 0 recomputes the
    first frame of every shard and compares it bit for bit with the all-gathered joints."""
    import socket

    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "verify.json")
    mp.spawn(_verify_worker, args=(2, port, out), nprocs=2, join=True)
    good, bad = json.load(open(out))
    assert good == {"gather_verified": True, "frames_recomputed": [0, 3]}
    assert bad["gather_verified"] is False
