"""Multi-process (gloo, CPU) tests of the frame-sharded path: the gathered joints of a
sharded run equal a single-process run bit-for-bit (frames are independent).  The
per-rank compute here is the CPU oracle; on the GPU box the same driver runs the HIP
ops over RCCL (bench.py --gpus N)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

GLOBAL_B = 5           # ragged over 2 ranks: 3 + 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames(start, count):
    from mvn_rocm import synth
    vb = synth.volumetric_batch(count, n_views=3, channels=4, heatmap=24, volume=8, seed=3, first_frame=start)
    return vb


def _compute(vb):
    from oracle import capi
    vol = capi.unproject(vb.features.numpy(), vb.proj.numpy(), vb.coords.numpy(), "softmax")
    xyz, _ = capi.softargmax3d(vol[:, :3], vb.coords.numpy(), True, 1.0, return_volume=False)
    return torch.from_numpy(xyz)


def _worker(rank, world, port, out_path):
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mvn_rocm import dist as mdist
    got = mdist.run_sharded(GLOBAL_B, _frames, _compute)
    if rank == 0:
        np.save(out_path, got.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_the_batch():
    from mvn_rocm.dist import shard
    for B in (1, 5, 8, 128, 130):
        for W in (1, 2, 3, 4, 8):
            ranges = [shard(B, W, r) for r in range(W)]
            assert sum(c for _, c in ranges) == B
            assert all(ranges[r][0] + ranges[r][1] == ranges[r + 1][0] for r in range(W - 1))
            assert max(c for _, c in ranges) - min(c for _, c in ranges) <= 1
    with pytest.raises(ValueError):
        shard(8, 2, 2)


def test_per_frame_generation_is_shard_independent():
    """Frames built by a rank for its own range equal the same frames of a full batch."""
    full = _frames(0, GLOBAL_B)
    part = _frames(3, 2)
    torch.testing.assert_close(part.features, full.features[3:5], rtol=0, atol=0)
    torch.testing.assert_close(part.coords, full.coords[3:5], rtol=0, atol=0)
    torch.testing.assert_close(part.proj, full.proj[3:5], rtol=0, atol=0)


@pytest.mark.parametrize("world", (2, 3))
def test_gloo_sharded_equals_single_process(tmp_path, world):
    out = str(tmp_path / "joints.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    single = _compute(_frames(0, GLOBAL_B)).numpy()
    np.testing.assert_array_equal(np.load(out), single)
