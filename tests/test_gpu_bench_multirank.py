"""The bench's multi-rank protocol on the MI355X: rank processes
launched by `bench.py --gpus N`, per-rank frame shards computed by the HIP kernels, the
max-over-ranks timing, the joints all-gather and `verify_gather` (rank 0 recomputes the
first frame of every shard and compares the gathered joints bit for bit).  One GPU box
has one device and RCCL refuses two ranks on one device ("Duplicate GPU detected"), so
the ranks share cuda:0 and the collectives run on gloo with host tensors
(`--dist-backend gloo --share-device`); the RCCL calls themselves run at world size 1 in
`tools/probe_rccl.py` and at N > 1 on the driver's 8-GPU node."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dist-backend", "gloo", "--share-device",
                        "--settle", "0", "--no-cpu-baseline", *extra],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_two_ranks_gather_verified():
    line = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--no-secondary", timeout=240)
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 16
    assert line["config"]["parallelism"] == "dp2" and "gloo" in line["config"]["collective"]
    assert line["gather"]["gather_verified"] is True
    assert line["gather"]["frames_recomputed"] == [0, 8]
    assert line["value"] > 0


@pytest.mark.timeout(600)
def test_three_ranks_ragged_config4_gather_verified():
    """Config 4's global batch of 128 over 3 ranks: shards of 43, 43 and 42 frames, the ragged
    all-gather padded to the largest shard."""
    line = _bench("--gpus", "3", "--steps", "2", "--warmup", "1", "--no-in-kernel-coords", timeout=540)
    assert line["gather"]["gather_verified"] is True
    c4 = line["config4"]
    assert c4["global_batch"] == 128 and c4["gather"]["gather_verified"] is True
    assert c4["gather"]["frames_recomputed"] == [0, 43, 86]
