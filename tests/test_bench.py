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
