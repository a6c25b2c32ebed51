"""Rehearsal of the driver's multi-GPU bench command on the one GPU of a test box.

The driver's scaling run is ``python bench.py --gpus N`` (or the same under torchrun): bench.spawn_ranks starts
N rank processes under torch.distributed.run, each builds a world-N STCGAN (rank 0's weights broadcast, the
gradient buckets all-reduced inside the backward) and the ranks' timings are max-reduced into one JSON line
(the reference's multi-GPU path is nn.DataParallel, STCGAN/stcgan.py:53-59).  STC_DIST_BACKEND=gloo lets two
ranks share one GPU here; the path through spawn_ranks, process-group setup, the world-2 trainer, the exchange
and the output contract is the one the 8-GPU run takes.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_bench_two_ranks_one_json_line():
    env = dict(os.environ, STC_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-u", "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-extras",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 64 and out["config"]["per_gpu_batch"] == 32
    assert out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["scaling"] == "weak"
