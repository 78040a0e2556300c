"""The bench's multi-rank path (one process per GPU) rehearsed on one GPU: `bench.py --gpus 2` starts
its two ranks itself (launch_ranks, no external launcher), every rank's engine on GPU 0 and the collectives over gloo on the host
(DG_DIST_BACKEND=gloo, DG_BENCH_DEVICE=0 — RCCL refuses two ranks on one device). It runs the
groupBy key-range exchange (dg_result_export, dg_keys_partition, all_to_all, dg_merge on the GPU), the
barriers and the max-over-ranks timing, and rank 0 prints one JSON line with n_gpus = 2."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_groupby_bench_line(tmp_path):
    env = dict(os.environ, DG_DIST_BACKEND="gloo", DG_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--config",
           "groupby", "--rows", "200000", "--segments", "2", "--steps", "2", "--warmup", "1", "--data-dir",
           str(tmp_path), "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    b = json.loads(lines[0])
    assert b["n_gpus"] == 2 and b["value"] > 0 and b["groups_per_step"] > 0
