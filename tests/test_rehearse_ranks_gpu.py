"""The bench's multi-rank path (one process per GPU) rehearsed on one GPU: `bench.py --gpus 2` starts
its two ranks itself (launch_ranks, no external launcher), every rank's engine on GPU 0 and the collectives over gloo on the host
(DG_DIST_BACKEND=gloo, DG_BENCH_DEVICE=0 — RCCL refuses two ranks on one device). It runs the
groupBy key-range exchange (dg_result_export, dg_keys_partition, all_to_all, dg_merge on the GPU), the
barriers and the max-over-ranks timing, and rank 0 prints one JSON line with n_gpus = 2 whose
result_checks compare the final answer with the CPU engine's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config", ["groupby", "timeseries", "topn"])
def test_two_rank_bench_line_checks_its_answer(tmp_path, config):
    """The 2-rank line carries result_checks: the exchanged groupBy result against both ranks' CPU-engine
    groups (totals, ranges, sampled groups one by one), the all-reduced timeseries against the ranks'
    all-reduced CPU results, the folded topN against the CPU engine over both ranks' segments."""
    env = dict(os.environ, DG_DIST_BACKEND="gloo", DG_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--config",
           config, "--rows", "200000", "--segments", "2", "--steps", "2", "--warmup", "1", "--data-dir",
           str(tmp_path), "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    b = json.loads(lines[0])
    assert b["n_gpus"] == 2 and b["value"] > 0
    rc = b["result_checks"]
    if config == "groupby":
        assert b["groups_per_step"] > 0
        assert rc["all_equal"] and rc["ranks"] == 2 and rc["sample_groups"] > 0, rc
        assert rc["groups"] >= b["groups_per_step"]  # (rank 0's local count is a lower bound)
    elif config == "timeseries":
        assert rc["per_bucket_equal"], rc
    else:
        assert rc["per_entry_equal"] and rc["entries"] == 10, rc
