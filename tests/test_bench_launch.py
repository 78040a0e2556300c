"""CPU: bench.py's rank contract. `--gpus N` without a launcher starts N ranks itself (launch_ranks:
RANK = LOCAL_RANK = r, WORLD_SIZE = N, one rendezvous address, a failing rank's exit code
propagates); under a launcher WORLD_SIZE must equal --gpus."""
import argparse
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_rank_env_contract(monkeypatch):
    args = argparse.Namespace(gpus=1)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.rank_env(args) == (1, 0, 0)
    args.gpus = 2
    with pytest.raises(SystemExit):  # N > 1 ranks come from launch_ranks (or a launcher)
        bench.rank_env(args)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert bench.rank_env(args) == (2, 1, 1)
    args.gpus = 4
    with pytest.raises(SystemExit):  # a launcher's world that disagrees with --gpus
        bench.rank_env(args)


def test_launch_ranks_env_and_exit_codes(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(
        "import json, os, sys\n"
        "keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT']\n"
        "open(os.path.join(sys.argv[1], 'rank%s.json' % os.environ['RANK']), 'w').write(\n"
        "    json.dumps({k: os.environ.get(k) for k in keys}))\n"
        "sys.exit(int(sys.argv[2]) if os.environ['RANK'] == sys.argv[3] else 0)\n")
    assert bench.launch_ranks(3, [str(tmp_path), "0", "-1"], script=str(script)) == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"} and {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert bench.launch_ranks(2, [str(tmp_path), "7", "1"], script=str(script)) == 7  # rank 1 fails
