"""CPU: `bench.py --gpus N` starts N rank processes itself when no launcher set WORLD_SIZE.

The driver may run `python bench.py --gpus 8` directly (no torchrun).  The parent must start the
ranks before anything touches a GPU, with the environment torch.distributed.run would give them
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT on 127.0.0.1), and only rank 0 may
print the result line.  --dry-ranks makes each rank report its environment and stop before
importing the library (no GPU here); under a launcher (WORLD_SIZE set) nothing is spawned.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True,
                          env=e, timeout=120)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_spawns_n_ranks_with_launcher_env(n):
    r = run(["--gpus", str(n), "--dry-ranks"])
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(ln) for ln in r.stderr.splitlines() if ln.startswith("{")]
    assert sorted(int(x["RANK"]) for x in ranks) == list(range(n))
    assert all(x["LOCAL_RANK"] == x["RANK"] for x in ranks)
    assert {x["WORLD_SIZE"] for x in ranks} == {str(n)}
    assert {x["MASTER_ADDR"] for x in ranks} == {"127.0.0.1"}
    assert len({x["MASTER_PORT"] for x in ranks}) == 1
    out = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(out) == 1 and json.loads(out[0]) == {"n_gpus": n, "rank": 0}


def test_no_spawn_under_a_launcher():
    """With WORLD_SIZE set (torchrun), the process is one rank: it does not spawn."""
    r = run(["--gpus", "2", "--dry-ranks"], env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1",
                                                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1"})
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(ln) for ln in r.stderr.splitlines() if ln.startswith("{")]
    assert len(ranks) == 1 and ranks[0]["RANK"] == "1"
    assert r.stdout.strip() == ""  # (not rank 0)


def test_gpus_mismatch_with_launcher_is_an_error():
    r = run(["--gpus", "4", "--dry-ranks"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0


def test_failed_rank_fails_the_job():
    """A rank that exits non-zero makes the parent exit with its status and stops the other ranks
    at once (they would otherwise wait in a collective for the dead one)."""
    import time
    t0 = time.time()
    r = run(["--gpus", "3", "--dry-ranks", "--dry-fail-rank", "1"])
    assert r.returncode == 3
    assert time.time() - t0 < 30
