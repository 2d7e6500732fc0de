"""bench.py's launcher (one process per GPU, N = 1/2/4/8): `--gpus N` must give an
N-rank job whether or not an outside torch.distributed.run started it.  CPU only: the decision
is printed by --plan-only (no GPU call), and --launch-check starts the ranks exactly as the bench
does and joins them over gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_plan_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--plan-only"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["launch"] == "spawn" and plan["world"] == n
    assert [x["rank"] for x in plan["ranks"]] == list(range(n))
    assert [x["device"] for x in plan["ranks"]] == [f"cuda:{k}" for k in range(n)]


def test_plan_single_gpu_is_direct():
    plan = json.loads(_run(["--plan-only"]).stdout.strip().splitlines()[-1])
    assert plan == {"launch": "direct", "world": 1, "rank": 0, "local_rank": 0}


def test_plan_under_outside_launcher():
    r = _run(["--gpus", "8", "--plan-only"], {"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"})
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan == {"launch": "direct", "world": 8, "rank": 5, "local_rank": 5}


@pytest.mark.parametrize("ws,gpus", [("2", "8"), ("8", "1"), ("1", "2")])
def test_world_size_mismatch_fails(ws, gpus):
    r = _run(["--gpus", gpus, "--plan-only"], {"WORLD_SIZE": ws})
    assert r.returncode != 0 and "disagree" in r.stderr


def test_launch_check_joins_all_ranks():
    """The real spawn path: `bench.py --gpus 4` starts 4 fresh processes, which join one job."""
    r = _run(["--gpus", "4", "--launch-check"], timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["world"] == 4 and out["n_gpus"] == 4 and out["ranks"] == [0, 1, 2, 3]


def test_hung_collective_exits_nonzero():
    """the split/gather watchdog must fail the job.  Rank 1 never joins the
    all-gather, so ranks 0 and 2 hang in it; the watchdog (3 s here, 120 s in the bench) ends every
    rank with a non-zero code, and the launcher's exit code is non-zero too."""
    r = _run(["--gpus", "3", "--launch-check", "--stall-rank", "1", "--split-timeout", "3"], timeout=180)
    assert r.returncode != 0, (r.stdout, r.stderr[-2000:])
    assert "watchdog fired" in r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "timeout" in json.loads(lines[0])["error"]
