"""bench.py's N-rank launch (driver contract): `python bench.py --gpus N` started without an outer
torch.distributed.run starts one itself as a child process and passes exactly one JSON line through;
under an outer launcher WORLD_SIZE must equal --gpus.  Exercised with --stub-step (the real rank
plumbing, timing and line around a host-only step over gloo), so no GPU is needed."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                         "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=e, timeout=240)


def test_gpus_2_starts_two_ranks_and_prints_one_line():
    r = _run(["--gpus", "2", "--stub-step", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 16384
    assert d["config"]["parallelism"].startswith("dp2")
    assert d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["data"].startswith("stub")


def test_gpus_1_runs_in_process():
    r = _run(["--stub-step", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 8192


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--stub-step", "--steps", "1", "--warmup", "0"], WORLD_SIZE="2", RANK="0",
             LOCAL_RANK="0")
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "WORLD_SIZE=2" in r.stderr


def test_failing_rank_fails_the_launch():
    # --steps 0: rank 0 fails computing ms/step (ZeroDivisionError) after the group is up; the
    # launcher must return non-zero and print no line
    r = _run(["--gpus", "2", "--stub-step", "--steps", "0", "--warmup", "0"])
    assert r.returncode != 0
    assert r.stdout.strip() == ""
