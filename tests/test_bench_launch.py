"""bench.py --gpus N without torchrun starts its own N ranks.

The driver may run ``python bench.py --gpus 8`` directly; the bench must then measure 8 ranks,
not one. These CPU tests run the launcher with a probe hook (``ARENA_BENCH_ENV_PROBE=1``: each
rank prints its torch.distributed environment and exits before importing torch) and check the
environments and the gang behaviour (a failing rank takes the rest down, the launcher exits with
its code). The GPU side (same-GPU emulation, W = 8) is in tests/test_bench_gpu.py.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env.update(PYTHONPATH=REPO, ARENA_BENCH_ENV_PROBE="1", **kw)
    return env


def test_bench_spawns_n_ranks_with_distinct_environments():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "7"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 4, r.stdout
    assert sorted(int(e["RANK"]) for e in lines) == [0, 1, 2, 3]
    for e in lines:
        assert e["LOCAL_RANK"] == e["RANK"]
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["ARENA_BENCH_LAUNCHED"] == "1"
        assert e["ARENA_BENCH_SAME_GPU"] is None
    assert len({e["MASTER_PORT"] for e in lines}) == 1
    assert "launching 4 ranks" in r.stderr


def test_bench_same_gpu_flag_reaches_every_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--same-gpu"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 2 and all(e["ARENA_BENCH_SAME_GPU"] == "1" for e in lines)


def test_bench_failing_rank_takes_the_gang_down():
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"],
                       env=_env(ARENA_BENCH_PROBE_FAIL_RANK="2", ARENA_BENCH_PROBE_SLEEP="90"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert time.time() - t0 < 60


def test_bench_under_torchrun_env_does_not_relaunch():
    env = _env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["RANK"] == "1" and lines[0]["ARENA_BENCH_LAUNCHED"] is None
