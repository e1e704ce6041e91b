"""bench.py's N > 1 path end to end on one GPU: ``--gpus 2 --same-gpu``
starts two ranks itself, both on device 0 (gloo + same-device xGMI mappings), and must print one
JSON line with ``n_gpus: 2``, the MNIST xGMI Adam step replica-verified, and the data-parallel
ResNet-50 step (ShardedMasterSGD, hipGraph) replica-verified as ``dp2``."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_same_gpu_end_to_end():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["PYTHONPATH"] = REPO
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--same-gpu",
           "--steps", "60", "--warmup", "20", "--verify-every", "20",
           "--resnet-batch", "16", "--resnet-steps", "4", "--resnet-verify-every", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2", line
    assert line["config"]["launch"] == "bench.py" and "emulated" in line, line
    assert "comm=xgmi" in line["config"]["exec"], line
    assert line["replicas_verified"] > 0, line
    assert "resnet50_error" not in line, line
    rc = line["resnet50_config"]
    assert rc["parallelism"] == "dp2" and rc["replicas_verified"] > 0, line
    assert rc["comm"].startswith("xgmi-sharded-sgd"), line
    # north-star #2 rows: xGMI timed at every size, RCCL marked skipped under gloo
    ccl = line["ccl"]
    assert ccl["xgmi"]["form"] == "pull", ccl
    assert all(v == "ok" for v in ccl["xgmi"]["selftest"].values()), ccl
    assert {"allreduce_oneshot", "allreduce_twoshot", "adam", "sgd_bf16", "sgd_f32",
            "broadcast_direct", "allgather"} <= set(ccl["xgmi"]["selftest"]), ccl
    ops = [r["op"] for r in ccl["rows"]]
    assert ops.count("allreduce") == 5 and "sharded_sgd_bf16_bucket" in ops, ccl
    assert all("xgmi_us" in r and "rccl_us" not in r and "gloo" in r["rccl"]
               for r in ccl["rows"]), ccl


def test_bench_failed_resnet_fails_the_run():
    """A ResNet-50 failure at N > 1 is reported in the line AND exits non-zero."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(PYTHONPATH=REPO, ARENA_BENCH_FAIL_RESNET="1")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--same-gpu",
           "--steps", "20", "--warmup", "10", "--ccl", "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stdout[-2000:]
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["failed"] == ["resnet50"] and "injected" in line["resnet50_error"], line
