"""Job-wide conv plans: rank 0 decides, every rank adopts; a plan file skips
the timing on the next run.

CPU: ``planstore.decide`` over a gloo world of 2 with rank-dependent "tuning" results (each rank
would pick a different variant on its own). GPU: ``conv.plan_for`` autotuning a real layer with
two ranks sharing one GPU -- identical plans on both ranks, and a second job with the plan file
times nothing."""
from __future__ import annotations

import json
import os
import socket
import traceback

import pytest
import torch
import torch.multiprocessing as mp


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu_worker(rank, world, port, plan_file, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), ARENA_CONV_PLAN=plan_file)
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from arena_amd.ops import planstore
        planstore.reset()
        calls = []

        def tune():
            calls.append(rank)
            return {"fwd": 4096 + rank, "wgrad": [3, 7 + rank], "times": {"fwd:1": 1.5}}

        a = planstore.decide("conv", ((8, 64, 14, 14), (64, 64, 3, 3), 1, 1), "cpu", tune)
        b = planstore.decide("conv", ((8, 64, 7, 7), (64, 64, 3, 3), 1, 1), "cpu", tune)
        with planstore.rank_local():
            c = planstore.decide("stem", ((rank + 1, 16, 8, 8),), "cpu", tune)
        dist.barrier()
        res = {"a": a, "b": b, "c": c, "calls": calls, "stats": planstore.stats()}
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


def _run(fn, world, *args, timeout=120):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=fn, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            r, res, err = q.get(timeout=timeout)
            assert err is None, f"rank {r} failed:\n{err}"
            out[r] = res
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    return out


def test_plans_decided_by_rank0_and_persisted(tmp_path):
    f = str(tmp_path / "plans.json")
    out = _run(_cpu_worker, 2, f)
    assert out[0]["calls"] == [0, 0, 0] and out[1]["calls"] == [1]   # only rank-local tuned on 1
    for r in (0, 1):
        assert out[r]["a"]["fwd"] == 4096 and out[r]["b"]["wgrad"] == [3, 7], out
        assert out[r]["c"]["fwd"] == 4096 + r         # rank_local: each rank's own choice
    assert out[0]["stats"]["shared"] == 2 and out[1]["stats"]["received"] == 2
    doc = json.load(open(f))
    assert len(doc["plans"]) == 3                     # rank 0's two shared + its rank-local one
    # second job: every shared plan comes from rank 0's file (nothing timed); the hit is still
    # broadcast, so the collective sequence does not depend on what each rank's file holds
    out2 = _run(_cpu_worker, 2, f)
    for r in (0, 1):
        assert out2[r]["a"]["fwd"] == 4096 and out2[r]["stats"]["file_hits"] >= 2, out2
    assert out2[0]["stats"]["shared"] == 2 and out2[1]["stats"]["received"] == 2, out2
    assert out2[0]["calls"] == [] and out2[1]["calls"] == [1]   # rank 1's stem key is new


def _split_file_worker(rank, world, port, files, q):
    # each rank names its OWN plan file (a node-local path on a multi-node job): only rank 1's
    # holds a plan for key a. The old per-rank lookup made rank 1 return without joining rank 0's
    # broadcast (hang / next key's plan adopted for this one).
    _cpu_worker(rank, world, port, files[rank], q)


def test_plan_file_on_some_ranks_only_does_not_desync(tmp_path):
    f0, f1 = str(tmp_path / "r0.json"), str(tmp_path / "r1.json")
    from arena_amd.ops import planstore
    key = planstore.file_key("conv", ((8, 64, 14, 14), (64, 64, 3, 3), 1, 1), "cpu")
    with open(f1, "w") as fh:
        json.dump({"version": 1, "plans": {key: {"fwd": 1, "wgrad": [0, 0]}}}, fh)
    out = _run(_split_file_worker, 2, [f0, f1])
    for r in (0, 1):
        assert out[r]["a"]["fwd"] == 4096 and out[r]["b"]["wgrad"] == [3, 7], out
    assert out[0]["calls"] == [0, 0, 0] and out[1]["stats"]["file_hits"] == 0, out


def _gpu_worker(rank, world, port, plan_file, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), ARENA_CONV_PLAN=plan_file)
        torch.cuda.set_device(0)
        import torch.distributed as dist
        dist.init_process_group("gloo")
        from arena_amd.ops import conv, planstore
        planstore.reset()
        conv.set_mode("auto")
        x = torch.randn(16, 128, 14, 14, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(128, 128, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        plan = conv.plan_for(x, w, 1, 1)
        res = {"plan": [str(plan.fwd), str(plan.bwd), str(plan.wgrad), str(plan.bwd_bn)],
               "stats": planstore.stats()}
        conv.set_mode(None)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception:  # noqa: BLE001
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.gpu
def test_conv_plans_identical_across_ranks_and_reused(tmp_path):
    f = str(tmp_path / "plans.json")
    out = _run(_gpu_worker, 2, f, timeout=240)
    assert out[0]["plan"] == out[1]["plan"], out
    assert out[0]["stats"]["tuned"] == 1 and out[1]["stats"]["tuned"] == 0, out
    assert out[0]["stats"]["tune_s"] > 0
    out2 = _run(_gpu_worker, 2, f, timeout=240)
    for r in (0, 1):
        assert out2[r]["plan"] == out[0]["plan"], (out, out2)
        assert out2[r]["stats"]["tuned"] == 0 and out2[r]["stats"]["file_hits"] == 1, out2
