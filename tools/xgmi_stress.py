#!/usr/bin/env python3
"""Same-GPU xGMI rehearsal stress: W ranks on device 0 build XgmiComm (per-kernel self-test)
``--rounds`` times with a short barrier timeout and report every rank's per-kernel outcome and
wall time, so a failing kernel or a scheduling stall shows up by name.

    python tools/xgmi_stress.py --world 8 --rounds 3
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def worker(rank, world, port, rounds, elems, timeout_s, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from arena_amd.parallel.xgmi import XgmiComm, XgmiUnavailable
    out = []
    for r in range(rounds):
        t0 = time.time()
        try:
            comm = XgmiComm(staging_elems=elems, param_elems=elems, timeout_s=timeout_s)
            res = dict(comm.selftest_result)
            comm.close()
        except XgmiUnavailable as e:
            res = {"unavailable": str(e)[:300]}
        out.append({"round": r, "s": round(time.time() - t0, 2), "res": res})
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--elems", type=int, default=400000)
    ap.add_argument("--timeout-s", type=float, default=10.0)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.rounds, a.elems, a.timeout_s, q))
          for r in range(a.world)]
    for p in ps:
        p.start()
    for _ in range(a.world):
        rank, out = q.get(timeout=600)
        for o in out:
            print(json.dumps({"rank": rank, **o}), flush=True)
    for p in ps:
        p.join(30)


if __name__ == "__main__":
    main()
