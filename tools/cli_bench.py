#!/usr/bin/env python3
"""Control-plane latency (BASELINE.md north-star rows): local backend, real supervisor.

* submit -> RUNNING: wall time from `arena submit` until `arena list` shows RUNNING;
* `arena list` / `arena top job` latency with N finished jobs in the store.

    python tools/cli_bench.py --jobs 100
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=100)
    a = ap.parse_args()
    os.environ.setdefault("ARENA_LOCAL_GPUS", "8")
    from arena_amd.cli.commands import run
    from arena_amd.cluster.local import LocalBackend

    home = tempfile.mkdtemp(prefix="arena_cli_bench_")
    b = LocalBackend(home)

    def cli(*argv):
        out = io.StringIO()
        rc = run(list(argv), backend=b, out=out)
        return rc, out.getvalue()

    # submit -> RUNNING
    lat = []
    for i in range(5):
        t0 = time.perf_counter()
        cli("submit", "sj", "--name", f"lat{i}", "sleep 5")
        while "RUNNING" not in cli("list")[1]:
            time.sleep(0.005)
        lat.append(time.perf_counter() - t0)
        b.delete_release(f"lat{i}")
    # N finished jobs
    for i in range(a.jobs):
        cli("submit", "sj", "--name", f"job{i:03d}", "true")
    deadline = time.time() + 120
    while time.time() < deadline and any(not b._state(n).get("finished")
                                         for n in b._release_names()):
        time.sleep(0.1)

    def timeit(*argv, reps=5):
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            rc, out = cli(*argv)
            best = min(best, time.perf_counter() - t0)
        return best, out
    t_list, out = timeit("list")
    t_top, _ = timeit("top", "job")
    t_get, _ = timeit("get", "job050" if a.jobs > 50 else "job000")
    print(json.dumps({"submit_to_running_s": {"min": round(min(lat), 3), "max": round(max(lat), 3)},
                      "jobs": a.jobs, "list_s": round(t_list, 3), "top_job_s": round(t_top, 3),
                      "get_s": round(t_get, 3), "listed": len(out.strip().splitlines()) - 1}))
    for n in b._release_names():
        b.delete_release(n)


if __name__ == "__main__":
    main()
