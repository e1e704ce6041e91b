"""Job-wide convolution plans: decided once, identical on every rank, optionally persisted.

``conv.plan_for`` autotunes every convolution shape on first use (each candidate tile variant is
timed in a captured graph). Done independently per process, data-parallel ranks could pick
different variants for the same layer: ranks time-sharing a GPU see each other's load, and box
noise moves near-equal candidates. Different variants mean rank-dependent kernel times (the
slowest rank sets a synchronous step) and different fp32 accumulation orders. So:

* **one decision per job**: when a process group of more than one rank is initialised, rank 0
  times the candidates and broadcasts its choice (``broadcast_object_list``) before anything is
  captured; the other ranks wait (no GPU work) and adopt it. Every rank must reach the same
  ``plan_for`` calls in the same order -- true for data parallelism, where every rank runs the
  same model on same-shaped batches. Rank-local convolutions (evaluation on rank 0 only) must run
  inside :func:`rank_local`, or the job sets ``ARENA_CONV_PLAN_SHARE=0``;
* **persisted plans**: ``ARENA_CONV_PLAN=<path>`` names a JSON file of plans keyed by
  (kind, GPU arch, kernel-source hash, shape, stride, pad, mode flags). A plan found there is used
  without timing anything; plans decided in this run are merged into it by global rank 0. In a
  shared world only rank 0 consults the file and every decision is broadcast, hit or miss. Plans
  of a different build of the kernels (another source hash) never match;
* the time spent tuning is accumulated (:func:`stats`) and printed by the benchmarks.
"""
from __future__ import annotations

import contextlib
import json
import os
import sys
import time
from typing import Callable, Dict, Optional

_STATS = {"tuned": 0, "tune_s": 0.0, "file_hits": 0, "shared": 0, "received": 0}
_FILE: Dict[str, dict] = {}
_FILE_LOADED: Optional[str] = None
_LOCAL = 0


def stats() -> dict:
    return dict(_STATS)


def _src_hash() -> str:
    from . import _ext
    try:
        return str(getattr(_ext.load(), "src_hash", ""))
    except Exception:  # noqa: BLE001
        return ""


def _arch(device) -> str:
    import torch
    try:
        return str(torch.cuda.get_device_properties(device).gcnArchName).split(":")[0]
    except Exception:  # noqa: BLE001
        return "unknown"


def file_key(kind: str, key: tuple, device) -> str:
    return json.dumps([kind, _arch(device), _src_hash(), list(_jsonable(key))])


def _jsonable(x):
    if isinstance(x, (tuple, list)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (int, float, str, bool)) or x is None:
        return x
    return str(x)


def _path() -> Optional[str]:
    p = os.environ.get("ARENA_CONV_PLAN", "")
    return p or None


def _load_file() -> None:
    global _FILE_LOADED, _FILE
    p = _path()
    if p == _FILE_LOADED:
        return
    _FILE_LOADED, _FILE = p, {}
    if not p or not os.path.exists(p):
        return
    try:
        with open(p) as f:
            doc = json.load(f)
        plans = doc.get("plans", {})
        if not isinstance(plans, dict):
            raise ValueError("'plans' is not an object")
        _FILE = plans
    except (OSError, ValueError) as e:
        print(f"[conv-plan] ignoring unreadable plan file {p}: {e}", file=sys.stderr)


def _save(fkey: str, value: dict) -> None:
    p = _path()
    if not p:
        return
    _FILE[fkey] = value
    doc = {"version": 1, "plans": {}}
    try:
        if os.path.exists(p):
            with open(p) as f:
                old = json.load(f)
            if isinstance(old.get("plans"), dict):
                doc["plans"].update(old["plans"])
    except (OSError, ValueError):
        pass
    doc["plans"].update(_FILE)
    tmp = f"{p}.tmp{os.getpid()}"
    d = os.path.dirname(os.path.abspath(p))
    os.makedirs(d, exist_ok=True)
    with open(tmp, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=True)
    os.replace(tmp, p)


@contextlib.contextmanager
def rank_local():
    """Plans decided inside are this rank's own (no broadcast): for convolutions that only some
    ranks run."""
    global _LOCAL
    _LOCAL += 1
    try:
        yield
    finally:
        _LOCAL -= 1


def _shared_world():
    """(rank, world) when plans are decided job-wide, else None."""
    if _LOCAL or os.environ.get("ARENA_CONV_PLAN_SHARE", "1") == "0":
        return None
    try:
        import torch.distributed as dist
    except Exception:  # noqa: BLE001
        return None
    if not (dist.is_available() and dist.is_initialized()):
        return None
    w = dist.get_world_size()
    return (dist.get_rank(), w) if w > 1 else None


def decide(kind: str, key: tuple, device, tune: Callable[[], dict]) -> dict:
    """The plan (a JSON-able dict) for ``key``: from the plan file, else tuned -- in a shared world
    by rank 0 ALONE, which then broadcasts ``(from_file, plan)`` to every rank. Only rank 0 reads
    the file there, and every call is a broadcast, so the collective sequence is the same on every
    rank whatever each rank's copy of the file holds (a node-local file on a multi-node job, or a
    file rank 0 is still writing while a slow rank loads it, cannot desynchronise the ranks)."""
    fkey = file_key(kind, key, device)
    sw = _shared_world()
    value, from_file = None, False
    if sw is None or sw[0] == 0:
        _load_file()
        value = _FILE.get(fkey)
        from_file = value is not None
        if not from_file:
            t0 = time.perf_counter()
            value = tune()
            _STATS["tune_s"] += time.perf_counter() - t0
            _STATS["tuned"] += 1
    if sw is not None:
        import torch.distributed as dist
        box = [(from_file, value)]
        dist.broadcast_object_list(box, src=0)
        from_file, value = box[0]
        _STATS["shared" if sw[0] == 0 else "received"] += 1
    if from_file:
        _STATS["file_hits"] += 1
    elif _writer():
        try:
            _save(fkey, value)
        except OSError as e:
            print(f"[conv-plan] could not write {_path()}: {e}", file=sys.stderr)
    return value


def _writer() -> bool:
    """Only global rank 0 writes the plan file (one writer per job, no clobbering)."""
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank() == 0
    except Exception:  # noqa: BLE001
        pass
    return True


def reset() -> None:
    """Forget the loaded plan file (tests)."""
    global _FILE_LOADED, _FILE
    _FILE_LOADED, _FILE = None, {}
    for k in _STATS:
        _STATS[k] = 0 if isinstance(_STATS[k], int) else 0.0
