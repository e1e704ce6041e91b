"""Training-progress heartbeat: hang detection for ranks (SURVEY §5 failure detection).

The reference only notices failures when a process exits: the Job `backoffLimit`, TFJob restart
policies, and jobmon waiting for the MPI launcher. A rank stuck in a collective (a
peer died mid-allreduce, a wedged GPU queue) never exits, so the job hangs forever. Here a rank
marks progress with ``beat()``; the runtime kills a rank whose beats stop for longer than the job's
``--heartbeatTimeout``, and the normal retry / gang-restart policy takes over:

* local backend: ``arena-supervisor`` compares the heartbeat file's mtime against the timeout;
* k8s backend: the container gets an exec livenessProbe on the same file, so the kubelet
  restarts it.

Beats are progress-based on purpose. A background "alive" thread would keep beating while the
main thread is stuck in RCCL. The file is only touched once per ``min_interval`` seconds, so
``beat()`` can be called every training step. ``hvd.DistributedOptimizer.step()`` and the fused
trainers call it themselves. Without ``ARENA_HEARTBEAT_FILE`` in the environment, every call is
a no-op.
"""
from __future__ import annotations

import os
import time
from typing import Optional

ENV = "ARENA_HEARTBEAT_FILE"

_state = {"path": None, "next": 0.0, "min_interval": 0.5, "init": False}


def _path() -> Optional[str]:
    if not _state["init"]:
        _state["path"] = os.environ.get(ENV) or None
        _state["init"] = True
    return _state["path"]


def configure(path: Optional[str], min_interval: float = 0.5) -> None:
    """Override the heartbeat file (tests) -- None disables."""
    _state.update(path=path, init=True, next=0.0, min_interval=float(min_interval))


def beat(step: Optional[int] = None) -> None:
    """Record progress (throttled to one file touch per ``min_interval`` seconds)."""
    path = _path()
    if path is None:
        return
    now = time.monotonic()
    if now < _state["next"]:
        return
    _state["next"] = now + _state["min_interval"]
    try:
        with open(path, "w") as f:
            f.write(f"{int(time.time())} {'' if step is None else int(step)}\n")
    except OSError:
        pass  # a heartbeat must never take the training process down


def liveness_probe(path: str, timeout_s: float) -> dict:
    """Kubernetes exec livenessProbe: fails once the file exists and is older than the timeout
    (no file yet = still starting up, which the probe tolerates)."""
    t = int(max(1, round(timeout_s)))
    script = (f'f={path}; [ ! -f "$f" ] || '
              f'[ $(( $(date +%s) - $(stat -c %Y "$f") )) -lt {t} ]')
    return {"exec": {"command": ["sh", "-c", script]}, "initialDelaySeconds": t,
            "periodSeconds": max(1, min(10, t // 3)), "failureThreshold": 1}
