"""Parameter-server data parallelism (the reference's TFJob PS/worker mode).

Cluster spec comes from ``TF_CONFIG`` (or ``MX_CLUSTER_SPEC``) exactly as tf-operator injects it:
``{"cluster": {"ps": ["h:p", ...], "worker": [...]}, "task": {"type": "worker", "index": 0}}``.

* PS tasks run the native server (``arena-ps``, csrc/runtime/ps_server.cpp) as a child process;
  each owns one contiguous, 16-byte aligned shard of the flat fp32 parameter vector and applies
  the optimizer (Adam or SGD) itself, like TF variables placed on the PS.
* Workers compute gradients on their GPU (fused HIP kernels), copy the flat gradient to pinned
  host memory once, and push/pull all shards in parallel (one socket + thread per PS), getting
  the updated parameters back in the same round trip (PUSHPULL).

Async (default, TF's between-graph replication) or sync (``sync=True``: every round averages
one gradient from each worker, SyncReplicasOptimizer-style).
"""
from __future__ import annotations

import json
import os
import socket
import struct
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from .. import _build

MAGIC = 0x31535041
INIT, PULL, PUSH, PUSHPULL, DONE, STAT = 1, 2, 3, 4, 5, 6
_HDR = struct.Struct("<IIQ")


@dataclass
class ClusterSpec:
    ps: List[str]
    worker: List[str]
    task_type: str
    task_index: int

    @property
    def is_chief(self) -> bool:
        return self.task_type in ("chief", "master") or (
            self.task_type == "worker" and self.task_index == 0)

    @classmethod
    def from_env(cls, env=None) -> "ClusterSpec":
        env = os.environ if env is None else env
        raw = env.get("TF_CONFIG") or env.get("MX_CLUSTER_SPEC")
        if not raw:
            return cls(ps=[], worker=["127.0.0.1:0"], task_type="worker", task_index=0)
        spec = json.loads(raw)
        cl = spec.get("cluster", {})
        task = spec.get("task", {})
        workers = list(cl.get("chief", [])) + list(cl.get("master", [])) + list(cl.get("worker", []))
        ttype = task.get("type", "worker")
        idx = int(task.get("index", 0))
        if ttype == "worker" and (cl.get("chief") or cl.get("master")):
            idx += len(cl.get("chief", [])) + len(cl.get("master", []))
            ttype = "worker"
        return cls(ps=list(cl.get("ps", [])), worker=workers, task_type=ttype, task_index=idx)


def shard_ranges(n: int, num_ps: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) shards, boundaries aligned to 4 floats (16 B)."""
    per = -(-n // num_ps)
    per = (per + 3) // 4 * 4
    out = []
    for i in range(num_ps):
        lo, hi = min(i * per, n), min((i + 1) * per, n)
        out.append((lo, hi))
    return out


def _recv_full(sock: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        r = sock.recv_into(view[got:], n - got)
        if r == 0:
            raise ConnectionError("parameter server closed the connection")
        got += r
    return buf


class _Conn:
    def __init__(self, addr: str, timeout_s: float):
        host, port = addr.rsplit(":", 1)
        deadline = time.time() + timeout_s
        last = None
        while True:
            try:
                self.sock = socket.create_connection((host, int(port)), timeout=30)
                break
            except OSError as e:  # PS not up yet: the tf-operator start order is unspecified
                last = e
                if time.time() > deadline:
                    raise ConnectionError(f"cannot reach parameter server {addr}: {last}")
                time.sleep(0.1)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock.settimeout(None)

    def call(self, op: int, payload: Optional[np.ndarray] = None, out: Optional[np.ndarray] = None):
        nb = 0 if payload is None else payload.nbytes
        self.sock.sendall(_HDR.pack(MAGIC, op, nb))
        if nb:
            self.sock.sendall(memoryview(payload).cast("B"))
        magic, status, n = _HDR.unpack(_recv_full(self.sock, _HDR.size))
        if magic != MAGIC:
            raise ConnectionError("bad reply from parameter server")
        if status != 0:
            raise RuntimeError(f"parameter server rejected op {op} (status {status})")
        step = None
        if n >= 8:
            step = struct.unpack("<Q", _recv_full(self.sock, 8))[0]
            n -= 8
        if n:
            if out is None or out.nbytes != n:
                raise RuntimeError(f"unexpected {n}-byte payload from parameter server")
            view = memoryview(out).cast("B")
            got = 0
            while got < n:
                r = self.sock.recv_into(view[got:], n - got)
                if r == 0:
                    raise ConnectionError("parameter server closed the connection")
                got += r
        return step

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


class PSClient:
    """Worker side: flat fp32 vector split over all PS tasks, pushed/pulled in parallel."""

    def __init__(self, ps_addrs: List[str], n: int, timeout_s: float = 120.0):
        if not ps_addrs:
            raise ValueError("no parameter servers in the cluster spec")
        self.n = n
        self.ranges = shard_ranges(n, len(ps_addrs))
        self.conns = [_Conn(a, timeout_s) for a in ps_addrs]
        self.pool = ThreadPoolExecutor(max_workers=len(ps_addrs))
        self.step = 0

    def _each(self, fn):
        futs = [self.pool.submit(fn, i, c, lo, hi)
                for i, (c, (lo, hi)) in enumerate(zip(self.conns, self.ranges))]
        return [f.result() for f in futs]

    def init(self, params: np.ndarray) -> None:
        """Seed the shards (only the first INIT per shard takes effect: the chief's)."""
        self._each(lambda i, c, lo, hi: c.call(INIT, np.ascontiguousarray(params[lo:hi])))

    def pull(self, out: np.ndarray) -> int:
        steps = self._each(lambda i, c, lo, hi: c.call(PULL, None, out[lo:hi]))
        self.step = min(steps)
        return self.step

    def push_pull(self, grad: np.ndarray, out: np.ndarray) -> int:
        steps = self._each(lambda i, c, lo, hi: c.call(PUSHPULL, grad[lo:hi], out[lo:hi]))
        self.step = min(steps)
        return self.step

    def push(self, grad: np.ndarray) -> int:
        steps = self._each(lambda i, c, lo, hi: c.call(PUSH, grad[lo:hi]))
        self.step = min(steps)
        return self.step

    def stats(self) -> List[Tuple[int, int, int]]:
        res = []
        for c in self.conns:
            buf = np.zeros(2, dtype=np.uint64)
            step = c.call(STAT, None, buf)
            res.append((step, int(buf[0]), int(buf[1])))
        return res

    def done(self) -> None:
        for c in self.conns:
            try:
                c.call(DONE)
            except (ConnectionError, OSError):
                pass
            c.close()
        self.pool.shutdown(wait=False)


def run_server(port: int, workers: int, sync: bool = False, optimizer: str = "adam",
               lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, tf_adam: bool = False,
               host: str = "0.0.0.0") -> int:
    """Run the native PS in the foreground (child process; returns its exit code)."""
    argv = [_build.ensure_tool("arena-ps"), "--port", str(port), "--host", host,
            "--workers", str(workers), "--optimizer", optimizer, "--lr", repr(lr),
            "--beta1", repr(betas[0]), "--beta2", repr(betas[1]), "--eps", repr(eps)]
    if sync:
        argv.append("--sync")
    if tf_adam:
        argv.append("--tf-adam")
    sys.stdout.flush()
    return subprocess.call(argv)


def spawn_server(port: int, workers: int, **kw) -> subprocess.Popen:
    """Start the native PS in the background (tests / single-process demos)."""
    argv = [_build.ensure_tool("arena-ps"), "--port", str(port), "--host", kw.get("host", "127.0.0.1"),
            "--workers", str(workers), "--optimizer", kw.get("optimizer", "adam"),
            "--lr", repr(kw.get("lr", 1e-3))]
    if kw.get("sync"):
        argv.append("--sync")
    env = dict(os.environ)
    for k, v in _build.sanitizer_env().items():       # ARENA_NATIVE_SANITIZE=asan|tsan
        env.setdefault(k, v)
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=env)
    line = p.stdout.readline()          # "arena-ps: serving on ..."
    if "serving" not in line:
        p.kill()
        raise RuntimeError(f"arena-ps failed to start: {line.strip()}")
    threading.Thread(target=lambda: [None for _ in p.stdout], daemon=True).start()
    return p
