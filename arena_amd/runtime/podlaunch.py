"""In-pod rank launcher: several data-parallel ranks per pod (Horovod's hosts x GPUs layout).

The reference launches ``mpirun`` over a hostfile with ``hvd-distribute.sh <hosts> <gpus>``
(charts/tf-horovod/README.md:66-69, hostfile at charts/tf-horovod/templates/config.yaml:13-17):
a pod that holds 4 GPUs runs 4 ranks. Here there is no sshd and no mpirun: every pod's entry
process is this launcher, which starts one child per rank BEFORE anything touches a GPU (it never
imports torch or HIP), gives each the torch.distributed environment, and supervises them:

* ``RANK = pod_index * nproc + local_rank``, ``WORLD_SIZE = pods * nproc``;
  ``LOCAL_RANK`` / ``LOCAL_WORLD_SIZE`` = the rank's index / count on this node (in a K8s pod:
  within the pod, whose device-plugin allocation is exactly its ``nproc`` GPUs; on the local
  backend, node-wide indices into the job's GPU set, passed as ``ARENA_RANK_LOCAL_IDS`` and
  ``ARENA_NODE_RANKS``, so all ranks of a one-node job can map each other for xGMI);
  ``GROUP_RANK`` / ``GROUP_WORLD_SIZE`` = pod index / pod count (torchrun's names);
* the first rank that exits non-zero takes the others down (SIGTERM, then SIGKILL after a grace
  period) and the launcher exits with that code -- a crashed rank must not leave its peers
  blocked in a collective until the RCCL timeout. Every rank runs in its own process session and
  is signalled as a process GROUP, so the real rank behind a compound command
  (``cd /w && python train.py``: a grandchild of the launcher) goes down with its shell;
* SIGTERM/SIGINT to the launcher (pod deletion, ``arena delete``) is forwarded to every rank;
* the ranks' stdout/stderr are forwarded line by line (one pod log, never two ranks' output
  spliced into one line); ``ARENA_RANK_TAG_OUTPUT=1`` prefixes every line with ``[<rank>]``, like
  mpirun's ``--tag-output``.

Configured through the environment (so a chart needs no quoting of the user's command):
``ARENA_RANK_COMMAND`` (the shell command every rank runs), ``ARENA_RANKS_PER_POD``,
``ARENA_PODS``, ``ARENA_POD_INDEX`` (or ``POD_NAME`` = ``<statefulset>-<ordinal>`` -> ordinal + 1;
the launcher pod is index 0), optional ``ARENA_RANK_PROFILE_DIR`` (each rank under
``rocprofv3 --kernel-trace --stats``; commands without shell syntax only).

    ARENA_RANK_COMMAND="python train.py" ARENA_RANKS_PER_POD=4 ARENA_PODS=2 ARENA_POD_INDEX=1 \\
        python -m arena_amd.runtime.podlaunch
"""
from __future__ import annotations

import os
import shlex
import shutil
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional

_SHELL_META = set("|&;<>()$`\\\"'*?[#~=%")


def pod_index(env: Dict[str, str]) -> int:
    if env.get("ARENA_POD_INDEX", "") != "":
        return int(env["ARENA_POD_INDEX"])
    name = env.get("POD_NAME", "")
    tail = name.rsplit("-", 1)[-1]
    if not tail.isdigit():
        raise SystemExit("podlaunch: set ARENA_POD_INDEX, or POD_NAME=<statefulset>-<ordinal>")
    return int(tail) + 1     # StatefulSet ordinal i is pod i + 1 (the launcher pod is 0)


def rank_envs(env: Dict[str, str]) -> List[Dict[str, str]]:
    """The environment of every rank this pod runs (pure function: tested on CPU)."""
    nproc = int(env.get("ARENA_RANKS_PER_POD", "1"))
    pods = int(env.get("ARENA_PODS", "1"))
    if nproc < 1 or pods < 1:
        raise SystemExit("podlaunch: ARENA_RANKS_PER_POD and ARENA_PODS must be >= 1")
    idx = pod_index(env)
    if not 0 <= idx < pods:
        raise SystemExit(f"podlaunch: pod index {idx} outside 0..{pods - 1}")
    local_ids = [int(x) for x in env.get("ARENA_RANK_LOCAL_IDS", "").split(",") if x != ""]
    if local_ids and len(local_ids) != nproc:
        raise SystemExit(f"podlaunch: ARENA_RANK_LOCAL_IDS names {len(local_ids)} ranks, "
                         f"ARENA_RANKS_PER_POD is {nproc}")
    node_ranks = int(env.get("ARENA_NODE_RANKS", str(nproc)))
    out = []
    for lr in range(nproc):
        e = dict(env)
        e.update(RANK=str(idx * nproc + lr), WORLD_SIZE=str(pods * nproc),
                 LOCAL_RANK=str(local_ids[lr] if local_ids else lr),
                 LOCAL_WORLD_SIZE=str(node_ranks), GROUP_RANK=str(idx),
                 GROUP_WORLD_SIZE=str(pods), ARENA_POD_LOCAL_RANK=str(lr))
        out.append(e)
    return out


def rank_argv(command: str, env: Dict[str, str]) -> List[str]:
    prof = env.get("ARENA_RANK_PROFILE_DIR", "")
    if prof and shutil.which("rocprofv3") and not (_SHELL_META & set(command)):
        # rocprofv3 must exec the program itself (no shell hop under its preload)
        d = os.path.join(prof, f"rank{env['RANK']}")
        os.makedirs(d, exist_ok=True)
        return ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", d,
                "-o", "run", "--"] + shlex.split(command)
    return ["/bin/sh", "-c", command]


_OUT_LOCK = threading.Lock()


def _pump(src, dst, prefix: bytes) -> None:
    """Copy a rank's pipe to the launcher's stream one whole line at a time."""
    for line in iter(src.readline, b""):
        if not line.endswith(b"\n"):
            line += b"\n"
        with _OUT_LOCK:
            dst.write(prefix + line)
            dst.flush()
    src.close()


class _Gang:
    def __init__(self, grace_s: float, tag: bool = False):
        self.procs: List[subprocess.Popen] = []
        self.pumps: List[threading.Thread] = []
        self.grace_s = grace_s
        self.tag = tag
        self.stopping = False

    def start(self, argv: List[str], env: Dict[str, str]) -> None:
        # own session: the rank and everything it starts form one process group (pgid == pid)
        p = subprocess.Popen(argv, env=env, stdin=subprocess.DEVNULL, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, start_new_session=True)
        self.procs.append(p)
        prefix = f"[{env['RANK']}] ".encode() if self.tag else b""
        for src, dst in ((p.stdout, sys.stdout.buffer), (p.stderr, sys.stderr.buffer)):
            t = threading.Thread(target=_pump, args=(src, dst, prefix), daemon=True)
            t.start()
            self.pumps.append(t)

    def drain(self, timeout_s: float = 5.0) -> None:
        deadline = time.time() + timeout_s
        for t in self.pumps:
            t.join(max(0.0, deadline - time.time()))

    def signal_all(self, sig: int) -> None:
        """Signal every rank's process group -- also of a rank whose shell already exited, since
        a grandchild it started may still hold the group (and a GPU)."""
        for p in self.procs:
            try:
                os.killpg(p.pid, sig)
            except (ProcessLookupError, PermissionError):
                pass
            except OSError:
                if p.poll() is None:
                    try:
                        p.send_signal(sig)
                    except OSError:
                        pass

    def _group_alive(self, p: subprocess.Popen) -> bool:
        if p.poll() is None:
            return True
        try:
            os.killpg(p.pid, 0)
            return True
        except OSError:
            return False

    def stop(self) -> None:
        """SIGTERM every live rank, SIGKILL what is left after the grace period."""
        self.stopping = True
        self.signal_all(signal.SIGTERM)
        deadline = time.time() + self.grace_s
        while time.time() < deadline and any(self._group_alive(p) for p in self.procs):
            time.sleep(0.05)
        self.signal_all(signal.SIGKILL)
        for p in self.procs:
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                pass

    def wait(self) -> int:
        """0 when every rank succeeded, else the first failing rank's code (signals -> 128+n)."""
        while True:
            live = 0
            for p in self.procs:
                rc = p.poll()
                if rc is None:
                    live += 1
                elif rc != 0:
                    self.stop()
                    return rc if rc > 0 else 128 - rc
            if live == 0:
                return 0
            time.sleep(0.05)


def run_gang(argvs: List[List[str]], envs: List[Dict[str, str]], grace_s: float = 10.0,
             tag: bool = False) -> int:
    """Start one process per (argv, env), supervise them as a gang (first failure takes the rest
    down), forward SIGTERM/SIGINT, relay their output line by line; the gang's exit code."""
    gang = _Gang(grace_s, tag=tag)
    prev = {}

    def forward(sig, _frame):
        gang.stop()
        gang.drain(1.0)
        sys.exit(128 + sig)

    for s in (signal.SIGTERM, signal.SIGINT):
        prev[s] = signal.signal(s, forward)
    try:
        for a, e in zip(argvs, envs):
            gang.start(a, e)
        rc = gang.wait()
        gang.drain()
        return rc
    finally:
        if any(p.poll() is None for p in gang.procs):
            gang.stop()
        for s, h in prev.items():
            signal.signal(s, h)


def local_world_envs(nproc: int, env: Optional[Dict[str, str]] = None,
                     master_port: Optional[int] = None) -> List[Dict[str, str]]:
    """torch.distributed environments of a one-node world of ``nproc`` ranks on this host (what
    ``torchrun --standalone --nproc-per-node nproc`` would set), for a launcher that starts the
    ranks itself: RANK = LOCAL_RANK = i, WORLD_SIZE = LOCAL_WORLD_SIZE = nproc, rendezvous at
    127.0.0.1 on a free port."""
    base = dict(os.environ if env is None else env)
    if master_port is None:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            master_port = s.getsockname()[1]
    base.update(ARENA_RANKS_PER_POD=str(nproc), ARENA_PODS="1", ARENA_POD_INDEX="0")
    base.pop("ARENA_RANK_LOCAL_IDS", None)
    base.pop("ARENA_NODE_RANKS", None)
    out = []
    for e in rank_envs(base):
        e.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port))
        for k in ("ARENA_RANKS_PER_POD", "ARENA_PODS", "ARENA_POD_INDEX"):
            e.pop(k, None)
        out.append(e)
    return out


def main(argv: Optional[List[str]] = None) -> int:
    env = dict(os.environ)
    command = env.get("ARENA_RANK_COMMAND", "")
    args = list(sys.argv[1:] if argv is None else argv)
    if args[:1] == ["--"]:
        args = args[1:]
    if args:
        command = " ".join(args)
    if not command:
        print("podlaunch: no command (ARENA_RANK_COMMAND or arguments after --)", file=sys.stderr)
        return 2
    envs = rank_envs(env)
    return run_gang([rank_argv(command, e) for e in envs], envs,
                    float(env.get("ARENA_RANK_GRACE_S", "10")),
                    tag=env.get("ARENA_RANK_TAG_OUTPUT", "0") == "1")


if __name__ == "__main__":
    sys.exit(main())
