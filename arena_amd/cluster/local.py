"""Local backend: run jobs as real processes on this machine's GPUs.

Replaces helm + Kubernetes + tf-operator + mpirun for a single MI355X node:
  * a release = a job directory ``$ARENA_HOME/jobs/<name>/`` (release.json, plan.json,
    state.json, logs/<pod>.log, code/, tb/, traces/);
  * manifests are rendered by the same chart code as the K8s backend and instantiated by the
    in-process controller, so discovery/status/GPU accounting run unchanged;
  * the native C++ supervisor (csrc/runtime/supervisor.cpp) owns the processes, log capture and
    the retry / clean-pod / launcher-reap policies, and publishes state.json;
  * GPUs are assigned from the xGMI topology reported by the native probe (arena-probe), exported
    as HIP_VISIBLE_DEVICES; allreduce ranks of one job see the job's whole GPU set (RCCL P2P over
    xGMI) and pick theirs with LOCAL_RANK; rendezvous is a TCPStore on 127.0.0.1.
"""
from __future__ import annotations

import json
import os
import shlex
import shutil
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, Iterator, List, Optional

from .. import _build
from ..utils.logs import get_logger
from ..utils.timefmt import parse_rfc3339
from . import charts
from .backend import Backend, BackendError, Release
from .controller import ClusterState
from .objects import (AMD_GPU, GPU_RESOURCES, Endpoints, Meta, Node, POD_FAILED, POD_PENDING,
                      POD_RUNNING, POD_SUCCEEDED, matches)

log = get_logger("local")
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_SHELL_META = set("|&;<>()$`\\\"'*?[#~=%")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _host_ip() -> str:
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def _pid_alive(pid: int) -> bool:
    if pid <= 0:
        return False
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    # a zombie child of ours counts as dead
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except OSError:
        return False


def probe_gpus() -> dict:
    """GPU inventory from the native probe; ``ARENA_LOCAL_GPUS=N`` overrides the count (tests)."""
    override = os.environ.get("ARENA_LOCAL_GPUS")
    if override is not None:
        n = int(override)
        return {"count": n, "gpus": [{"index": i, "hive_id": "0", "links": []} for i in range(n)]}
    try:
        out = subprocess.run([_build.ensure_tool("arena-probe")], capture_output=True, text=True,
                             timeout=10, check=True).stdout
        return json.loads(out)
    except Exception as e:  # noqa: BLE001
        log.debug("arena-probe failed: %s", e)
        return {"count": 0, "gpus": []}


def pick_gpus(inventory: dict, busy: set, need: int, prefer_hive: Optional[str] = None) -> List[int]:
    """Choose ``need`` free GPUs, keeping a job inside one xGMI hive (all 8 MI355X of a node are
    one fully-connected hive; across hives traffic falls back to PCIe/network)."""
    free = [g for g in inventory.get("gpus", []) if g["index"] not in busy]
    by_hive: Dict[str, list] = {}
    for g in free:
        by_hive.setdefault(str(g.get("hive_id", "0")), []).append(g["index"])
    hives = sorted(by_hive.items(), key=lambda kv: (kv[0] != prefer_hive, -len(kv[1]), kv[0]))
    for _, ids in hives:
        if len(ids) >= need:
            return sorted(ids)[:need]
    ids = sorted(g["index"] for g in free)
    if len(ids) < need:
        raise BackendError(f"insufficient GPUs on this node: need {need}, free {len(ids)} "
                           f"(of {inventory.get('count', 0)})")
    return ids[:need]


class LocalBackend(Backend):
    name = "local"

    def __init__(self, home: str, node_name: Optional[str] = None):
        self.home = os.path.abspath(home)
        self.jobs_dir = os.path.join(self.home, "jobs")
        os.makedirs(self.jobs_dir, exist_ok=True)
        self.node_name = node_name or socket.gethostname()
        self._inv = None
        self._ip = None

    # ------------------------------------------------------------------------------ helpers
    def inventory(self) -> dict:
        if self._inv is None:
            self._inv = probe_gpus()
        return self._inv

    def node_ip(self) -> str:
        if self._ip is None:
            self._ip = os.environ.get("ARENA_NODE_IP") or _host_ip()
        return self._ip

    def _node(self) -> Node:
        n = self.inventory().get("count", 0)
        meta = Meta(name=self.node_name, namespace="",
                    labels={"kubernetes.io/hostname": self.node_name,
                            "arena.amd.com/gpu-arch": "gfx950"})
        return Node(meta=meta, capacity={AMD_GPU: n} if n else {},
                    addresses=[("InternalIP", self.node_ip()), ("Hostname", self.node_name)])

    def job_dir(self, name: str) -> str:
        return os.path.join(self.jobs_dir, name)

    def _read_json(self, path: str, default=None):
        try:
            with open(path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return default

    def _release_names(self) -> List[str]:
        try:
            return sorted(d for d in os.listdir(self.jobs_dir)
                          if os.path.exists(os.path.join(self.jobs_dir, d, "release.json")))
        except OSError:
            return []

    def _busy_gpus(self, exclude: Optional[str] = None) -> set:
        busy = set()
        for name in self._release_names():
            if name == exclude:
                continue
            rel = self._read_json(os.path.join(self.job_dir(name), "release.json"), {})
            st = self._state(name)
            for pod, ids in (rel.get("gpus") or {}).items():
                ps = (st.get("pods") or {}).get(pod, {})
                alive = ps.get("phase", "Pending") in ("Pending", "Running") and not ps.get("deleted")
                if alive and not (st.get("finished") and ps.get("phase") != "Running"):
                    busy.update(ids)
        return busy

    def _state(self, name: str) -> dict:
        st = self._read_json(os.path.join(self.job_dir(name), "state.json"), {}) or {}
        pid = int(st.get("supervisor_pid", 0) or 0)
        if st and not st.get("finished") and not _pid_alive(pid):
            # supervisor died (host reboot, kill -9): nothing is running any more
            st["finished"] = True
            st["phase"] = "Failed" if st.get("phase") in ("Running", "Pending", None) else st["phase"]
            for ps in (st.get("pods") or {}).values():
                if ps.get("phase") in ("Running", "Pending"):
                    ps["phase"] = "Failed"
                    ps["exit_code"] = ps.get("exit_code", -1)
        return st

    # ----------------------------------------------------------------------------- install
    def install_release(self, name, namespace, chart, values) -> Release:
        if self.release_exists(name):
            raise BackendError(f"the job {name} is already exist, please delete it first. "
                               f"use 'arena delete {name}'")
        jd = self.job_dir(name)
        created = time.time()
        manifests = charts.render(chart, name, namespace, values)
        state = ClusterState(clock=lambda: created)
        state.nodes[self.node_name] = self._node()
        state.apply(manifests)
        os.makedirs(os.path.join(jd, "logs"), exist_ok=True)
        os.makedirs(os.path.join(jd, "control"), exist_ok=True)
        try:
            self._sync_code(values, jd)
            plan, gpus, ports = self._plan(name, namespace, chart, values, state, jd)
        except Exception:
            shutil.rmtree(jd, ignore_errors=True)
            raise
        rel = {"name": name, "namespace": namespace, "chart": chart, "values": values,
               "manifests": manifests, "created": created, "gpus": gpus, "ports": ports,
               "node": self.node_name, "backend": "local"}
        with open(os.path.join(jd, "release.json"), "w") as f:
            json.dump(rel, f, indent=1)
        with open(os.path.join(jd, "plan.json"), "w") as f:
            json.dump(plan, f, indent=1)
        self._spawn_supervisor(jd)
        return Release(name, namespace, chart, values, manifests, created)

    def _spawn_supervisor(self, jd: str) -> None:
        sup = _build.ensure_tool("arena-supervisor")
        env = dict(os.environ)
        for k, v in _build.sanitizer_env().items():   # ARENA_NATIVE_SANITIZE=asan|tsan
            env.setdefault(k, v)
        with open(os.path.join(jd, "supervisor.log"), "ab") as lf:
            p = subprocess.Popen([sup, jd], stdin=subprocess.DEVNULL, stdout=lf, stderr=lf,
                                 start_new_session=True, env=env, close_fds=True)
        with open(os.path.join(jd, "supervisor.pid"), "w") as f:
            f.write(str(p.pid))
        # wait briefly for the first state publication so `arena list` right after submit works
        deadline = time.time() + 5
        while time.time() < deadline and not os.path.exists(os.path.join(jd, "state.json")):
            time.sleep(0.01)

    def _sync_code(self, values: dict, jd: str) -> None:
        """The init container's job (git-sync / rsync into $workingDir/code), done at submit."""
        mode, src = values.get("syncMode"), values.get("syncSource", "")
        if not mode:
            return
        code = os.path.join(jd, "code")
        os.makedirs(code, exist_ok=True)
        if mode == "git":
            dest = os.path.join(code, values.get("syncGitProjectName") or "repo")
            r = subprocess.run(["git", "clone", "--depth", "1", src, dest], capture_output=True,
                               text=True)
            if r.returncode != 0:
                raise BackendError(f"git sync failed: {r.stderr.strip()}")
        else:
            if shutil.which("rsync"):
                r = subprocess.run(["rsync", "-a", src, code + "/"], capture_output=True, text=True)
                if r.returncode != 0:
                    raise BackendError(f"rsync failed: {r.stderr.strip()}")
            elif os.path.isdir(src):
                shutil.copytree(src, os.path.join(code, os.path.basename(src.rstrip("/"))),
                                dirs_exist_ok=True)
            elif os.path.isfile(src):
                shutil.copy2(src, code)
            else:
                raise BackendError(f"rsync source {src!r} not found (and no rsync binary)")

    def _workdir(self, values: dict, jd: str) -> str:
        wd = os.path.join(jd, "work")
        os.makedirs(wd, exist_ok=True)
        code = os.path.join(jd, "code")
        link = os.path.join(wd, "code")
        if os.path.isdir(code) and not os.path.exists(link):
            os.symlink(code, link)
        want = values.get("workingDir", "")
        if want and os.path.isdir(want) and os.access(want, os.W_OK) and not values.get("syncMode"):
            return want
        return wd

    def _data_env(self, values: dict, jd: str) -> Dict[str, str]:
        env = {}
        mnt = os.path.join(jd, "mnt")
        for name, path in (values.get("dataset") or {}).items():
            host = os.path.join(self.home, "volumes", name)   # a local "PVC" is a directory
            os.makedirs(host, exist_ok=True)
            env[f"ARENA_DATA_{name.upper().replace('-', '_').replace('.', '_')}"] = host
            self._mount_link(mnt, path, host)
        for d in values.get("dataDirs") or []:
            env[f"ARENA_DATADIR_{d['name'].upper().replace('-', '_')}"] = d["hostPath"]
            self._mount_link(mnt, d["containerPath"], d["hostPath"])
        if env:
            env["ARENA_MOUNT_ROOT"] = mnt
        return env

    @staticmethod
    def _mount_link(mnt: str, ctr_path: str, host: str) -> None:
        target = os.path.join(mnt, ctr_path.lstrip("/"))
        os.makedirs(os.path.dirname(target), exist_ok=True)
        if not os.path.lexists(target):
            os.symlink(host, target)

    def _argv(self, command: List[str], values: dict, jd: str, pod: str) -> List[str]:
        argv = list(command)
        if argv[:2] == ["sh", "-c"]:
            argv[0] = "/bin/sh"
        if argv and argv[0] == "arena-jobmon":
            argv = [sys.executable, "-m", "arena_amd.runtime.jobmon"]
        if values.get("profileGPU") and shutil.which("rocprofv3") and argv[:2] == ["/bin/sh", "-c"]:
            script = argv[2]
            body = script.split("; ", 1)[-1] if script.startswith("export RANK=") else script
            if not (_SHELL_META & set(body)):
                # rocprofv3 must exec the program itself (no shell hop under its preload)
                tdir = os.path.join(jd, "traces", pod)
                os.makedirs(tdir, exist_ok=True)
                argv = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv",
                        "-d", tdir, "-o", "run", "--"] + shlex.split(body)
            else:
                log.warning("--profile-gpu: command of %s uses shell syntax; not profiled", pod)
        return argv

    def _plan(self, name, ns, chart, values, state: ClusterState, jd: str):
        inv = self.inventory()
        busy = self._busy_gpus(exclude=name)
        pods = sorted((p for p in state.pods.values() if p.meta.labels.get("role") != "jobmon"),
                      key=lambda p: (p.meta.labels.get("role") != "mpimaster", p.name))
        wd = self._workdir(values, jd)
        data_env = self._data_env(values, jd)
        tb_dir = os.path.join(jd, "tb")
        os.makedirs(tb_dir, exist_ok=True)
        gpus: Dict[str, List[int]] = {}
        hive = None
        for p in pods:
            need = sum(c.limits.get(r, 0) for c in p.containers for r in GPU_RESOURCES)
            if need:
                ids = pick_gpus(inv, busy, need, hive)
                busy.update(ids)
                gpus[p.name] = ids
                hive = next((str(g.get("hive_id")) for g in inv.get("gpus", [])
                             if g["index"] == ids[0]), hive)
        ports: Dict[str, int] = {}
        kind = {"training": "standalone", "tfjob": "tfjob", "tf-horovod": "allreduce"}[chart]
        base_env = {"ARENA_JOB_NAME": name, "ARENA_NAMESPACE": ns, "ARENA_JOB_DIR": jd,
                    "ARENA_TRAINING_LOGDIR": tb_dir, "ARENA_BACKEND": "local",
                    "ARENA_HOME": self.home, "PYTHONUNBUFFERED": "1",
                    "PYTHONPATH": REPO_ROOT + (os.pathsep + os.environ["PYTHONPATH"]
                                               if os.environ.get("PYTHONPATH") else ""),
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0", **data_env}
        launcher = ""
        rpp = max(1, int(values.get("ranksPerPod", 1)))
        if kind == "allreduce":
            ranks = [p for p in pods if p.meta.labels.get("role") in ("mpimaster", "mpiworker")]
            union = sorted({i for p in ranks for i in gpus.get(p.name, [])})
            port = _free_port()
            ports["rdzv"] = port
            launcher = next(p.name for p in ranks if p.meta.labels.get("role") == "mpimaster")
        if kind == "tfjob":
            for p in pods:
                if p.meta.labels.get("tf-replica-type"):
                    ports[p.name] = _free_port()
            cluster: Dict[str, list] = {}
            for p in sorted(pods, key=lambda q: (q.meta.labels.get("tf-replica-type", ""),
                                                 int(q.meta.labels.get("tf-replica-index", 0)))):
                t = p.meta.labels.get("tf-replica-type")
                if t:
                    cluster.setdefault(t, []).append(f"127.0.0.1:{ports[p.name]}")
        out_pods = []
        for p in pods:
            c = p.containers[0]
            env = dict(base_env)
            env.update(c.env)
            env["HOSTNAME"] = p.name
            env["ARENA_POD_NAME"] = p.name
            role = p.meta.labels.get("role") or p.meta.labels.get("tf-replica-type") or "job"
            long_running = role == "tensorboard"
            if long_running:
                tport = _free_port()
                ports["tensorboard"] = tport
                argv = [sys.executable, "-m", "arena_amd.tb.server", "--logdir", tb_dir,
                        "--port", str(tport), "--host", "0.0.0.0"]
            else:
                argv = self._argv(c.command, values, jd, p.name)
            own = gpus.get(p.name, [])
            if kind == "allreduce" and role in ("mpimaster", "mpiworker"):
                pidx = 0 if role == "mpimaster" else int(p.name.rsplit("-", 1)[1]) + 1
                env["MASTER_ADDR"] = "127.0.0.1"
                env["MASTER_PORT"] = str(ports["rdzv"])
                # every rank of every pod runs on this node
                env["LOCAL_WORLD_SIZE"] = str(len(ranks) * rpp)
                if union:
                    env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, union))
                    env["ARENA_RANK_GPUS"] = ",".join(str(union.index(i)) for i in own)
                if rpp == 1:
                    # the chart's `export RANK=...` prefix, resolved here as well: a
                    # --profile-gpu rank runs without the shell (rocprofv3 execs the program)
                    env["RANK"] = str(pidx)
                    env["LOCAL_RANK"] = str(union.index(own[0])) if (union and own) else "0"
                else:
                    # in-pod launcher (arena_amd.runtime.podlaunch) with node-wide local ranks:
                    # all ranks of the job see the job's whole GPU set and can map each other
                    env["ARENA_POD_INDEX"] = str(pidx)
                    env["ARENA_NODE_RANKS"] = str(len(ranks) * rpp)
                    env["ARENA_RANK_LOCAL_IDS"] = ",".join(
                        str(union.index(i)) for i in own[:rpp]) if (union and own) else \
                        ",".join(str(pidx * rpp + lr) for lr in range(rpp))
                    if not (role == "mpimaster" and values.get("jupyter")):
                        argv = [sys.executable, "-m", "arena_amd.runtime.podlaunch"]
                        if values.get("profileGPU"):
                            env["ARENA_RANK_PROFILE_DIR"] = os.path.join(jd, "traces", p.name)
            elif own:
                env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, own))
                env["LOCAL_RANK"] = "0"
            elif not own and kind != "allreduce":
                env.setdefault("HIP_VISIBLE_DEVICES", "")  # no GPU requested: none visible
            if kind == "tfjob" and p.meta.labels.get("tf-replica-type"):
                t = p.meta.labels["tf-replica-type"]
                idx = int(p.meta.labels.get("tf-replica-index", 0))
                spec = {"cluster": cluster, "task": {"type": t, "index": idx},
                        "environment": "cloud"}
                env["TF_CONFIG"] = json.dumps(spec)
                env["MX_CLUSTER_SPEC"] = env["TF_CONFIG"]
            hb = ""
            if float(values.get("heartbeatTimeout", 0) or 0) > 0 and not long_running:
                os.makedirs(os.path.join(jd, "heartbeat"), exist_ok=True)
                hb = os.path.join(jd, "heartbeat", p.name)
                env["ARENA_HEARTBEAT_FILE"] = hb
            out_pods.append({"name": p.name, "role": role, "argv": argv, "env": env, "cwd": wd,
                             "log": os.path.join(jd, "logs", p.name + ".log"),
                             "long_running": long_running, "heartbeat": hb})
        plan = {"kind": kind, "retry": int(values.get("retry", 0)), "launcher": launcher,
                "clean_pod_policy": values.get("cleanPodPolicy", "Running"),
                "restart_policy": values.get("restartPolicy", "Never"),
                "grace_s": float(values.get("gracePeriodSeconds", 5)),
                "heartbeat_timeout_s": float(values.get("heartbeatTimeout", 0) or 0),
                "pods": out_pods}
        return plan, gpus, ports

    # ------------------------------------------------------------------------ release store
    def release_exists(self, name) -> bool:
        return os.path.exists(os.path.join(self.job_dir(name), "release.json"))

    def get_release(self, name):
        rel = self._read_json(os.path.join(self.job_dir(name), "release.json"))
        if rel is None:
            return None
        return Release(rel["name"], rel["namespace"], rel["chart"], rel["values"],
                       rel["manifests"], rel["created"])

    def delete_release(self, name) -> None:
        jd = self.job_dir(name)
        if not self.release_exists(name):
            raise BackendError(f"release: \"{name}\" not found")
        st = self._read_json(os.path.join(jd, "state.json"), {}) or {}
        pid = int(st.get("supervisor_pid", 0) or 0)
        if not pid:
            try:
                pid = int(open(os.path.join(jd, "supervisor.pid")).read().strip())
            except (OSError, ValueError):
                pid = 0
        if _pid_alive(pid):
            try:
                open(os.path.join(jd, "control", "stop"), "w").close()
            except OSError:
                pass
            deadline = time.time() + 15
            while _pid_alive(pid) and time.time() < deadline:
                time.sleep(0.05)
            if _pid_alive(pid):
                try:
                    os.killpg(pid, signal.SIGKILL)
                except OSError:
                    pass
        try:  # reap it if it is our child (same-process submit + delete, as in tests)
            os.waitpid(pid, os.WNOHANG)
        except (ChildProcessError, OSError):
            pass
        shutil.rmtree(jd, ignore_errors=True)

    def list_releases(self) -> Dict[str, str]:
        out = {}
        for n in self._release_names():
            rel = self._read_json(os.path.join(self.job_dir(n), "release.json"), {}) or {}
            out[n] = rel.get("namespace", "default")
        return out

    # ------------------------------------------------------------------------- cluster view
    def _cluster(self, only: Optional[str] = None) -> ClusterState:
        """The cluster view rebuilt from the job store. ``only``: just that release (every
        object a release renders carries its ``release`` label, and each release's view is built
        independently), so a label query for one job reads one job's files, not the whole store."""
        full = ClusterState()
        node = self._node()
        full.nodes[node.name] = node
        names = self._release_names()
        if only is not None:
            names = [n for n in names if n == only]
        for name in names:
            rel = self._read_json(os.path.join(self.job_dir(name), "release.json"))
            if not rel:
                continue
            created = rel["created"]
            st = ClusterState(clock=lambda c=created: c)
            st.nodes = full.nodes
            st.apply(rel["manifests"])
            state = self._state(name)
            spods = state.get("pods") or {}
            finished = bool(state.get("finished")) or state.get("phase") in ("Succeeded", "Failed")
            for key, pod in list(st.pods.items()):
                if pod.meta.labels.get("role") == "jobmon":
                    # the supervisor implements jobmon natively: it "runs" until the job ends
                    pod.phase = POD_SUCCEEDED if finished else POD_RUNNING
                    pod.node_name, pod.host_ip = node.name, self.node_ip()
                    pod.start_time = created
                    continue
                ps = spods.get(pod.name)
                if ps is None:
                    continue
                if ps.get("deleted"):
                    del st.pods[key]
                    continue
                phase = ps.get("phase", POD_PENDING)
                pod.phase = phase if phase in (POD_PENDING, POD_RUNNING, POD_SUCCEEDED,
                                               POD_FAILED) else POD_FAILED
                if phase != POD_PENDING:
                    pod.node_name, pod.host_ip = node.name, self.node_ip()
                    pod.start_time = ps.get("start") or None
                ec = ps.get("exit_code", -1)
                pod.exit_code = None if ec is None or ec < 0 else ec
                pod.restart_count = int(ps.get("restarts", 0))
            # services: NodePort of the local TensorBoard = its real port
            for svc in st.services.values():
                if svc.meta.labels.get("role") == "tensorboard":
                    for p in svc.ports:
                        p.node_port = (rel.get("ports") or {}).get("tensorboard", 0)
            for key in rel.get("deleted_services", []):
                st.services.pop(tuple(key), None)
            st.reconcile()
            # the view is rebuilt per call: the operator's StartTime = the first task start
            starts = [ps.get("start") for ps in spods.values() if ps.get("start")]
            for tf in st.tfjobs.values():
                if tf.start_time is None and starts:
                    tf.start_time = min(starts)
            # a Job whose pods were all deleted keeps its terminal counters
            for job in st.jobs.values():
                if job.meta.labels.get("role") == "mpimaster" and state.get("phase") == "Failed":
                    if job.active == 0 and job.failed == 0:
                        job.failed = 1
            for store in ("pods", "jobs", "statefulsets", "services", "tfjobs", "endpoints"):
                getattr(full, store).update(getattr(st, store))
            # StatefulSets / Jobs deleted by jobmon disappear (their pods were killed)
            for key in rel.get("deleted_statefulsets", []):
                full.statefulsets.pop(tuple(key), None)
            for key in rel.get("deleted_jobs", []):
                full.jobs.pop(tuple(key), None)
        return full

    @staticmethod
    def _only(selector) -> Optional[str]:
        return selector.get("release") if selector else None

    def list_pods(self, namespace=None, selector=None, active_only=False):
        return [p for p in self._cluster(self._only(selector)).pods.values()
                if (not namespace or p.namespace == namespace) and matches(p.meta.labels, selector)
                and not (active_only and p.phase in (POD_SUCCEEDED, POD_FAILED))]

    def list_jobs(self, namespace=None, selector=None):
        return [j for j in self._cluster(self._only(selector)).jobs.values()
                if (not namespace or j.meta.namespace == namespace)
                and matches(j.meta.labels, selector)]

    def list_tfjobs(self, namespace=None, selector=None):
        return [t for t in self._cluster(self._only(selector)).tfjobs.values()
                if (not namespace or t.meta.namespace == namespace)
                and matches(t.meta.labels, selector)]

    def list_nodes(self):
        return [self._node()]

    def list_services(self, namespace, selector=None):
        return [s for s in self._cluster(self._only(selector)).services.values()
                if s.meta.namespace == namespace and matches(s.meta.labels, selector)]

    _DASHBOARDS = ("kubernetes-dashboard", "tf-job-dashboard")

    def get_endpoints(self, namespace, name):
        if name in self._DASHBOARDS:
            lv = self._logviewer()
            if lv is None:
                return None
            return Endpoints(meta=Meta(name=name, namespace=namespace),
                             addresses=[self.node_ip()], ports=[lv["port"]])
        return self._cluster().endpoints.get((namespace, name))

    def _logviewer(self) -> Optional[dict]:
        info = self._read_json(os.path.join(self.home, "logviewer.json"))
        if info and _pid_alive(int(info.get("pid", 0))):
            return info
        return None

    def ensure_logviewer(self, timeout_s: float = 10.0) -> Optional[dict]:
        """Start the built-in log viewer (arena_amd.runtime.logviewer) once per job store."""
        info = self._logviewer()
        if info is not None:
            return info
        ready = os.path.join(self.home, "logviewer.json")
        try:
            os.unlink(ready)
        except OSError:
            pass
        env = dict(os.environ)
        env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        with open(os.path.join(self.home, "logviewer.log"), "ab") as lf:
            subprocess.Popen([sys.executable, "-m", "arena_amd.runtime.logviewer", "--home", self.home,
                              "--port", os.environ.get("ARENA_LOGVIEWER_PORT", "0"),
                              "--ready-file", ready],
                             stdin=subprocess.DEVNULL, stdout=lf, stderr=lf, start_new_session=True,
                             env=env, close_fds=True)
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            info = self._logviewer()
            if info is not None:
                return info
            time.sleep(0.05)
        return None

    def get_pod(self, namespace, name):
        return self._cluster().pods.get((namespace, name))

    def get_job(self, namespace, name):
        return self._cluster().jobs.get((namespace, name))

    def get_statefulset(self, namespace, name):
        return self._cluster().statefulsets.get((namespace, name))

    def _release_of(self, namespace, name, store) -> Optional[str]:
        obj = getattr(self._cluster(), store).get((namespace, name))
        return obj.meta.labels.get("release") if obj is not None else None

    def delete_statefulset(self, namespace, name):
        rel_name = self._release_of(namespace, name, "statefulsets")
        if rel_name is None:
            raise BackendError(f"statefulsets \"{name}\" not found")
        jd = self.job_dir(rel_name)
        for p in self.list_pods(namespace, {"release": rel_name, "role": "mpiworker"}):
            open(os.path.join(jd, "control", f"kill-{p.name}"), "w").close()
        self._append_rel_list(rel_name, "deleted_statefulsets", [namespace, name])

    def delete_job(self, namespace, name):
        rel_name = self._release_of(namespace, name, "jobs")
        if rel_name is None:
            raise BackendError(f"jobs.batch \"{name}\" not found")
        jd = self.job_dir(rel_name)
        for p in self.list_pods(namespace, {"release": rel_name}):
            if "Job" in p.meta.owner_kinds and p.name.rsplit("-", 1)[0] == name:
                open(os.path.join(jd, "control", f"kill-{p.name}"), "w").close()
        self._append_rel_list(rel_name, "deleted_jobs", [namespace, name])

    def delete_service(self, namespace, name):
        rel_name = self._release_of(namespace, name, "services")
        if rel_name is None:
            raise BackendError(f"services \"{name}\" not found")
        self._append_rel_list(rel_name, "deleted_services", [namespace, name])

    def _append_rel_list(self, rel_name, key, item):
        path = os.path.join(self.job_dir(rel_name), "release.json")
        rel = self._read_json(path, {})
        rel.setdefault(key, []).append(item)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(rel, f, indent=1)
        os.replace(tmp, path)

    def ensure_namespace(self, namespace):
        return None

    def pod_logs(self, namespace, pod, follow=False, since_seconds=None, since_time=None,
                 tail=-1, timestamps=False) -> Iterator[str]:
        p = self.get_pod(namespace, pod)
        if p is None:
            raise BackendError(f"pods \"{pod}\" not found")
        rel = p.meta.labels.get("release", "")
        path = os.path.join(self.job_dir(rel), "logs", pod + ".log")
        cutoff = None
        if since_seconds is not None:
            cutoff = time.time() - since_seconds
        if since_time is not None:
            cutoff = max(cutoff or since_time, since_time)

        def fmt(raw: str) -> Optional[str]:
            ts, _, text = raw.rstrip("\n").partition(" ")
            if cutoff is not None:
                try:
                    if parse_rfc3339(ts[:26] + "Z" if len(ts) > 27 else ts) < cutoff:
                        return None
                except ValueError:
                    pass
            return (f"{ts} {text}\n" if timestamps else f"{text}\n")

        lines: List[str] = []
        pos = 0
        if os.path.exists(path):
            with open(path, errors="replace") as f:
                lines = f.readlines()
                pos = f.tell()
        out = [x for x in (fmt(r) for r in lines) if x is not None]
        if tail is not None and tail >= 0:
            out = out[-tail:] if tail else []
        yield from out
        if not follow:
            return
        partial = ""
        while True:
            grew = False
            if os.path.exists(path):
                with open(path, errors="replace") as f:
                    f.seek(pos)
                    chunk = f.read()
                    pos = f.tell()
                if chunk:
                    grew = True
                    partial += chunk
                    *full, partial = partial.split("\n")
                    for r in full:
                        x = fmt(r)
                        if x is not None:
                            yield x
            if not grew:
                cur = self.get_pod(namespace, pod)
                if cur is None or cur.phase in (POD_SUCCEEDED, POD_FAILED):
                    return
                time.sleep(0.2)

    # ----------------------------------------------------------------------------- telemetry
    def node_telemetry(self, node: str) -> Optional[dict]:
        inv = probe_gpus() if os.environ.get("ARENA_LOCAL_GPUS") is None else None
        if not inv or not inv.get("gpus"):
            return None
        busy = [g.get("busy_percent", -1) for g in inv["gpus"] if g.get("busy_percent", -1) >= 0]
        used = sum(max(g.get("vram_used", 0), 0) for g in inv["gpus"])
        total = sum(max(g.get("vram_total", 0), 0) for g in inv["gpus"])
        power = [g.get("power_uw", -1) for g in inv["gpus"] if g.get("power_uw", -1) >= 0]
        return {"busy": f"{sum(busy) // len(busy)}%" if busy else "N/A",
                "vram": f"{used / 2**30:.0f}/{total / 2**30:.0f}" if total else "N/A",
                "power": f"{sum(power) / 1e6:.0f}" if power else "N/A"}   # node total
