"""The `arena` command tree (reference: cmd/arena/commands/*.go).

Command names, aliases, flags and defaults follow the reference; quirks fixed where SURVEY §2.14
recommends (Q1 standalone installs once, Q2 delete loops over all names, Q3 errors propagate,
Q8 --timestamps honoured, Q9 --since takes durations, Q10 namespace parameter respected,
Q11 jobmon reaps on failure, Q13 message, Q16 InternalIP). Each command returns an exit code.
"""
from __future__ import annotations

import argparse
import sys
import time
from typing import List

from .. import version as _version
from ..cluster.backend import BackendError
from ..jobs import spec as S
from ..jobs.nodes import describe_nodes
from ..jobs.tensorboard import tensorboard_url
from ..jobs.trainer import (ClusterCache, get_training_job, new_trainers, order_by_age,
                            order_by_gpu)
from ..utils.duration import parse_duration
from ..utils.errors import ArenaError
from ..utils.logs import get_logger, set_log_level
from ..utils.timefmt import parse_rfc3339
from ..utils.validate import ValidationError
from . import display

log = get_logger("cli")


class _Ctx:
    """Per-invocation context: parsed globals + lazily created backend."""

    def __init__(self, args, backend=None, out=None):
        self.args = args
        self._backend = backend
        self.out = out or sys.stdout

    @property
    def backend(self):
        if self._backend is None:
            from .backends import make_backend
            self._backend = make_backend(self.args)
        return self._backend

    @property
    def namespace(self) -> str:
        return self.args.namespace


# ------------------------------------------------------------------------------------ submit
def _add_common_flags(p: argparse.ArgumentParser) -> None:
    p.add_argument("--name", required=True, help="override name")
    p.add_argument("--image", default="", help="the container image of the training job")
    p.add_argument("--gpus", type=int, default=0,
                   help="the GPU count of each worker to run the training.")
    p.add_argument("--workers", type=int, default=1,
                   help="the worker number to run the distributed training.")
    p.add_argument("--retry", type=int, default=0, help="retry times.")
    p.add_argument("--workingDir", default="/root",
                   help="working directory to extract the code. If using syncMode, the "
                        "$workingDir/code contains the code")
    p.add_argument("-e", "--env", action="append", default=[], help="the environment variables")
    p.add_argument("-d", "--data", action="append", default=[],
                   help="specify the datasource to mount to the job, like "
                        "<name_of_datasource>:<mount_point_on_job>")
    p.add_argument("--dataDir", action="append", default=[],
                   help="the data dir. If you specify /data, it means mounting hostpath /data "
                        "into container path /data")
    p.add_argument("--gpuResource", default="amd.com/gpu",
                   help="extended resource name of the GPUs (MI355X: amd.com/gpu)")
    p.add_argument("--profile-gpu", dest="profile_gpu", action="store_true",
                   help="run the ranks under rocprofv3 --kernel-trace --stats; traces go to "
                        "<job dir>/traces/")
    p.add_argument("--heartbeatTimeout", type=float, default=0.0,
                   help="seconds without training progress (arena_amd.runtime.heartbeat beats) "
                        "after which a rank counts as hung and is killed, so the retry policy "
                        "applies; 0 disables")
    p.add_argument("command", nargs=argparse.REMAINDER, help="the training command")


def _add_sync_flags(p):
    p.add_argument("--syncMode", default="", help="syncMode: support rsync, git")
    p.add_argument("--syncSource", default="",
                   help="syncSource: for rsync, a path or host::module/path; for git, a repo url")
    p.add_argument("--syncImage", default="", help="the container image of syncImage")


def _add_tensorboard_flags(p, tf_defaults=True):
    p.add_argument("--tensorboard", action="store_true", help="enable tensorboard")
    p.add_argument("--tensorboardImage", default=S.DEFAULT_TENSORBOARD_IMAGE,
                   help="the image of tensorboard")
    p.add_argument("--logdir", default="/training_logs", help="the training logs dir")


def _fill_common(a: S.SubmitArgs, ns) -> S.SubmitArgs:
    a.name = ns.name
    a.image = ns.image
    a.gpu_count = ns.gpus
    a.workers = ns.workers
    a.retry = ns.retry
    a.working_dir = ns.workingDir
    a.env_list = list(ns.env)
    a.dataset_list = list(ns.data)
    a.data_dir_list = list(ns.dataDir)
    a.gpu_resource = ns.gpuResource
    a.profile_gpu = ns.profile_gpu
    a.heartbeat_timeout = ns.heartbeatTimeout
    return a


def _fill_sync_tb(a, ns):
    a.sync = S.SyncCodeArgs(sync_mode=ns.syncMode, sync_source=ns.syncSource,
                            sync_image=ns.syncImage)
    a.tensorboard = S.TensorboardArgs(use_tensorboard=ns.tensorboard,
                                      tensorboard_image=ns.tensorboardImage,
                                      training_logdir=ns.logdir)


def _command_args(ns) -> List[str]:
    cmd = list(ns.command)
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    return cmd


def _submit(ctx: _Ctx, a: S.SubmitArgs, cmd: List[str]) -> int:
    a.namespace = ctx.namespace
    b = ctx.backend
    if not a.image and getattr(b, "name", "") == "local":
        a.image = "local"   # processes on this host: there is no container image to pull
    a.prepare(cmd)
    b.ensure_namespace(ctx.namespace)
    if b.release_exists(a.name):
        raise ArenaError(f"the job {a.name} is already exist, please delete it first. "
                         f"use 'arena delete {a.name}'")
    rel = b.install_release(a.name, ctx.namespace, a.chart, a.values())
    display.release_summary(ctx.out, rel)
    return 0


def cmd_submit_tf(ctx, ns) -> int:
    a = _fill_common(S.TFJobArgs(), ns)
    a.port = ns.port
    a.worker_image = ns.workerImage
    a.ps_image = ns.psImage
    a.ps_count = ns.ps
    a.ps_port = ns.psPort
    a.worker_port = ns.workerPort
    a.worker_cpu, a.worker_memory = ns.workerCpu, ns.workerMemory
    a.ps_cpu, a.ps_memory = ns.psCpu, ns.psMemory
    a.clean_pod_policy = ns.cleanTaskPolicy
    a.tf_operator = ns.tfOperator
    _fill_sync_tb(a, ns)
    return _submit(ctx, a, _command_args(ns))


def cmd_submit_mpi(ctx, ns) -> int:
    a = _fill_common(S.MPIJobArgs(), ns)
    a.cpu, a.memory = ns.cpu, ns.memory
    a.ssh_port = ns.sshPort
    a.rdzv_port = ns.rdzvPort
    a.shm_size = ns.shmSize
    a.ranks_per_pod = ns.ranksPerPod
    a.jupyter = ns.jupyter
    _fill_sync_tb(a, ns)
    rc = _submit(ctx, a, _command_args(ns))
    rpp = a.effective_ranks_per_pod()
    if rpp > 1 and getattr(ctx.backend, "name", "") != "local":
        # the pods' entry point is now the in-pod launcher, which runs inside the user's image
        log.warning(f"each pod starts {rpp} ranks (one per GPU) through `python3 -m "
                    f"arena_amd.runtime.podlaunch`: the image {a.image!r} must have arena_amd "
                    f"installed (pods exit 127 with a message otherwise); --ranksPerPod 1 runs "
                    f"the command once per pod as given")
    return rc


def cmd_submit_sj(ctx, ns) -> int:
    log.warning("standalonejob is deprecated; it may be removed in a future release")
    a = _fill_common(S.StandaloneJobArgs(), ns)
    a.cpu, a.memory = ns.cpu, ns.memory
    _fill_sync_tb(a, ns)
    return _submit(ctx, a, _command_args(ns))   # Q1 fixed: installed exactly once


# -------------------------------------------------------------------------------- list / get
def _all_jobs(ctx) -> list:
    b = ctx.backend
    releases = b.list_releases()
    cache = ClusterCache(b)
    trainers = new_trainers(b, cache)
    jobs = []
    for name, ns in releases.items():
        for t in trainers:
            if t.is_supported(name, ns):
                jobs.append(t.get_training_job(name, ns))
                break
        else:
            log.debug("Unknown chart %s", name)
    return jobs


def cmd_list(ctx, ns) -> int:
    display.training_job_list(ctx.out, order_by_age(_all_jobs(ctx)), False)
    return 0


def cmd_top_job(ctx, ns) -> int:
    display.training_job_list(ctx.out, order_by_gpu(_all_jobs(ctx)), True)
    return 0


def cmd_get(ctx, ns) -> int:
    name = ns.job
    b = ctx.backend
    if not b.release_exists(name):
        ctx.out.write(f"The job {name} doesn't exist, please create it first. use 'arena submit'\n")
        return 1
    job = get_training_job(b, name, ctx.namespace)
    if ns.output == "name":
        ctx.out.write(job.name() + "\n")
        return 0
    if ns.output not in ("", "wide"):
        raise ArenaError(f"Unknown output format: {ns.output}")
    url = tensorboard_url(b, name, job.namespace())
    display.single_job(ctx.out, job, url)
    return 0


def cmd_logviewer(ctx, ns) -> int:
    name = ns.job
    b = ctx.backend
    if not b.release_exists(name):
        ctx.out.write(f"The job {name} doesn't exist, please create it first. use 'arena submit'\n")
        return 1
    job = get_training_job(b, name, ctx.namespace)
    if hasattr(b, "ensure_logviewer"):
        b.ensure_logviewer()   # local backend: the built-in viewer stands in for the dashboards
    try:
        urls = job.get_job_dashboards(b, ctx.args.arenaNamespace)
    except LookupError as e:
        ctx.out.write(f"{e}\n")
        return 1
    if not urls:
        ctx.out.write(f"No logviewer found for job {name}\n")
        return 1
    ctx.out.write("Your LogViewer will be available on:\n")
    for u in urls:
        ctx.out.write(u + "\n")
    return 0


# -------------------------------------------------------------------------------------- logs
def cmd_logs(ctx, ns) -> int:
    name = ns.job
    b = ctx.backend
    job = get_training_job(b, name, ctx.namespace)
    pod = job.chief_pod()
    if ns.instance:
        pod = next((p for p in job.all_pods() if p.name == ns.instance), None)
        if pod is None:
            raise ArenaError(f"Failed to find instance {ns.instance} in job {name}")
    if pod is None:
        raise ArenaError(f"Failed to find the chief pod of job {name}")
    since_seconds = parse_duration(ns.since) if ns.since else None
    since_time = parse_rfc3339(ns.since_time) if ns.since_time else None
    # ensureContainerStarted (logs.go:198): a few quick polls for a pending pod
    for _ in range(5):
        p = b.get_pod(pod.namespace, pod.name)
        if p is None or p.phase != "Pending":
            break
        time.sleep(0.001)
    for line in b.pod_logs(pod.namespace, pod.name, follow=ns.follow, since_seconds=since_seconds,
                           since_time=since_time, tail=ns.tail, timestamps=ns.timestamps):
        ctx.out.write(line)
        if ns.follow:
            ctx.out.flush()
    return 0


# ------------------------------------------------------------------------------------ delete
def cmd_delete(ctx, ns) -> int:
    rc = 0
    for name in ns.jobs:   # Q2 fixed: every name, not just the first
        try:
            ctx.backend.delete_release(name)
            ctx.out.write(f"release \"{name}\" deleted\n")
        except Exception as e:  # noqa: BLE001
            ctx.out.write(f"Failed to delete {name}: {e}\n")
            rc = 1
    return rc


# --------------------------------------------------------------------------------------- top
def cmd_top_node(ctx, ns) -> int:
    infos = describe_nodes(ctx.backend)
    if ns.details:
        display.top_node_details(ctx.out, infos)
    else:
        tel = {i.node.name: ctx.backend.node_telemetry(i.node.name) for i in infos}
        display.top_node_summary(ctx.out, infos, tel)
    return 0


# ----------------------------------------------------------------------------------- version
def cmd_version(ctx, ns) -> int:
    v = _version.get_version()
    if ns.short:
        ctx.out.write(f"{v['version']}\n")
        return 0
    for k in ("version", "buildDate", "gitCommit", "gitTreeState", "gitTag", "pythonVersion",
              "torchVersion", "rocmVersion", "platform"):
        label = {"version": "Version", "buildDate": "BuildDate", "gitCommit": "GitCommit",
                 "gitTreeState": "GitTreeState", "gitTag": "GitTag",
                 "pythonVersion": "PythonVersion", "torchVersion": "TorchVersion",
                 "rocmVersion": "ROCmVersion", "platform": "Platform"}[k]
        ctx.out.write(f"{label}: {v.get(k, '')}\n")
    return 0


def cmd_completion(ctx, ns) -> int:
    from .completion import completion_script
    ctx.out.write(completion_script(ns.shell, build_parser()))
    return 0


# ------------------------------------------------------------------------------------ parser
def _add_global_flags(p: argparse.ArgumentParser, defaults: bool) -> None:
    def d(v):
        return v if defaults else argparse.SUPPRESS
    p.add_argument("--config", default=d(""), help="Path to a kube config. Only required if "
                                                    "out-of-cluster (k8s backend)")
    p.add_argument("--namespace", default=d("default"), help="the namespace of the job")
    p.add_argument("--loglevel", default=d("info"), help="Set the logging level. One of: "
                                                          "debug|info|warn|error")
    p.add_argument("--pprof", action="store_true", default=d(False),
                   help="enable cpu profile (/tmp/cpu_profile)")
    p.add_argument("--arenaNamespace", default=d("arena-system"),
                   help="The namespace of arena system service, like TFJob")
    p.add_argument("--backend", default=d(None),
                   help="local | k8s (default: $ARENA_BACKEND or local)")
    p.add_argument("--home", default=d(None), help="job store directory (default: $ARENA_HOME "
                                                   "or ~/.arena)")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog="arena",
        description="arena is the command line interface to Arena (MI355X-native): submit, "
                    "monitor and manage training jobs on AMD Instinct GPUs.")
    _add_global_flags(p, defaults=True)
    # cobra persistent flags (root.go:39-44,60-70) are accepted after any subcommand too:
    # every subparser inherits the global flags with SUPPRESS defaults, so a flag given after
    # the subcommand overrides the root value and an absent one leaves it untouched.
    glob = argparse.ArgumentParser(add_help=False)
    _add_global_flags(glob, defaults=False)
    _orig_sub = argparse._SubParsersAction.add_parser  # noqa: SLF001

    def _add_parser(self, name, **kw):
        kw.setdefault("parents", []).append(glob)
        return _orig_sub(self, name, **kw)

    sub = p.add_subparsers(dest="cmd", metavar="COMMAND")
    sub.add_parser = _add_parser.__get__(sub)

    sp = sub.add_parser("submit", help="Submit a job.")
    ssub = sp.add_subparsers(dest="kind", metavar="KIND")
    ssub.add_parser = _add_parser.__get__(ssub)
    tf = ssub.add_parser("tfjob", aliases=["tf"], help="Submit a parameter-server/worker job.")
    _add_common_flags(tf)
    _add_sync_flags(tf)
    _add_tensorboard_flags(tf)
    tf.add_argument("--workerImage", default="", help="the image of the worker")
    tf.add_argument("--psImage", default="", help="the image of the PS")
    tf.add_argument("--ps", type=int, default=0, help="the number of the parameter servers.")
    tf.add_argument("--port", type=int, default=0, help="port for PS and workers when not set")
    tf.add_argument("--psPort", type=int, default=22223, help="the port of the parameter server.")
    tf.add_argument("--workerPort", type=int, default=22222, help="the port of the worker.")
    tf.add_argument("--workerCpu", default="", help="the cpu resource to use for the worker")
    tf.add_argument("--workerMemory", default="", help="the memory resource for the worker")
    tf.add_argument("--psCpu", default="", help="the cpu resource to use for the PS")
    tf.add_argument("--psMemory", default="", help="the memory resource for the PS")
    tf.add_argument("--cleanTaskPolicy", default="Running",
                    help="How to clean tasks after Training is done, only support Running, None.")
    tf.add_argument("--tfOperator", action="store_true",
                    help="render a kubeflow.org TFJob for a cluster running tf-operator, instead "
                         "of the built-in per-task Jobs + headless Services")
    tf.set_defaults(func=cmd_submit_tf)

    mpi = ssub.add_parser("mpijob", aliases=["mpi"], help="Submit an allreduce (MPI) job.")
    _add_common_flags(mpi)
    _add_sync_flags(mpi)
    _add_tensorboard_flags(mpi)
    mpi.add_argument("--cpu", default="", help="the cpu resource to use for the training")
    mpi.add_argument("--memory", default="", help="the memory resource to use for the training")
    mpi.add_argument("--sshPort", type=int, default=33, help="ssh port (kept for compatibility)")
    mpi.add_argument("--rdzvPort", type=int, default=29500,
                     help="TCPStore rendezvous port served by rank 0")
    mpi.add_argument("--shmSize", default="2Gi", help="size of the /dev/shm tmpfs per rank")
    mpi.add_argument("--ranksPerPod", type=int, default=-1,
                     help="data-parallel ranks per pod (default: one per GPU, as hvd-distribute.sh "
                          "<hosts> <gpus>; 1 for CPU pods). WORLD_SIZE = workers x ranksPerPod")
    mpi.add_argument("--jupyter", action="store_true",
                     help="run the launcher pod as a Jupyter notebook server (port 8888, "
                          "<job>-tf-horovod-jupyter Service) instead of the command; the worker "
                          "pods idle until ranks are started from the notebook")
    mpi.set_defaults(func=cmd_submit_mpi)

    sj = ssub.add_parser("standalonejob", aliases=["sj"], help="Submit a standalone job.")
    _add_common_flags(sj)
    _add_sync_flags(sj)
    _add_tensorboard_flags(sj)
    sj.add_argument("--cpu", default="", help="the cpu resource to use for the training")
    sj.add_argument("--memory", default="", help="the memory resource to use for the training")
    sj.set_defaults(func=cmd_submit_sj)

    ls = sub.add_parser("list", help="list all the training jobs")
    ls.set_defaults(func=cmd_list)

    g = sub.add_parser("get", help="display details of a training job")
    g.add_argument("job")
    g.add_argument("-o", "--output", default="", help="Output format. One of: wide|name")
    g.set_defaults(func=cmd_get)

    lv = sub.add_parser("logviewer", help="display Log Viewer URL of a training job")
    lv.add_argument("job")
    lv.set_defaults(func=cmd_logviewer)

    lg = sub.add_parser("logs", help="print the logs for a task of the training job")
    lg.add_argument("job")
    lg.add_argument("-f", "--follow", action="store_true", help="Specify if the logs should be "
                                                                "streamed.")
    lg.add_argument("--since", default="", help="Only return logs newer than a relative duration "
                                                "like 5s, 2m, or 3h. Defaults to all logs.")
    lg.add_argument("--since-time", dest="since_time", default="",
                    help="Only return logs after a specific date (RFC3339).")
    lg.add_argument("--tail", type=int, default=-1, help="Lines of recent log file to display.")
    lg.add_argument("--timestamps", action="store_true",
                    help="Include timestamps on each line in the log output")
    lg.add_argument("-i", "--instance", default="", help="Specify the task instance to get log")
    lg.set_defaults(func=cmd_logs)

    d = sub.add_parser("delete", help="delete a training job and its associated pods")
    d.add_argument("jobs", nargs="+")
    d.set_defaults(func=cmd_delete)

    tp = sub.add_parser("top", help="Display Resource (GPU) usage.")
    tsub = tp.add_subparsers(dest="topkind", metavar="KIND")
    tsub.add_parser = _add_parser.__get__(tsub)
    tn = tsub.add_parser("node", help="Display Resource (GPU) usage of nodes")
    tn.add_argument("-d", "--details", action="store_true", help="Display details")
    tn.set_defaults(func=cmd_top_node)
    tj = tsub.add_parser("job", help="Display Resource (GPU) usage of jobs")
    tj.set_defaults(func=cmd_top_job)

    v = sub.add_parser("version", help="Print version information")
    v.add_argument("--short", action="store_true", help="print just the version number")
    v.set_defaults(func=cmd_version)

    c = sub.add_parser("completion", help="output shell completion code for bash or zsh")
    c.add_argument("shell", choices=["bash", "zsh"])
    c.set_defaults(func=cmd_completion)
    return p


def run(argv: List[str], backend=None, out=None) -> int:
    parser = build_parser()
    args = parser.parse_args(argv)
    set_log_level(args.loglevel)
    func = getattr(args, "func", None)
    if func is None:
        target = parser
        if args.cmd == "submit":
            target = parser._subparsers._group_actions[0].choices["submit"]  # noqa: SLF001
        elif args.cmd == "top":
            target = parser._subparsers._group_actions[0].choices["top"]  # noqa: SLF001
        target.print_help(out or sys.stdout)
        return 0 if args.cmd is None else 1
    ctx = _Ctx(args, backend, out)
    try:
        return func(ctx, args)
    except (ArenaError, ValidationError, LookupError, BackendError) as e:
        (out or sys.stdout).write(f"{e}\n")
        return 1
