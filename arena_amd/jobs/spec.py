"""Submit arguments -> chart values (reference: submit.go:25-124, submit_tfjob.go:82-207,
submit_horovod.go:63-116, submit_standalone.go:63-140, sync_code.go:11-54, tensorboard.go:11-16).

The values dict uses the reference's YAML keys so a values file written by either
tool reads the same, plus MI355X-native keys (``gpuResource``, ``devices``, ``shmSize``,
``rdzvPort``). Quirks fixed here: Q3 (transform errors are raised, not swallowed), Q5 (psCPU is the
one key used everywhere), Q7 (git sync works for every job kind).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..cluster.objects import AMD_GPU
from ..utils.random import random_int32
from ..utils.validate import ValidationError, validate_job_name
from ..utils.volume import parse_data_dir_raw, validate_datasets

DEFAULT_IMAGE = "rocm/pytorch:latest"
DEFAULT_TENSORBOARD_IMAGE = "rocm/tensorboard:latest"
DEFAULT_SYNC_IMAGE = "alpine/git:latest"

TF_CHART, MPI_CHART, STANDALONE_CHART = "tfjob", "tf-horovod", "training"


def transform_slice_to_map(items: List[str], sep: str) -> Dict[str, str]:
    """Split each item on the FIRST separator (submit.go:160-170); items without it are skipped."""
    out: Dict[str, str] = {}
    for it in items:
        k, s, v = it.partition(sep)
        if s:
            out[k] = v
    return out


@dataclass
class SyncCodeArgs:
    sync_mode: str = ""          # "" | git | rsync
    sync_source: str = ""
    sync_image: str = ""
    sync_git_project_name: str = ""

    def handle(self) -> None:
        if self.sync_mode == "":
            return
        if self.sync_mode not in ("git", "rsync"):
            raise ValidationError(f"Unknown sync mode: {self.sync_mode}, it should be git or rsync")
        if not self.sync_source:
            raise ValidationError("--syncSource should be set when syncMode is set")
        if self.sync_mode == "git":
            last = self.sync_source.strip("/").split("/")[-1]
            self.sync_git_project_name = last.split(".git")[0]
            if not self.sync_image:
                self.sync_image = DEFAULT_SYNC_IMAGE  # Q7: git sync needs an image everywhere

    def values(self) -> dict:
        v = {"syncMode": self.sync_mode, "syncSource": self.sync_source}
        if self.sync_image:
            v["syncImage"] = self.sync_image
        if self.sync_git_project_name:
            v["syncGitProjectName"] = self.sync_git_project_name
        return v


@dataclass
class TensorboardArgs:
    use_tensorboard: bool = False
    tensorboard_image: str = DEFAULT_TENSORBOARD_IMAGE
    training_logdir: str = "/training_logs"
    host_log_path: str = ""

    def transform(self) -> None:
        if self.use_tensorboard and not self.host_log_path:
            self.host_log_path = f"/arena_logs/training{random_int32()}"

    def values(self) -> dict:
        return {"useTensorboard": self.use_tensorboard, "tensorboardImage": self.tensorboard_image,
                "trainingLogdir": self.training_logdir, "hostLogPath": self.host_log_path}


@dataclass
class SubmitArgs:
    """Fields shared by every job kind (submitArgs, submit.go:25-46)."""
    name: str = ""
    namespace: str = "default"
    image: str = ""
    gpu_count: int = 0
    envs: Dict[str, str] = field(default_factory=dict)
    working_dir: str = "/root"
    command: str = ""
    mode: str = ""
    workers: int = 1
    retry: int = 0
    dataset: Dict[str, str] = field(default_factory=dict)
    data_dirs: List[dict] = field(default_factory=list)
    # raw CLI inputs
    env_list: List[str] = field(default_factory=list)
    dataset_list: List[str] = field(default_factory=list)
    data_dir_list: List[str] = field(default_factory=list)
    # MI355X-native placement/runtime knobs
    gpu_resource: str = AMD_GPU
    profile_gpu: bool = False
    heartbeat_timeout: float = 0.0   # hang detection (0 = off), see arena_amd/runtime/heartbeat.py

    def check(self) -> None:
        if not self.name:
            raise ValidationError("--name must be set")
        validate_job_name(self.name)
        if self.gpu_count < 0:
            raise ValidationError("--gpus must be >= 0")
        if self.retry < 0:
            raise ValidationError("--retry must be >= 0")
        if self.heartbeat_timeout < 0:
            raise ValidationError("--heartbeatTimeout must be >= 0")

    def transform(self) -> None:
        if self.data_dir_list:
            self.data_dirs = []
            for i, raw in enumerate(self.data_dir_list):
                host, ctr = parse_data_dir_raw(raw)
                self.data_dirs.append({"name": f"training-data-{i}", "hostPath": host,
                                       "containerPath": ctr})
        if self.dataset_list:
            validate_datasets(self.dataset_list)
            self.dataset = transform_slice_to_map(self.dataset_list, ":")

    def apply_envs(self) -> None:
        # Q4 kept: --env replaces the map, then workers/gpus are injected (submit.go:96-102)
        if self.env_list:
            self.envs = transform_slice_to_map(self.env_list, "=")
        self.envs = dict(self.envs)
        self.envs["workers"] = str(self.workers)
        self.envs["gpus"] = str(self.gpu_count)

    def values(self) -> dict:
        v = {"image": self.image, "gpuCount": self.gpu_count, "envs": dict(self.envs),
             "workingDir": self.working_dir, "command": self.command, "mode": self.mode,
             "workers": self.workers, "retry": self.retry, "dataset": dict(self.dataset),
             "dataDirs": copy.deepcopy(self.data_dirs), "gpuResource": self.gpu_resource,
             "devices": ["/dev/kfd", "/dev/dri"], "profileGPU": self.profile_gpu}
        if self.heartbeat_timeout > 0:
            v["heartbeatTimeout"] = self.heartbeat_timeout
        return v


@dataclass
class TFJobArgs(SubmitArgs):
    """Parameter-server/worker job (submitTFJobArgs, submit_tfjob.go:82-103)."""
    port: int = 0
    worker_image: str = ""
    worker_port: int = 22222
    ps_port: int = 22223
    ps_count: int = 0
    ps_image: str = ""
    worker_cpu: str = ""
    worker_memory: str = ""
    ps_cpu: str = ""
    ps_memory: str = ""
    clean_pod_policy: str = "Running"
    tf_operator: bool = False   # render a kubeflow.org TFJob for tf-operator instead of Jobs
    tensorboard: TensorboardArgs = field(default_factory=TensorboardArgs)
    sync: SyncCodeArgs = field(default_factory=SyncCodeArgs)
    chart: str = TF_CHART

    def prepare(self, args: List[str]) -> None:
        """Order matters and follows submit_tfjob.go:105-136."""
        self.command = " ".join(args)
        if self.worker_port == 0:
            self.worker_port = self.port
        if not self.worker_image:
            self.worker_image = self.image
        if self.ps_count > 0:
            if self.ps_port == 0:
                self.ps_port = self.port
            if not self.ps_image:
                self.ps_image = self.image
        self.tensorboard.transform()
        self.check()
        self.sync.handle()
        self.transform()
        self.apply_envs()

    def check(self) -> None:
        super().check()
        if self.clean_pod_policy not in ("None", "Running"):
            raise ValidationError(f"Unsupported cleanTaskPolicy {self.clean_pod_policy}")
        if self.workers == 0:
            raise ValidationError("--workers must be greater than 0")
        if not self.worker_image:
            raise ValidationError("--image or --workerImage must be set")
        if self.workers + self.ps_count > 1 and self.worker_port <= 0:
            raise ValidationError("--port or --workerPort must be set")
        if self.ps_count > 0:
            if not self.ps_image:
                raise ValidationError("--image or --psImage must be set")
            if self.ps_port <= 0:
                raise ValidationError("--port or --psPort must be set")

    def values(self) -> dict:
        v = super().values()
        v.update({"port": self.port, "workerImage": self.worker_image,
                  "workerPort": self.worker_port, "psPort": self.ps_port, "ps": self.ps_count,
                  "psImage": self.ps_image, "workerCPU": self.worker_cpu,
                  "workerMemory": self.worker_memory, "psCPU": self.ps_cpu,
                  "psMemory": self.ps_memory, "cleanPodPolicy": self.clean_pod_policy})
        if self.tf_operator:
            v["tfOperator"] = True
        v.update(self.tensorboard.values())
        v.update(self.sync.values())
        return v


@dataclass
class MPIJobArgs(SubmitArgs):
    """Allreduce (Horovod-style) job (submitHorovodJobArgs, submit_horovod.go:63-76).

    ``workers`` is the TOTAL rank count as typed by the user; the chart gets workers-1 StatefulSet
    replicas because the launcher (master) is also a rank (submit_horovod.go:132-133)."""
    ssh_port: int = 33          # kept for values compatibility; the local runtime rendezvous is
    rdzv_port: int = 29500      # a TCPStore (MASTER_ADDR/MASTER_PORT), no sshd
    cpu: str = ""
    memory: str = ""
    shm_size: str = "2Gi"
    ranks_per_pod: int = -1     # -1: one rank per GPU (hvd-distribute.sh <hosts> <gpus>)
    jupyter: bool = False       # launcher pod runs Jupyter (charts/tf-horovod/values.yaml:23-27)
    tensorboard: TensorboardArgs = field(default_factory=TensorboardArgs)
    sync: SyncCodeArgs = field(default_factory=SyncCodeArgs)
    chart: str = MPI_CHART

    def effective_ranks_per_pod(self) -> int:
        if self.ranks_per_pod > 0:
            return self.ranks_per_pod
        return max(1, self.gpu_count)

    def prepare(self, args: List[str]) -> None:
        self.command = " ".join(args)
        self.check()
        self.tensorboard.transform()
        self.sync.handle()            # Q7 fixed: sync works for mpijob too
        self.transform()
        self.apply_envs()             # env `workers` = total ranks (set before the decrement)

    def check(self) -> None:
        super().check()
        if not self.image:
            raise ValidationError("--image must be set ")
        if self.workers < 1:
            raise ValidationError("--workers must be greater than 0")
        if self.ranks_per_pod == 0 or self.ranks_per_pod < -1:
            raise ValidationError("--ranksPerPod must be >= 1 (or -1: one per GPU)")
        if self.gpu_count > 0 and self.effective_ranks_per_pod() > self.gpu_count:
            raise ValidationError(f"--ranksPerPod {self.ranks_per_pod} exceeds --gpus "
                                  f"{self.gpu_count}: every rank needs its own GPU")

    def values(self) -> dict:
        v = super().values()
        v["workers"] = self.workers - 1   # master is a rank too
        v.update({"sshPort": self.ssh_port, "rdzvPort": self.rdzv_port, "cpu": self.cpu,
                  "memory": self.memory, "shmSize": self.shm_size,
                  "ranksPerPod": self.effective_ranks_per_pod()})
        if self.jupyter:
            v["jupyter"] = True
        v.update(self.tensorboard.values())
        v.update(self.sync.values())
        return v


@dataclass
class StandaloneJobArgs(SubmitArgs):
    """Single-pod job (submitStandaloneJobArgs, submit_standalone.go:63-74)."""
    cpu: str = ""
    memory: str = ""
    tensorboard: TensorboardArgs = field(default_factory=TensorboardArgs)
    sync: SyncCodeArgs = field(default_factory=SyncCodeArgs)
    chart: str = STANDALONE_CHART

    def prepare(self, args: List[str]) -> None:
        self.command = " ".join(args)
        self.check()
        self.tensorboard.transform()
        self.sync.handle()
        self.transform()
        self.apply_envs()

    def check(self) -> None:
        super().check()
        if not self.image:
            raise ValidationError("--image must be set")

    def values(self) -> dict:
        v = super().values()
        v.update({"cpu": self.cpu, "memory": self.memory})
        v.update(self.tensorboard.values())
        v.update(self.sync.values())
        return v


def chart_of(args: SubmitArgs) -> str:
    return getattr(args, "chart")


def default_image(image: Optional[str]) -> str:
    return image or DEFAULT_IMAGE
