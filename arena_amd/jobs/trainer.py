"""TrainingJob / Trainer interfaces, trainer registry and orderings
(reference: trainer_interface.go:10-54, trainer.go:10-75)."""
from __future__ import annotations

import abc
import time
from typing import List, Optional

from ..cluster.objects import Pod
from ..utils.duration import short_human_duration
from .gpu import gpu_in_active_pod, gpu_in_pod


class TrainingJob(abc.ABC):
    def __init__(self, name: str, trainer_type: str, pods: List[Pod], chief: Optional[Pod]):
        self._name = name
        self._trainer = trainer_type
        self._pods = pods
        self._chief = chief
        self._requested: Optional[int] = None
        self._allocated: Optional[int] = None

    def name(self) -> str:
        return self._name

    def trainer(self) -> str:
        return self._trainer

    def chief_pod(self) -> Optional[Pod]:
        return self._chief

    def all_pods(self) -> List[Pod]:
        return self._pods

    @abc.abstractmethod
    def get_status(self) -> str: ...

    @abc.abstractmethod
    def start_time(self) -> Optional[float]: ...

    @abc.abstractmethod
    def get_job_dashboards(self, backend, arena_namespace: str) -> List[str]: ...

    def age(self, now: Optional[float] = None) -> str:
        st = self.start_time()
        if not st:
            return "0s"
        return short_human_duration((now if now is not None else time.time()) - st)

    def requested_gpu(self) -> int:
        if self._requested is None:  # memoised (job_info.go:50-70)
            self._requested = sum(gpu_in_pod(p) for p in self._pods)
        return self._requested

    def allocated_gpu(self) -> int:
        if self._allocated is None:
            self._allocated = sum(gpu_in_active_pod(p) for p in self._pods)
        return self._allocated

    def host_ip_of_chief(self) -> str:
        if self.get_status() == "RUNNING" and self._chief is not None:
            return self._chief.host_ip or "N/A"
        return "N/A"

    def namespace(self) -> str:
        return self._chief.namespace if self._chief is not None else "default"


class Trainer(abc.ABC):
    def __init__(self, backend, cache=None):
        self.backend = backend
        self.cache = cache  # ClusterCache or None (non-cached path queries by label)

    @abc.abstractmethod
    def type(self) -> str: ...

    @abc.abstractmethod
    def is_supported(self, name: str, namespace: str) -> bool: ...

    @abc.abstractmethod
    def get_training_job(self, name: str, namespace: str) -> TrainingJob: ...


class ClusterCache:
    """All pods / jobs / TFJobs fetched once for list/top (list.go:36-47, pod_helper.go), indexed
    by their ``release`` label: every trainer selector names its release, so a lookup touches only
    that release's objects and listing N jobs stays linear in N (a scan of every object per job
    made ``arena list`` quadratic: 100 jobs took 0.12-0.15 s, most of it in label matching)."""

    def __init__(self, backend):
        self.pods = backend.list_pods()
        self.jobs = backend.list_jobs()
        try:
            self.tfjobs = backend.list_tfjobs()
        except Exception:  # noqa: BLE001 - TFJob API absent -> trainer disabled
            self.tfjobs = []
        self._index = {}
        for kind in ("pods", "jobs", "tfjobs"):
            idx = self._index[kind] = {}
            for o in getattr(self, kind):
                idx.setdefault(o.meta.labels.get("release"), []).append(o)

    def of_release(self, kind: str, release: str) -> list:
        """The cached ``kind`` objects labelled ``release=<release>`` (any namespace)."""
        return self._index[kind].get(release, [])

    def select(self, kind: str, namespace: str, sel: dict) -> list:
        """The cached ``kind`` objects in ``namespace`` matching the equality selector ``sel``
        (which must name a release)."""
        from ..cluster.objects import matches
        return [o for o in self.of_release(kind, sel["release"])
                if o.meta.namespace == namespace and matches(o.meta.labels, sel)]


def new_trainers(backend, cache=None) -> List[Trainer]:
    """Order matters -- first match wins: MPI, Standalone, TensorFlow (trainer.go:13-16)."""
    from .mpi import MPIJobTrainer
    from .standalone import StandaloneJobTrainer
    from .tensorflow import TensorFlowJobTrainer
    return [MPIJobTrainer(backend, cache), StandaloneJobTrainer(backend, cache),
            TensorFlowJobTrainer(backend, cache)]


def order_by_age(jobs: List[TrainingJob]) -> List[TrainingJob]:
    """Newest first; jobs without a start time first (trainer.go:39-66)."""
    return sorted(jobs, key=lambda j: (j.start_time() is not None, -(j.start_time() or 0)))


def order_by_gpu(jobs: List[TrainingJob]) -> List[TrainingJob]:
    """Requested GPUs, descending (trainer.go:25-37, 68-75)."""
    return sorted(jobs, key=lambda j: -j.requested_gpu())


def get_training_job(backend, name: str, namespace: str, cache=None) -> TrainingJob:
    for t in new_trainers(backend, cache):
        if t.is_supported(name, namespace):
            return t.get_training_job(name, namespace)
    raise LookupError(f"Failed to find the training job {name} in namespace {namespace}")
