"""Batch-Job-backed training job (reference: job_info.go:10-108): status from the Job counters,
RUNNING downgraded to PENDING while the chief has no host IP or is still Pending."""
from __future__ import annotations

from typing import List, Optional

from ..cluster.objects import Job, Pod, POD_PENDING
from .dashboard import dashboard
from .trainer import TrainingJob


class JobInfo(TrainingJob):
    def __init__(self, name: str, trainer_type: str, job: Optional[Job], pods: List[Pod],
                 chief: Optional[Pod]):
        super().__init__(name, trainer_type, pods, chief)
        self.job = job

    def get_status(self) -> str:
        job, pod = self.job, self._chief
        status = ""
        if job is not None:
            if job.active > 0:
                status = "RUNNING"
            elif job.succeeded > 0:
                status = "SUCCEEDED"
            elif job.failed > 0:
                status = "FAILED"
        if status == "RUNNING":
            if pod is None or not pod.host_ip or pod.phase == POD_PENDING:
                status = "PENDING"
        return status

    def start_time(self):
        return self.job.start_time if self.job is not None else None

    def get_job_dashboards(self, backend, arena_namespace: str) -> List[str]:
        """kubernetes-dashboard log URL of the chief (trainer_mpi.go:34-63)."""
        url = dashboard(backend, arena_namespace, "kubernetes-dashboard") or \
            dashboard(backend, "kube-system", "kubernetes-dashboard")
        if not url:
            raise LookupError("No LOGVIEWER Installed.")
        pod = self._chief
        if pod is None:
            return []
        container = pod.containers[0].name if pod.containers else ""
        return [f"{url}/#!/log/{pod.namespace}/{pod.name}/{container}?namespace={pod.namespace}"]
