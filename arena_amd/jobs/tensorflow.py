"""PS/worker ("tfjob") trainer (reference: trainer_tensorflow.go:33-439).

Discovery through TFJobs labelled release=<name>, app=tfjob; pods additionally need
group_name=kubeflow.org. The chief is worker 0. Status precedence from TFJob conditions:
Succeeded > Failed > (Created | Restarting) = PENDING > RUNNING; UNKNOWN without a TFJob.
"""
from __future__ import annotations

from typing import List, Optional

from ..cluster.objects import TFJob, matches
from .dashboard import dashboard
from .trainer import Trainer, TrainingJob

APP = "tfjob"


def has_condition(tf: TFJob, ctype: str) -> bool:
    return any(c.type == ctype and c.status == "True" for c in tf.conditions)


class TensorFlowJob(TrainingJob):
    def __init__(self, name, trainer_type, tfjob: Optional[TFJob], pods, chief):
        super().__init__(name, trainer_type, pods, chief)
        self.tfjob = tfjob

    def get_status(self) -> str:
        tf = self.tfjob
        if tf is None or not tf.name:
            return "UNKNOWN"
        if has_condition(tf, "Succeeded"):
            return "SUCCEEDED"
        if has_condition(tf, "Failed"):
            return "FAILED"
        if has_condition(tf, "Created") or has_condition(tf, "Restarting"):
            return "PENDING"
        return "RUNNING"

    def start_time(self):
        return self.tfjob.start_time if self.tfjob is not None else None

    def get_job_dashboards(self, backend, arena_namespace) -> List[str]:
        url = dashboard(backend, arena_namespace, "tf-job-dashboard") or \
            dashboard(backend, "kubeflow", "tf-job-dashboard")
        if not url:
            raise LookupError("No LOGVIEWER Installed.")
        tf = self.tfjob
        return [f"{url}/tfjobs/ui/#/{tf.meta.namespace}/{tf.name}"]


class TensorFlowJobTrainer(Trainer):
    def type(self) -> str:
        return "tfjob"

    def _sel(self, name):
        return {"release": name, "app": APP}

    def _is_pod(self, name, ns, p) -> bool:
        return (p.namespace == ns and matches(p.meta.labels, self._sel(name))
                and p.meta.labels.get("group_name") == "kubeflow.org")

    def is_supported(self, name, namespace) -> bool:
        sel = self._sel(name)
        if self.cache is not None:
            return any(t.meta.namespace == namespace and matches(t.meta.labels, sel)
                       for t in self.cache.tfjobs)
        try:
            return len(self.backend.list_tfjobs(namespace, sel)) > 0
        except Exception:  # noqa: BLE001 - no TFJob support in this cluster
            return False

    def get_training_job(self, name, namespace):
        sel = self._sel(name)
        if self.cache is not None:
            tfjobs = [t for t in self.cache.tfjobs
                      if t.meta.namespace == namespace and matches(t.meta.labels, sel)]
            pods = self.cache.pods
        else:
            tfjobs = self.backend.list_tfjobs(namespace, sel)
            if not tfjobs:
                raise LookupError(f"Failed to find the job for {name}")
            pods = self.backend.list_pods(namespace, {"release": name})
        tf = tfjobs[0] if tfjobs else None
        chief, out = None, []
        for p in pods:
            if not self._is_pod(name, namespace, p):
                continue
            if (p.meta.labels.get("tf-replica-type") == "worker"
                    and p.meta.labels.get("tf-replica-index") == "0"):
                chief = p
            out.append(p)
        return TensorFlowJob(name, self.type(), tf, out, chief)
