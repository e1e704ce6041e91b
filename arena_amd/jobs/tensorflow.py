"""PS/worker ("tfjob") trainer (reference: trainer_tensorflow.go:33-439).

Discovery through labels release=<name>, app=tfjob; pods additionally need
group_name=kubeflow.org. The chief is worker 0. Status precedence from TFJob conditions:
Succeeded > Failed > (Created | Restarting) = PENDING > RUNNING; UNKNOWN without a job.

Two shapes of the same job are understood:

* the operator-free default (``charts.render_tfjob``): one batch Job per task
  (``<release>-tfjob-<type>-<i>``). The TFJob conditions tf-operator would have written are
  derived here from those Jobs and their pods (:func:`tfjob_from_jobs`) -- Succeeded once every
  worker Job succeeded, Failed once any task Job failed for good, Running once a task pod runs,
  else Created;
* a ``kubeflow.org`` TFJob (``--tfOperator``), whose conditions come from the operator.
"""
from __future__ import annotations

from typing import List, Optional

from ..cluster.objects import Condition, Job, Meta, POD_RUNNING, TFJob, matches
from .dashboard import dashboard
from .trainer import Trainer, TrainingJob

APP = "tfjob"


def has_condition(tf: TFJob, ctype: str) -> bool:
    return any(c.type == ctype and c.status == "True" for c in tf.conditions)


def _job_failed(j: Job) -> bool:
    return j.failed > 0 and j.active == 0 and j.failed > j.backoff_limit and j.succeeded == 0


def task_jobs_phase(jobs: List[Job]) -> Optional[str]:
    """Terminal phase of an operator-free PS/worker job from its per-task Jobs, or None while it
    runs. The ONE rule both the CLI status (:func:`tfjob_from_jobs`) and jobmon's clean-up wait
    (``runtime.jobmon.wait_tfjob_done``) use:

    * ``Succeeded`` once EVERY worker task Job succeeded (the all-workers rule: a finished
      worker 0 with other workers still training is still running);
    * ``Failed`` once any task Job (worker or PS) failed for good (failures past its
      backoffLimit, nothing active, never succeeded);
    * None otherwise (including no worker Jobs yet).

    tf-operator's controller source is not vendored in the reference, so whether its v1alpha2
    condition used this all-workers rule or a chief/worker-0 rule is parity unpinned; the
    all-workers rule matches what `arena get`/`list` in the reference's docs show for finished
    distributed jobs (docs/userguide/3-tfjob-distributed.md:56-77)."""
    workers = [j for j in jobs if j.meta.labels.get("tf-replica-type") == "worker"]
    if workers and all(j.succeeded > 0 for j in workers):
        return "Succeeded"
    if any(_job_failed(j) for j in jobs):
        return "Failed"
    return None


def tfjob_from_jobs(release: str, namespace: str, jobs: List[Job], pods) -> Optional[TFJob]:
    """The TFJob status tf-operator would report, computed from the per-task Jobs."""
    if not jobs:
        return None
    tf = TFJob(meta=Meta(name=f"{release}-tfjob", namespace=namespace,
                         labels={"app": APP, "release": release},
                         creation_timestamp=min(j.meta.creation_timestamp for j in jobs)))
    for j in jobs:
        t = j.meta.labels.get("tf-replica-type", "")
        key = {"ps": "PS", "worker": "Worker", "chief": "Chief", "evaluator": "Evaluator"}.get(t, t)
        tf.replicas[key] = tf.replicas.get(key, 0) + 1
    starts = [j.start_time for j in jobs if j.start_time]
    tf.start_time = min(starts) if starts else None
    phase = task_jobs_phase(jobs)
    if phase is not None:
        tf.conditions.append(Condition(phase, "True"))
    elif any(p.phase == POD_RUNNING for p in pods):
        tf.conditions.append(Condition("Running", "True"))
    else:
        tf.conditions.append(Condition("Created", "True"))
    return tf


class TensorFlowJob(TrainingJob):
    def __init__(self, name, trainer_type, tfjob: Optional[TFJob], pods, chief,
                 operator: bool = True):
        super().__init__(name, trainer_type, pods, chief)
        self.tfjob = tfjob
        self.operator = operator

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
        """tf-job-dashboard URL (trainer_tensorflow.go:106-133); without tf-operator's dashboard,
        the log viewer's per-pod URL of the chief (the kubernetes-dashboard shape)."""
        url = dashboard(backend, arena_namespace, "tf-job-dashboard") or \
            dashboard(backend, "kubeflow", "tf-job-dashboard")
        if url:
            tf = self.tfjob
            return [f"{url}/tfjobs/ui/#/{tf.meta.namespace}/{tf.name}"]
        url = dashboard(backend, arena_namespace, "kubernetes-dashboard") or \
            dashboard(backend, "kube-system", "kubernetes-dashboard")
        if not url:
            raise LookupError("No LOGVIEWER Installed.")
        pod = self._chief
        if pod is None:
            return []
        container = pod.containers[0].name if pod.containers else ""
        return [f"{url}/#!/log/{pod.namespace}/{pod.name}/{container}?namespace={pod.namespace}"]


class TensorFlowJobTrainer(Trainer):
    def type(self) -> str:
        return "tfjob"

    def _sel(self, name):
        return {"release": name, "app": APP}

    def _is_pod(self, name, ns, p) -> bool:
        return (p.namespace == ns and matches(p.meta.labels, self._sel(name))
                and p.meta.labels.get("group_name") == "kubeflow.org")

    def _task_jobs(self, name, namespace) -> List[Job]:
        sel = self._sel(name)
        if self.cache is not None:
            jobs = self.cache.select("jobs", namespace, sel)
        else:
            jobs = self.backend.list_jobs(namespace, sel)
        return [j for j in jobs if j.meta.labels.get("tf-replica-type")]

    def _tfjobs(self, name, namespace) -> List[TFJob]:
        sel = self._sel(name)
        if self.cache is not None:
            return self.cache.select("tfjobs", namespace, sel)
        try:
            return self.backend.list_tfjobs(namespace, sel)
        except Exception:  # noqa: BLE001 - no TFJob API in this cluster
            return []

    def is_supported(self, name, namespace) -> bool:
        return bool(self._tfjobs(name, namespace)) or bool(self._task_jobs(name, namespace))

    def get_training_job(self, name, namespace):
        tfjobs = self._tfjobs(name, namespace)
        if self.cache is not None:
            pods = self.cache.of_release("pods", name)
        else:
            pods = self.backend.list_pods(namespace, {"release": name})
        chief, out = None, []
        for p in pods:
            if not self._is_pod(name, namespace, p):
                continue
            if (p.meta.labels.get("tf-replica-type") == "worker"
                    and p.meta.labels.get("tf-replica-index") == "0"):
                # a retried task has several pods: the newest is the live one
                if chief is None or chief.meta.creation_timestamp <= p.meta.creation_timestamp:
                    chief = p
            out.append(p)
        if tfjobs:
            return TensorFlowJob(name, self.type(), tfjobs[0], out, chief, operator=True)
        jobs = self._task_jobs(name, namespace)
        if not jobs and self.cache is None:
            raise LookupError(f"Failed to find the job for {name}")
        return TensorFlowJob(name, self.type(), tfjob_from_jobs(name, namespace, jobs, out), out,
                             chief, operator=False)
