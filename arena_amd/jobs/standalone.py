"""Standalone ("standalonejob") trainer (reference: trainer_standalone.go:72-273): Job labelled
release=<name>, app=training; the chief is the newest pod; the pod list is [chief]."""
from __future__ import annotations

from .job_info import JobInfo
from .trainer import Trainer

APP = "training"


class StandaloneJobTrainer(Trainer):
    def type(self) -> str:
        return "standalonejob"

    def _sel(self, name):
        return {"release": name, "app": APP}

    def is_supported(self, name, namespace) -> bool:
        sel = self._sel(name)
        if self.cache is not None:
            return bool(self.cache.select("jobs", namespace, sel))
        return len(self.backend.list_jobs(namespace, sel)) > 0

    def get_training_job(self, name, namespace):
        sel = self._sel(name)
        if self.cache is not None:
            jobs = self.cache.select("jobs", namespace, sel)
            pods = self.cache.select("pods", namespace, sel)
        else:
            jobs = self.backend.list_jobs(namespace, sel)
            pods = self.backend.list_pods(namespace, sel)
        job = jobs[0] if jobs else None
        chief = None
        for p in pods:
            if p.meta.labels.get("role") == "tensorboard":
                continue
            if chief is None or chief.meta.creation_timestamp < p.meta.creation_timestamp:
                chief = p
        return JobInfo(name, self.type(), job, [chief] if chief is not None else [], chief)
