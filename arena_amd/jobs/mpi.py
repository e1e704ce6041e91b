"""Allreduce ("mpijob") trainer (reference: trainer_mpi.go:72-332).

Discovery: batch Job labelled release=<name>, app=tf-horovod; pods with the same labels. The
chief is the NEWEST pod owned by a Job (the launcher, possibly retried); StatefulSet worker pods
are listed too, chief last.
"""
from __future__ import annotations

from .job_info import JobInfo
from .trainer import Trainer

APP = "tf-horovod"


class MPIJobTrainer(Trainer):
    def type(self) -> str:
        return "mpijob"

    def _sel(self, name):
        return {"release": name, "app": APP}

    def is_supported(self, name, namespace) -> bool:
        sel = self._sel(name)
        if self.cache is not None:
            return bool(self.cache.select("jobs", namespace, sel))
        return len(self.backend.list_jobs(namespace, sel)) > 0   # Q10: use ns, not a global

    def get_training_job(self, name, namespace):
        sel = self._sel(name)
        if self.cache is not None:
            jobs = self.cache.select("jobs", namespace, sel)
            pods = self.cache.select("pods", namespace, sel)
        else:
            jobs = self.backend.list_jobs(namespace, sel)
            pods = self.backend.list_pods(namespace, sel)
        # the master Job (not the jobmon Job, which lives in arena-system)
        job = next((j for j in jobs if j.meta.labels.get("role", "mpimaster") == "mpimaster"),
                   jobs[0] if jobs else None)
        chief, others = None, []
        for p in pods:
            if "Job" in p.meta.owner_kinds:
                if chief is None or chief.meta.creation_timestamp < p.meta.creation_timestamp:
                    chief = p
            else:
                others.append(p)
        all_pods = others + ([chief] if chief is not None else [])
        return JobInfo(name, self.type(), job, all_pods, chief)
