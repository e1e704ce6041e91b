"""arena-jobmon: reap a distributed job's leftover tasks once it is done
(reference: cmd/job-monitor/main.go:31-174).

Allreduce jobs -- env contract of the reference: NAMESPACE, JOBNAME (the launcher Job),
STATEFULSETNAME. Waits (poll 5 s) until the Job has started and then SUCCEEDED -- or FAILED (quirk
Q11: the reference waited forever on a failed launcher and nil-dereferenced on API errors) --
then deletes the workers' headless Service and the StatefulSet and waits (10 min, tick 10 s)
until it is gone.

PS/worker jobs (the operator-free tfjob chart) -- env NAMESPACE, TFJOBNAME, RELEASE,
CLEANPODPOLICY: plays tf-operator's ``cleanPodPolicy`` (vendor/.../v1alpha2 defaults.go): once
every worker Job succeeded, or any task Job failed, the task Jobs still running (``Running``: the
parameter servers, which never exit on their own) or all of them (``All``) are deleted.

The wait is bounded by ``ARENA_JOBMON_TIMEOUT`` (a Go duration: ``168h`` = 7 days by default, ``90m``,
``3600``; ``0``/``inf`` = unbounded, the reference's ``math.MaxInt64``): a launcher that never
starts or hangs ends jobmon with exit code 3 instead of a pod that waits forever.
Works against any backend (``ARENA_BACKEND``): the in-cluster K8s API, the local job store, or
the fake backend in tests. The local supervisor applies the same policy natively.
"""
from __future__ import annotations

import os
import sys
import time

from ..utils.duration import parse_duration
from ..utils.errors import NEED_WAIT
from ..utils.logs import get_logger, set_log_level
from ..utils.retry import retry_during

log = get_logger("jobmon")
DEFAULT_TIMEOUT = "168h"


class JobmonConfigError(RuntimeError):
    pass


class JobmonTimeout(RuntimeError):
    pass


def config_from_env(env=None):
    env = os.environ if env is None else env
    keys = (("NAMESPACE", "TFJOBNAME", "RELEASE", "CLEANPODPOLICY") if env.get("TFJOBNAME")
            else ("NAMESPACE", "JOBNAME", "STATEFULSETNAME"))
    out = {}
    for k in keys:
        v = env.get(k, "")
        if not v:
            raise JobmonConfigError(f"Failed to get {k.lower()} from env {k}")
        out[k] = v
    if out.get("CLEANPODPOLICY", "Running") not in ("Running", "All", "None"):
        raise JobmonConfigError(f"unsupported CLEANPODPOLICY {out['CLEANPODPOLICY']}")
    raw = env.get("ARENA_JOBMON_TIMEOUT", DEFAULT_TIMEOUT).strip().lower()
    try:
        t = float("inf") if raw in ("", "0", "inf", "none") else parse_duration(raw)
    except ValueError as e:
        raise JobmonConfigError(f"bad ARENA_JOBMON_TIMEOUT {raw!r}: {e}") from None
    if t < 0:
        raise JobmonConfigError(f"bad ARENA_JOBMON_TIMEOUT {raw!r}: negative")
    out["TIMEOUT_S"] = t
    return out


def wait_job_complete(backend, namespace, job_name, duration_s=float("inf"), tick_s=5.0,
                      clock=time.monotonic, sleep=time.sleep) -> str:
    """Returns 'Succeeded' or 'Failed' once the launcher Job has finished."""
    result = {}

    def check():
        try:
            job = backend.get_job(namespace, job_name)
        except Exception as e:  # noqa: BLE001 - API hiccup: keep waiting (no nil deref)
            log.info("get job %s failed (%s), need to wait.", job_name, e)
            raise RuntimeError(NEED_WAIT) from e
        if job is None:
            log.info("Job %s doesn't exist, need to wait.", job_name)
            raise RuntimeError(NEED_WAIT)
        if not job.start_time:
            raise RuntimeError(NEED_WAIT)
        if job.succeeded > 0:
            result["phase"] = "Succeeded"
            return
        if job.failed > 0 and job.active == 0 and job.failed > job.backoff_limit:
            result["phase"] = "Failed"
            return
        raise RuntimeError(NEED_WAIT)

    try:
        retry_during(duration_s, tick_s, check, clock=clock, sleep=sleep)
    except RuntimeError as e:
        if "phase" not in result:
            raise JobmonTimeout(f"launcher {job_name} did not finish within {duration_s:.0f}s: "
                                f"{e}") from e
        raise
    return result["phase"]


def _task_jobs(backend, namespace, release):
    return [j for j in backend.list_jobs(namespace, {"release": release, "app": "tfjob"})
            if j.meta.labels.get("tf-replica-type")]


def wait_tfjob_done(backend, namespace, release, duration_s=float("inf"), tick_s=5.0,
                    clock=time.monotonic, sleep=time.sleep) -> str:
    """The job's terminal phase by the same rule as its CLI status
    (``arena_amd.jobs.tensorflow.task_jobs_phase``: Succeeded once EVERY worker task Job
    succeeded, Failed once any task Job failed for good)."""
    from ..jobs.tensorflow import task_jobs_phase
    result = {}

    def check():
        try:
            jobs = _task_jobs(backend, namespace, release)
        except Exception as e:  # noqa: BLE001 - API hiccup: keep waiting
            raise RuntimeError(NEED_WAIT) from e
        phase = task_jobs_phase(jobs)
        if phase is None:
            raise RuntimeError(NEED_WAIT)
        result["phase"] = phase

    try:
        retry_during(duration_s, tick_s, check, clock=clock, sleep=sleep)
    except RuntimeError as e:
        if "phase" not in result:
            raise JobmonTimeout(f"tfjob {release} did not finish within {duration_s:.0f}s") from e
        raise
    return result["phase"]


def clean_tfjob(backend, namespace, release, policy: str):
    """Delete the task Jobs the policy names; returns their names."""
    gone = []
    for j in _task_jobs(backend, namespace, release):
        if policy == "All" or (policy == "Running" and j.active > 0):
            backend.delete_job(namespace, j.name)
            gone.append(j.name)
    return gone


def delete_statefulset(backend, namespace, name, duration_s=600.0, tick_s=10.0,
                       clock=time.monotonic, sleep=time.sleep) -> None:
    ss = backend.get_statefulset(namespace, name)
    if ss is None:
        log.info("The statefulset %s in namespace %s is not found, it has been deleted.",
                  name, namespace)
        return
    svc = ss.template.get("serviceName") if isinstance(ss.template, dict) else None
    try:
        backend.delete_service(namespace, svc or name)
    except Exception as e:  # noqa: BLE001
        log.info("The service of %s in namespace %s has been deleted (%s).", name, namespace, e)
    backend.delete_statefulset(namespace, name)

    def gone():
        if backend.get_statefulset(namespace, name) is not None:
            raise RuntimeError(NEED_WAIT)

    retry_during(duration_s, tick_s, gone, clock=clock, sleep=sleep)


def run(backend, env=None, **kw) -> str:
    cfg = config_from_env(env)
    kw.setdefault("duration_s", cfg["TIMEOUT_S"])
    if "TFJOBNAME" in cfg:
        log.info("tfjob: %s, namespace: %s, cleanPodPolicy %s", cfg["TFJOBNAME"],
                 cfg["NAMESPACE"], cfg["CLEANPODPOLICY"])
        phase = wait_tfjob_done(backend, cfg["NAMESPACE"], cfg["RELEASE"], **kw)
        gone = clean_tfjob(backend, cfg["NAMESPACE"], cfg["RELEASE"], cfg["CLEANPODPOLICY"])
        log.info("tfjob %s finished: %s; deleted %s", cfg["TFJOBNAME"], phase, gone or "nothing")
        return phase
    log.info("jobName: %s, namespace: %s, statefulset %s", cfg["JOBNAME"], cfg["NAMESPACE"],
             cfg["STATEFULSETNAME"])
    phase = wait_job_complete(backend, cfg["NAMESPACE"], cfg["JOBNAME"], **kw)
    log.info("launcher %s finished: %s; reaping workers", cfg["JOBNAME"], phase)
    delete_statefulset(backend, cfg["NAMESPACE"], cfg["STATEFULSETNAME"],
                       clock=kw.get("clock", time.monotonic), sleep=kw.get("sleep", time.sleep))
    return phase


def main(argv=None) -> int:
    set_log_level(os.environ.get("ARENA_LOGLEVEL", "info"))
    from ..cli.backends import make_backend

    class _A:
        backend = None
        home = None
        config = ""

    try:
        run(make_backend(_A()))
    except JobmonConfigError as e:
        sys.stderr.write(f"{e}\n")
        return 2
    except JobmonTimeout as e:
        sys.stderr.write(f"jobmon: {e}\n")
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
