"""arena-jobmon: reap an allreduce job's workers once its launcher finishes
(reference: cmd/job-monitor/main.go:31-174).

Env contract (same as the reference): NAMESPACE, JOBNAME (the launcher Job), STATEFULSETNAME.
Waits (poll 5 s) until the Job has started and then SUCCEEDED -- or FAILED (quirk Q11: the
reference waited forever on a failed launcher and nil-dereferenced on API errors) -- then deletes
the workers' headless Service and the StatefulSet and waits (10 min, tick 10 s) until it is gone.
Works against any backend (``ARENA_BACKEND``): the in-cluster K8s API, the local job store, or
the fake backend in tests. The local supervisor applies the same policy natively.
"""
from __future__ import annotations

import os
import sys
import time

from ..utils.errors import NEED_WAIT
from ..utils.logs import get_logger, set_log_level
from ..utils.retry import retry_during

log = get_logger("jobmon")


class JobmonConfigError(RuntimeError):
    pass


def config_from_env(env=None):
    env = os.environ if env is None else env
    out = {}
    for k in ("NAMESPACE", "JOBNAME", "STATEFULSETNAME"):
        v = env.get(k, "")
        if not v:
            raise JobmonConfigError(f"Failed to get {k.lower()} from env {k}")
        out[k] = v
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

    retry_during(duration_s, tick_s, check, clock=clock, sleep=sleep)
    return result["phase"]


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
    return 0


if __name__ == "__main__":
    sys.exit(main())
