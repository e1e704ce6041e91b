"""jobmon reaps the workers after the launcher succeeds OR fails (Q11), on the fake backend."""
import io

import pytest

from arena_amd.cli.commands import run as arena
from arena_amd.cluster.fake import FakeBackend, make_node
from arena_amd.runtime import jobmon


def _setup():
    fake = FakeBackend([make_node("n", "10.0.0.1", 8)])
    assert arena(["submit", "mpi", "--name", "h", "--workers", "3", "--gpus", "1", "--image", "i",
                  "python", "t.py"], backend=fake, out=io.StringIO()) == 0
    fake.schedule()
    env = {"NAMESPACE": "default", "JOBNAME": "h-tf-horovod-job", "STATEFULSETNAME": "h-tf-horovod"}
    return fake, env


def _launcher(fake):
    return next(p for p in fake.list_pods("default") if p.meta.labels.get("role") == "mpimaster")


@pytest.mark.parametrize("outcome", ["Succeeded", "Failed"])
def test_reap_on_success_and_failure(outcome):
    fake, env = _setup()
    polls = {"n": 0}

    def sleep(_s):
        polls["n"] += 1
        if polls["n"] == 2:
            fake.set_phase("default", _launcher(fake).name, outcome)

    assert len([p for p in fake.list_pods("default") if "StatefulSet" in p.meta.owner_kinds]) == 2
    phase = jobmon.run(fake, env, sleep=sleep)
    assert phase == outcome
    assert fake.get_statefulset("default", "h-tf-horovod") is None
    assert [p for p in fake.list_pods("default") if "StatefulSet" in p.meta.owner_kinds] == []
    assert all(s.name != "h-tf-horovod" for s in fake.list_services("default"))


def test_env_contract():
    with pytest.raises(jobmon.JobmonConfigError, match="JOBNAME"):
        jobmon.config_from_env({"NAMESPACE": "x", "STATEFULSETNAME": "s"})


def test_waits_for_missing_job_then_times_out():
    fake = FakeBackend([])
    t = {"now": 0.0}

    def clock():
        t["now"] += 5.0
        return t["now"]

    with pytest.raises(RuntimeError, match="attempts"):
        jobmon.wait_job_complete(fake, "default", "nope", duration_s=20, clock=clock,
                                 sleep=lambda s: None)


def test_launcher_never_starts_times_out(monkeypatch):
    """Q11 bounded: the launcher Job exists but its pod never starts (unschedulable, image pull
    failure). ARENA_JOBMON_TIMEOUT ends the wait with JobmonTimeout, and main() exits 3."""
    fake = FakeBackend([])     # no nodes: nothing is ever scheduled
    assert arena(["submit", "mpi", "--name", "h", "--workers", "2", "--gpus", "1", "--image", "i",
                  "python", "t.py"], backend=fake, out=io.StringIO()) == 0
    env = {"NAMESPACE": "default", "JOBNAME": "h-tf-horovod-job",
           "STATEFULSETNAME": "h-tf-horovod", "ARENA_JOBMON_TIMEOUT": "30s"}
    assert jobmon.config_from_env(env)["TIMEOUT_S"] == 30.0
    t = {"now": 0.0}

    def clock():
        return t["now"]

    def sleep(s):
        t["now"] += s

    # a Job whose pod never ran: no start time (the fake controller stamps creation as start,
    # so clear it to model a pod stuck in Pending before the Job controller saw it start)
    fake.get_job("default", "h-tf-horovod-job").start_time = None
    with pytest.raises(jobmon.JobmonTimeout, match="did not finish within 30s"):
        jobmon.run(fake, env, clock=clock, sleep=sleep)
    assert 30.0 <= t["now"] <= 40.0     # 5 s ticks: gave up right after the bound
    assert fake.get_statefulset("default", "h-tf-horovod") is not None   # nothing reaped
    # main(): exit code 3, no traceback
    monkeypatch.setattr("arena_amd.cli.backends.make_backend", lambda a: fake)
    for k, v in {**env, "ARENA_JOBMON_TIMEOUT": "0.001"}.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setattr(jobmon.time, "sleep", lambda s: None)
    assert jobmon.main() == 3


def test_timeout_parsing():
    base = {"NAMESPACE": "n", "JOBNAME": "j", "STATEFULSETNAME": "s"}
    assert jobmon.config_from_env(base)["TIMEOUT_S"] == 168 * 3600     # default: 7 days
    assert jobmon.config_from_env({**base, "ARENA_JOBMON_TIMEOUT": "1h30m"})["TIMEOUT_S"] == 5400
    assert jobmon.config_from_env({**base, "ARENA_JOBMON_TIMEOUT": "0"})["TIMEOUT_S"] == float("inf")
    with pytest.raises(jobmon.JobmonConfigError, match="ARENA_JOBMON_TIMEOUT"):
        jobmon.config_from_env({**base, "ARENA_JOBMON_TIMEOUT": "soon"})


@pytest.mark.parametrize("outcome", ["Succeeded", "Failed"])
def test_tfjob_clean_pod_policy(outcome):
    """PS/worker without tf-operator: once the workers are done (or one failed), the still
    running tasks -- the PS -- are deleted (cleanPodPolicy=Running)."""
    fake = FakeBackend([make_node("n", "10.0.0.1", 8)])
    assert arena(["submit", "tf", "--name", "d", "--workers", "2", "--ps", "1", "--gpus", "1",
                  "--image", "i", "python", "t.py"], backend=fake, out=io.StringIO()) == 0
    fake.schedule()
    jm = next(p for p in fake.list_pods("arena-system"))
    env = dict(jm.containers[0].env)
    assert env["TFJOBNAME"] == "d-tfjob" and env["CLEANPODPOLICY"] == "Running"

    def task(t):
        return next(p.name for p in fake.list_pods("default") if p.name.rsplit("-", 1)[0] == t)

    polls = {"n": 0}

    def sleep(_s):
        polls["n"] += 1
        if polls["n"] == 1:
            fake.set_phase("default", task("d-tfjob-worker-0"), "Succeeded")
        if polls["n"] == 2:
            fake.set_phase("default", task("d-tfjob-worker-1"), outcome)

    assert jobmon.run(fake, env, sleep=sleep) == outcome
    assert polls["n"] == 2
    assert fake.get_job("default", "d-tfjob-ps-0") is None
    assert not [p for p in fake.list_pods("default") if p.name.startswith("d-tfjob-ps-0-")]
    assert fake.get_job("default", "d-tfjob-worker-0") is not None


def test_tfjob_status_rule_shared_by_cli_and_jobmon():
    """Worker 0 finished while worker 1 still trains: the job is RUNNING for `arena list` and
    not finished for jobmon (one rule, arena_amd.jobs.tensorflow.task_jobs_phase)."""
    from arena_amd.jobs.tensorflow import task_jobs_phase
    fake = FakeBackend([make_node("n", "10.0.0.1", 8)])
    assert arena(["submit", "tf", "--name", "d", "--workers", "2", "--ps", "1", "--gpus", "1",
                  "--image", "i", "python", "t.py"], backend=fake, out=io.StringIO()) == 0
    fake.schedule()

    def task(t):
        return next(p.name for p in fake.list_pods("default") if p.name.rsplit("-", 1)[0] == t)

    for t in ("d-tfjob-ps-0", "d-tfjob-worker-0", "d-tfjob-worker-1"):
        fake.set_phase("default", task(t), "Running")
    fake.set_phase("default", task("d-tfjob-worker-0"), "Succeeded")
    jobs = fake.list_jobs("default", {"release": "d", "app": "tfjob"})
    assert task_jobs_phase(jobs) is None
    out = io.StringIO()
    assert arena(["list"], backend=fake, out=out) == 0
    assert out.getvalue().splitlines()[1].split()[1] == "RUNNING"
    fake.set_phase("default", task("d-tfjob-worker-1"), "Succeeded")
    jobs = fake.list_jobs("default", {"release": "d", "app": "tfjob"})
    assert task_jobs_phase(jobs) == "Succeeded"
    out = io.StringIO()
    assert arena(["list"], backend=fake, out=out) == 0
    assert out.getvalue().splitlines()[1].split()[1] == "SUCCEEDED"
