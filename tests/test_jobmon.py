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
