"""K8s backend through the real CLI against a file-backed fake ``kubectl`` (tests/fake_kubectl.py).

Covers the helm-equivalent release store (record ConfigMap + apply/delete of every rendered
object), discovery/status through ``kubectl get -o json`` parsing, logs flags, and the JSON codec.
"""
from __future__ import annotations

import io
import json
import os
import subprocess
import sys

import pytest

from arena_amd.cli.commands import run
from arena_amd.cluster import k8s_json as kj
from arena_amd.cluster.controller import ClusterState
from arena_amd.cluster.k8s import K8sBackend

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture
def kube(tmp_path, monkeypatch):
    state = tmp_path / "kube.json"
    monkeypatch.setenv("FAKE_KUBE_STATE", str(state))
    wrapper = tmp_path / "kubectl"
    wrapper.write_text(f"#!/bin/sh\nexec {sys.executable} {HERE}/fake_kubectl.py \"$@\"\n")
    wrapper.chmod(0o755)

    def k(*args):
        r = subprocess.run([str(wrapper), *args], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        return r.stdout
    k("fake-node", "mi355x-a", "10.1.0.1", "8")
    k("fake-node", "mi355x-b", "10.1.0.2", "8")
    b = K8sBackend(kubectl=str(wrapper))
    b.fake = k
    b.state = state
    return b


def cli(b, *argv):
    out = io.StringIO()
    rc = run(list(argv), backend=b, out=out)
    return out.getvalue() if rc == 0 else f"rc={rc}\n" + out.getvalue()


def rows(text):
    return [line.split() for line in text.strip().splitlines()[1:]]


def test_standalone_lifecycle(kube):
    out = cli(kube, "submit", "sj", "--name", "mnist", "--image", "rocm/pytorch", "--gpus", "2",
              "python main.py")
    assert "mnist-training" in out
    st = json.load(open(kube.state))
    assert "default/arena-release-mnist" in st["configmaps"]
    job = st["jobs"]["default/mnist-training"]
    ctr = job["spec"]["template"]["spec"]["containers"][0]
    assert ctr["resources"]["limits"]["amd.com/gpu"] == 2
    pod = next(k.split("/")[1] for k in st["pods"])
    assert rows(cli(kube, "list"))[0][:3] == ["mnist", "PENDING", "STANDALONEJOB"]
    kube.fake("fake-phase", "default", pod, "Running", "mi355x-b")
    r = rows(cli(kube, "list"))[0]
    assert r[:3] == ["mnist", "RUNNING", "STANDALONEJOB"] and r[-1] == "10.1.0.2"
    top = cli(kube, "top", "node")
    assert "mi355x-b" in top and "2/16" in top
    kube.fake("fake-log", "default", pod, "Accuracy at step 990: 0.9649")
    assert cli(kube, "logs", "mnist").strip() == "Accuracy at step 990: 0.9649"
    ts = cli(kube, "logs", "--timestamps", "--tail", "1", "mnist")
    assert ts.split()[0].endswith("Z")
    kube.fake("fake-phase", "default", pod, "Succeeded", "mi355x-b", "0")
    assert rows(cli(kube, "list"))[0][1] == "SUCCEEDED"
    assert "already exist" in cli(kube, "submit", "sj", "--name", "mnist", "--image", "x", "true")
    assert "deleted" in cli(kube, "delete", "mnist")
    st = json.load(open(kube.state))
    assert not st["jobs"] and not st["pods"] and "default/arena-release-mnist" not in st["configmaps"]
    assert cli(kube, "list").strip().splitlines()[1:] == []


def test_mpijob_discovery_and_gpu_accounting(kube):
    cli(kube, "submit", "mpi", "--name", "hvd", "--image", "rocm/pytorch", "--gpus", "1",
        "--workers", "3", "python train.py")
    st = json.load(open(kube.state))
    assert st["statefulsets"]["default/hvd-tf-horovod"]["spec"]["replicas"] == 2
    assert "arena-system/hvd-tf-horovod-jobmon" in st["jobs"]
    pods = sorted(k.split("/")[1] for k in st["pods"] if k.startswith("default/"))
    for p in pods:
        kube.fake("fake-phase", "default", p, "Running", "mi355x-a")
    got = cli(kube, "get", "hvd")
    assert got.count("hvd-tf-horovod") >= 3 and "RUNNING" in got
    tj = cli(kube, "top", "job")
    assert rows(tj)[0][:2] == ["hvd", "RUNNING"] and "3" in rows(tj)[0]
    # jobmon's part: the launcher succeeded -> StatefulSet + headless Service deleted
    kube.delete_statefulset("default", "hvd-tf-horovod")
    kube.delete_service("default", "hvd-tf-horovod")
    assert kube.get_statefulset("default", "hvd-tf-horovod") is None
    cli(kube, "delete", "hvd")
    assert not json.load(open(kube.state))["jobs"]


def test_tfjob_conditions_and_tensorboard(kube):
    out = cli(kube, "submit", "tf", "--name", "dist", "--image", "rocm/tf", "--gpus", "1",
              "--workers", "2", "--ps", "1", "--tensorboard", "python dist.py")
    assert "TFJob" in out
    st = json.load(open(kube.state))
    pods = [k.split("/")[1] for k in st["pods"]]
    assert {"dist-tfjob-ps-0", "dist-tfjob-worker-0", "dist-tfjob-worker-1"} <= set(pods)
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "PENDING"]   # Created condition
    for p in pods:
        kube.fake("fake-phase", "default", p, "Running", "mi355x-a")
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "RUNNING"]
    got = cli(kube, "get", "dist")
    assert "tensorboard will be available on" in got and "10.1.0.1:" in got
    for p in ("dist-tfjob-worker-0", "dist-tfjob-worker-1"):
        kube.fake("fake-phase", "default", p, "Succeeded", "mi355x-a", "0")
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "SUCCEEDED"]
    kube.fake("fake-endpoints", "arena-system", "tf-job-dashboard", "10.1.0.9", "8080")
    lv = cli(kube, "logviewer", "dist")
    assert "10.1.0.9:8080/tfjobs/ui/#/default/dist-tfjob" in lv


def test_codec_roundtrip():
    from arena_amd.cluster import charts
    from arena_amd.jobs import spec as S
    a = S.TFJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.ps_count, a.namespace = "rt", "img", 1, 2, 1, "ns1"
    a.prepare(["python", "x.py"])
    st = ClusterState(clock=lambda: 1_700_000_000.0)
    created = st.apply(charts.render(a.chart, "rt", "ns1", a.values()))
    st.set_pod_phase("ns1", "rt-tfjob-worker-0", "Running")
    for o in created:
        kind = type(o).__name__
        to = getattr(kj, kind.lower() + "_to", None)
        frm = getattr(kj, kind.lower() + "_from", None)
        if to is None:
            continue
        back = frm(json.loads(json.dumps(to(o))))
        assert back.meta.name == o.meta.name and back.meta.labels == o.meta.labels
        if kind == "Pod":
            assert back.containers[0].limits == o.containers[0].limits
            assert back.phase == o.phase
        if kind == "TFJob":
            assert [c.type for c in back.conditions] == [c.type for c in o.conditions]
            assert back.replicas == o.replicas


def test_missing_kubectl_is_a_clear_error(monkeypatch):
    monkeypatch.delenv("ARENA_KUBECTL", raising=False)
    monkeypatch.setenv("PATH", "/nonexistent")
    from arena_amd.cluster.backend import BackendError
    with pytest.raises(BackendError, match="kubectl not found"):
        K8sBackend()
