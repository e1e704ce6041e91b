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


def _pods(kube, ns="default"):
    return json.load(open(kube.state))["pods"]


def _task_pod(kube, task, ns="default"):
    (name,) = [k.split("/")[1] for k in _pods(kube) if k.startswith(ns + "/")
               and k.split("/")[1].rsplit("-", 1)[0] == task]
    return name


def test_tfjob_without_operator(kube, monkeypatch):
    """No tf-operator, no TFJob CRD: per-task Jobs + headless Services, TF_CONFIG from their DNS
    names, status from the Jobs, PS reaped by jobmon (cleanPodPolicy=Running)."""
    from arena_amd.runtime import jobmon
    monkeypatch.setenv("FAKE_KUBE_NO_TFJOB_CRD", "1")
    out = cli(kube, "submit", "tf", "--name", "dist", "--image", "rocm/tf", "--gpus", "1",
              "--workers", "2", "--ps", "1", "--tensorboard", "python dist.py")
    assert "==> batch/v1/Job" in out and "TFJob" not in out
    st = json.load(open(kube.state))
    assert not st["tfjobs"]
    tasks = {"ps-0": _task_pod(kube, "dist-tfjob-ps-0"),
             "worker-0": _task_pod(kube, "dist-tfjob-worker-0"),
             "worker-1": _task_pod(kube, "dist-tfjob-worker-1")}
    for t, pod in tasks.items():
        env = {e["name"]: e["value"] for e in
               st["pods"][f"default/{pod}"]["spec"]["containers"][0]["env"]}
        tfc = json.loads(env["TF_CONFIG"])
        assert tfc["task"] == {"type": t.split("-")[0], "index": int(t.split("-")[1])}
        # hostNetwork: one port per task (workers 22222, 22223; the PS the next free one)
        assert tfc["cluster"]["ps"] == ["dist-tfjob-ps-0.default.svc:22224"]
        assert tfc["cluster"]["worker"] == ["dist-tfjob-worker-0.default.svc:22222",
                                            "dist-tfjob-worker-1.default.svc:22223"]
    assert rows(cli(kube, "list"))[0][:3] == ["dist", "PENDING", "TFJOB"]
    for pod in tasks.values():
        kube.fake("fake-phase", "default", pod, "Running", "mi355x-a")
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "RUNNING"]
    # each task's headless Service resolves to its pod (endpoints controller)
    ep = kube.get_endpoints("default", "dist-tfjob-worker-1")
    assert ep.addresses == ["10.1.0.1"] and ep.ports == [22223]
    got = cli(kube, "get", "dist")
    assert tasks["worker-0"] in got and "tensorboard will be available on" in got
    for t in ("worker-0", "worker-1"):
        kube.fake("fake-phase", "default", tasks[t], "Succeeded", "mi355x-a", "0")
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "SUCCEEDED"]
    # jobmon (as rendered into arena-system) removes the still-running PS task
    st = json.load(open(kube.state))
    jm = st["jobs"]["arena-system/dist-tfjob-jobmon"]
    env = {e["name"]: e["value"]
           for e in jm["spec"]["template"]["spec"]["containers"][0]["env"]}
    assert jobmon.run(kube, env, sleep=lambda s: None) == "Succeeded"
    st = json.load(open(kube.state))
    assert "default/dist-tfjob-ps-0" not in st["jobs"]
    assert f"default/{tasks['ps-0']}" not in st["pods"]
    assert "default/dist-tfjob-worker-0" in st["jobs"]        # finished tasks are kept
    assert rows(cli(kube, "list"))[0][:2] == ["dist", "SUCCEEDED"]
    cli(kube, "delete", "dist")
    assert not [k for k in json.load(open(kube.state))["jobs"] if k.startswith("default/")]


def test_tfjob_failed_task(kube):
    cli(kube, "submit", "tf", "--name", "bad", "--image", "img", "--workers", "2", "--ps", "1",
        "python x.py")
    for t in ("bad-tfjob-ps-0", "bad-tfjob-worker-0", "bad-tfjob-worker-1"):
        kube.fake("fake-phase", "default", _task_pod(kube, t), "Running", "mi355x-b")
    kube.fake("fake-phase", "default", _task_pod(kube, "bad-tfjob-worker-1"), "Failed",
              "mi355x-b", "1")
    assert rows(cli(kube, "list"))[0][:2] == ["bad", "FAILED"]


def test_tfjob_operator_mode(kube):
    """--tfOperator keeps the reference's TFJob path for clusters that run tf-operator."""
    out = cli(kube, "submit", "tf", "--name", "op", "--image", "rocm/tf", "--gpus", "1",
              "--workers", "2", "--ps", "1", "--tfOperator", "python dist.py")
    assert "TFJob" in out
    st = json.load(open(kube.state))
    pods = [k.split("/")[1] for k in st["pods"]]
    assert {"op-tfjob-ps-0", "op-tfjob-worker-0", "op-tfjob-worker-1"} <= set(pods)
    assert rows(cli(kube, "list"))[0][:2] == ["op", "PENDING"]   # Created condition
    for p in pods:
        kube.fake("fake-phase", "default", p, "Running", "mi355x-a")
    assert rows(cli(kube, "list"))[0][:2] == ["op", "RUNNING"]
    for p in ("op-tfjob-worker-0", "op-tfjob-worker-1"):
        kube.fake("fake-phase", "default", p, "Succeeded", "mi355x-a", "0")
    assert rows(cli(kube, "list"))[0][:2] == ["op", "SUCCEEDED"]
    kube.fake("fake-endpoints", "arena-system", "tf-job-dashboard", "10.1.0.9", "8080")
    lv = cli(kube, "logviewer", "op")
    assert "10.1.0.9:8080/tfjobs/ui/#/default/op-tfjob" in lv


def test_allreduce_ranks_unique_under_host_network(kube):
    """Every allreduce pod runs on ONE node with hostNetwork (so $HOSTNAME is the node's name
    in all of them); the rendered command still gives ranks 0..N-1, each exactly once."""
    cli(kube, "submit", "mpi", "--name", "hn", "--image", "rocm/pytorch", "--gpus", "1",
        "--workers", "4", "echo RANK=$RANK WORLD=$WORLD_SIZE HOST=$HOSTNAME")
    st = json.load(open(kube.state))
    ranks = [k.split("/")[1] for k, p in st["pods"].items() if k.startswith("default/")
             and p["metadata"]["labels"].get("role") in ("mpimaster", "mpiworker")]
    assert len(ranks) == 4
    seen = []
    for pod in ranks:
        kube.fake("fake-phase", "default", pod, "Running", "mi355x-a")
        out = kube.fake("fake-exec", "default", pod).split()
        kv = dict(x.split("=", 1) for x in out)
        assert kv["HOST"] == "mi355x-a" and kv["WORLD"] == "4"
        seen.append(int(kv["RANK"]))
    assert sorted(seen) == [0, 1, 2, 3]


def test_allreduce_several_ranks_per_pod(kube):
    """`--workers 2 --gpus 4`: 2 pods x 4 ranks (hvd-distribute.sh <hosts> <gpus>). Each pod's
    entry process is the in-pod launcher; run as the kubelet would (fake-exec), the 8 ranks are
    0..7 exactly once, LOCAL_RANK 0..3 within each pod, LOCAL_WORLD_SIZE 4, WORLD_SIZE 8."""
    cli(kube, "submit", "mpi", "--name", "rpp", "--image", "rocm/pytorch", "--gpus", "4",
        "--workers", "2", "echo RANK=$RANK LOCAL=$LOCAL_RANK LWS=$LOCAL_WORLD_SIZE "
        "WORLD=$WORLD_SIZE GROUP=$GROUP_RANK")
    st = json.load(open(kube.state))
    pods = [k.split("/")[1] for k, p in st["pods"].items() if k.startswith("default/")
            and p["metadata"]["labels"].get("role") in ("mpimaster", "mpiworker")]
    assert len(pods) == 2
    for pod in pods:
        ctr = st["pods"][f"default/{pod}"]["spec"]["containers"][0]
        assert ctr["resources"]["limits"]["amd.com/gpu"] == 4
    seen = []
    for pod in pods:
        kube.fake("fake-phase", "default", pod, "Running", "mi355x-a")
        lines = kube.fake("fake-exec", "default", pod).strip().splitlines()
        assert len(lines) == 4, lines
        kvs = [dict(x.split("=", 1) for x in ln.split()) for ln in lines]
        assert {kv["LWS"] for kv in kvs} == {"4"} and {kv["WORLD"] for kv in kvs} == {"8"}
        assert sorted(int(kv["LOCAL"]) for kv in kvs) == [0, 1, 2, 3]
        group = {kv["GROUP"] for kv in kvs}
        assert len(group) == 1
        for kv in kvs:
            assert int(kv["RANK"]) == 4 * int(kv["GROUP"]) + int(kv["LOCAL"])
        seen += [int(kv["RANK"]) for kv in kvs]
    assert sorted(seen) == list(range(8))
    # env `workers` keeps the reference's meaning (pods, submit.go:100-101)
    ctr = st["pods"][f"default/{pods[0]}"]["spec"]["containers"][0]
    env = {e["name"]: e.get("value") for e in ctr["env"]}
    assert env["workers"] == "2" and env["gpus"] == "4"


def test_logviewer_deployment_on_k8s(kube):
    """deploy/logviewer.yaml stands in for kubernetes/dashboard/dashboard.yaml: once its pod runs,
    `arena logviewer` resolves the kubernetes-dashboard Endpoints to a per-pod log URL."""
    root = os.path.dirname(HERE)
    with open(os.path.join(root, "deploy", "logviewer.yaml")) as f:
        kube._run("apply", "-f", "-", stdin=f.read())
    cli(kube, "submit", "mpi", "--name", "lv", "--image", "img", "--workers", "2", "python t.py")
    assert "No LOGVIEWER Installed" in cli(kube, "logviewer", "lv")
    (lvpod,) = [k.split("/")[1] for k in _pods(kube) if k.startswith("arena-system/kubernetes-")]
    kube.fake("fake-phase", "arena-system", lvpod, "Running", "mi355x-b")
    for k, p in _pods(kube).items():
        if k.startswith("default/"):
            kube.fake("fake-phase", "default", k.split("/")[1], "Running", "mi355x-a")
    out = cli(kube, "logviewer", "lv")
    chief = next(k.split("/")[1] for k, p in _pods(kube).items()
                 if k.startswith("default/lv-tf-horovod-job-"))
    assert f"10.1.0.2:9090/#!/log/default/{chief}/mpimaster?namespace=default" in out


def test_logviewer_server_with_k8s_backend(kube):
    """The viewer process itself on the K8s backend: job list with status, and pod logs read
    through kubectl."""
    import threading
    import urllib.request
    from http.server import ThreadingHTTPServer
    from arena_amd.runtime.logviewer import make_handler
    cli(kube, "submit", "sj", "--name", "web", "--image", "img", "python x.py")
    pod = next(k.split("/")[1] for k in _pods(kube) if k.startswith("default/web-"))
    kube.fake("fake-phase", "default", pod, "Running", "mi355x-a")
    kube.fake("fake-log", "default", pod, "step 10 loss 0.5")
    srv = ThreadingHTTPServer(("127.0.0.1", 0), make_handler(kube))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        base = f"http://127.0.0.1:{srv.server_address[1]}"
        jobs = json.loads(urllib.request.urlopen(base + "/api/jobs", timeout=30).read())
        assert jobs[0]["name"] == "web" and jobs[0]["status"] == "RUNNING"
        assert jobs[0]["pods"][0]["name"] == pod
        log = urllib.request.urlopen(f"{base}/api/log/default/{pod}?tail=5", timeout=30).read()
        assert log.decode().strip() == "step 10 loss 0.5"
        page = urllib.request.urlopen(base + "/", timeout=30).read().decode()
        assert "#!\\/log" in page or "log/" in page
    finally:
        srv.shutdown()


def test_codec_roundtrip():
    from arena_amd.cluster import charts
    from arena_amd.jobs import spec as S
    a = S.TFJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.ps_count, a.namespace = "rt", "img", 1, 2, 1, "ns1"
    a.prepare(["python", "x.py"])
    st = ClusterState(clock=lambda: 1_700_000_000.0)
    created = st.apply(charts.render(a.chart, "rt", "ns1", a.values()))
    w0 = next(n for (_, n) in st.pods if n.rsplit("-", 1)[0] == "rt-tfjob-worker-0")
    st.set_pod_phase("ns1", w0, "Running")
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
