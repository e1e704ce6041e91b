"""Golden-manifest tests for the chart renderers ("Golden-manifest tests for the K8s
renderer"). The goldens in tests/golden/*.yaml are our rendered output for fixed inputs; set
ARENA_UPDATE_GOLDEN=1 to regenerate after an intended change. Key properties are also asserted
explicitly so a regenerated golden cannot silently drop them."""
from __future__ import annotations

import os

import pytest
import yaml

from arena_amd.cluster import charts
from arena_amd.jobs import spec as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _render(kind: str):
    if kind == "standalone":
        a = S.StandaloneJobArgs()
        a.cpu, a.memory = "8", "32Gi"
    elif kind == "tfjob":
        a = S.TFJobArgs()
        a.ps_count, a.worker_port, a.ps_port = 1, 22222, 22223
        a.tensorboard = S.TensorboardArgs(use_tensorboard=True, training_logdir="/training_logs")
        a.sync = S.SyncCodeArgs(sync_mode="git", sync_source="https://example.com/org/proj.git")
    else:
        a = S.MPIJobArgs()
        a.shm_size = "4Gi"
    a.name, a.image, a.gpu_count, a.namespace = "demo", "rocm/pytorch:latest", 2, "team-a"
    a.workers = 3 if kind != "standalone" else 1
    a.env_list = ["NCCL_DEBUG=WARN"]
    a.data_dir_list = ["/data/mnist:/mnist"]
    a.dataset_list = ["imagenet-pvc:/imagenet"]
    if kind == "tfjob":
        a.prepare(["python", "dist.py", "--logdir", "/training_logs"])
    else:
        a.prepare(["python", "train.py"])
    if kind == "tfjob":
        # hostLogPath carries a random 9-digit suffix (RandomInt32): pin it for the golden
        a.tensorboard.host_log_path = "/arena_logs/training000000001"
    return charts.render(a.chart, "demo", "team-a", a.values())


@pytest.mark.parametrize("kind", ["standalone", "tfjob", "mpijob"])
def test_manifest_golden(kind):
    docs = _render(kind)
    text = yaml.safe_dump_all(docs, sort_keys=True)
    path = os.path.join(GOLDEN, f"{kind}.yaml")
    if os.environ.get("ARENA_UPDATE_GOLDEN") or not os.path.exists(path):
        os.makedirs(GOLDEN, exist_ok=True)
        with open(path, "w") as f:
            f.write(text)
    with open(path) as f:
        assert text == f.read(), f"{kind} manifests changed; set ARENA_UPDATE_GOLDEN=1 if intended"


def _containers(doc):
    spec = doc["spec"]
    if doc["kind"] == "TFJob":
        return [c for r in spec["tfReplicaSpecs"].values() for c in r["template"]["spec"]["containers"]]
    return spec["template"]["spec"]["containers"]


def test_standalone_properties():
    (job,) = [d for d in _render("standalone") if d["kind"] == "Job"]
    assert job["metadata"]["name"] == "demo-training"
    assert job["metadata"]["labels"] == {"app": "training", "release": "demo", "role": "job"} or \
        job["metadata"]["labels"]["app"] == "training"
    (c,) = _containers(job)
    assert c["resources"]["limits"]["amd.com/gpu"] == 2
    env = {e["name"]: e["value"] for e in c["env"]}
    assert env["NCCL_DEBUG"] == "WARN" and env["workers"] == "1" and env["gpus"] == "2"
    assert job["spec"]["backoffLimit"] == 0
    vols = {v["name"]: v for v in job["spec"]["template"]["spec"]["volumes"]}
    # /dev/kfd + /dev/dri come from the amdgpu device plugin with the amd.com/gpu allocation
    assert any(v.get("persistentVolumeClaim", {}).get("claimName") == "imagenet-pvc"
               for v in vols.values())


def test_tfjob_properties():
    docs = _render("tfjob")
    (tf,) = [d for d in docs if d["kind"] == "TFJob"]
    reps = tf["spec"]["tfReplicaSpecs"]
    assert reps["PS"]["replicas"] == 1 and reps["Worker"]["replicas"] == 3
    ps_c = reps["PS"]["template"]["spec"]["containers"][0]
    wk_c = reps["Worker"]["template"]["spec"]["containers"][0]
    assert "amd.com/gpu" not in (ps_c.get("resources") or {}).get("limits", {})
    assert wk_c["resources"]["limits"]["amd.com/gpu"] == 2
    assert any(p["containerPort"] == 22222 for p in wk_c["ports"])
    assert any(p["containerPort"] == 22223 for p in ps_c["ports"])
    kinds = sorted(d["kind"] for d in docs)
    assert kinds == ["Deployment", "Service", "TFJob"]
    (dep,) = [d for d in docs if d["kind"] == "Deployment"]
    aff = dep["spec"]["template"]["spec"]["affinity"]["podAffinity"]
    assert aff  # TensorBoard pinned next to worker-0 (shared hostPath log dir)
    init = reps["Worker"]["template"]["spec"].get("initContainers") or []
    assert init and any("GIT_SYNC_REPO" in str(i) for i in init)   # Q7 fixed: git sync works


def test_mpijob_properties():
    docs = _render("mpijob")
    by = {(d["kind"], d["metadata"]["name"]): d for d in docs}
    job = by[("Job", "demo-tf-horovod-job")]
    ss = by[("StatefulSet", "demo-tf-horovod")]
    assert ss["spec"]["replicas"] == 2                       # workers - 1 (the launcher ranks too)
    jm = by[("Job", "demo-tf-horovod-jobmon")]
    assert jm["metadata"]["namespace"] == "arena-system"
    jenv = {e["name"]: e["value"] for e in _containers(jm)[0]["env"]}
    assert jenv == {**jenv, "NAMESPACE": "team-a", "JOBNAME": "demo-tf-horovod-job",
                    "STATEFULSETNAME": "demo-tf-horovod"}
    for d in (job, ss):
        c = _containers(d)[0]
        env = {e["name"]: e.get("value") for e in c["env"]}
        assert env["WORLD_SIZE"] == "3" and env["MASTER_PORT"] == "29500"
        assert env["MASTER_ADDR"] == "demo-tf-horovod-master"
        vols = d["spec"]["template"]["spec"]["volumes"]
        shm = [v for v in vols if v.get("emptyDir", {}).get("medium") == "Memory"]
        assert shm and shm[0]["emptyDir"]["sizeLimit"] == "4Gi"
        assert d["spec"]["template"]["spec"].get("hostIPC") is True
    assert "export RANK=0" in " ".join(_containers(job)[0]["command"])
    assert "HOSTNAME##*-" in " ".join(_containers(ss)[0]["command"])


def test_heartbeat_timeout_renders_liveness_probe():
    """--heartbeatTimeout: every training container gets the heartbeat file env and an exec
    livenessProbe on its age; jobmon and TensorBoard stay unprobed (they never beat)."""
    import subprocess
    import tempfile
    a = S.MPIJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.heartbeat_timeout = "hb", "img", 1, 2, 30.0
    a.prepare(["python", "train.py"])
    docs = charts.render(a.chart, "hb", "default", a.values())
    probed = 0
    for d in docs:
        if d["kind"] not in ("Job", "StatefulSet"):
            continue
        c = _containers(d)[0]
        if d["metadata"]["name"].endswith("jobmon"):
            assert "livenessProbe" not in c
            continue
        env = {e["name"]: e.get("value") for e in c["env"]}
        assert env["ARENA_HEARTBEAT_FILE"] == "/tmp/arena-heartbeat"
        probe = c["livenessProbe"]
        assert probe["initialDelaySeconds"] == 30 and probe["failureThreshold"] == 1
        probed += 1
        # the probe script itself: passes with no file / a fresh file, fails on a stale one
        script = probe["exec"]["command"][2]
        with tempfile.TemporaryDirectory() as td:
            f = os.path.join(td, "hb")
            s = script.replace("/tmp/arena-heartbeat", f)
            assert subprocess.run(["sh", "-c", s]).returncode == 0          # not started yet
            open(f, "w").close()
            assert subprocess.run(["sh", "-c", s]).returncode == 0          # fresh beat
            os.utime(f, (0, 0))
            assert subprocess.run(["sh", "-c", s]).returncode != 0          # stale: restart
    assert probed == 2
    # default: nothing rendered
    b = S.MPIJobArgs()
    b.name, b.image, b.workers = "nohb", "img", 2
    b.prepare(["python", "train.py"])
    assert all("livenessProbe" not in str(d) for d in charts.render(b.chart, "nohb", "default",
                                                                     b.values()))
