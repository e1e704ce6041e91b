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


def _env(c):
    return {e["name"]: e.get("value") for e in c["env"]}


def test_tfjob_properties():
    """Operator-free PS/worker job: a Job + headless Service per task, TF_CONFIG from the
    Services' stable DNS names, tf-operator's pod labels, cleanPodPolicy by jobmon."""
    import json
    docs = _render("tfjob")
    by = {(d["kind"], d["metadata"]["name"]): d for d in docs}
    tasks = ["demo-tfjob-ps-0"] + [f"demo-tfjob-worker-{i}" for i in range(3)]
    assert not [d for d in docs if d["kind"] == "TFJob"]
    # hostNetwork: per-task ports (workers 22222.., the PS skips the workers' range)
    want_cluster = {"ps": ["demo-tfjob-ps-0.team-a.svc:22225"],
                    "worker": [f"demo-tfjob-worker-{i}.team-a.svc:{22222 + i}" for i in range(3)]}
    for t in tasks:
        job, svc = by[("Job", t)], by[("Service", t)]
        tpl = job["spec"]["template"]
        labels = tpl["metadata"]["labels"]
        rtype, idx = t.split("-")[-2], int(t.split("-")[-1])
        assert labels["group_name"] == "kubeflow.org" and labels["tf-replica-type"] == rtype
        assert labels["tf-replica-index"] == str(idx) and labels["app"] == "tfjob"
        assert svc["spec"]["clusterIP"] == "None"
        assert all(labels[k] == v for k, v in svc["spec"]["selector"].items())
        (c,) = tpl["spec"]["containers"]
        tfc = json.loads(_env(c)["TF_CONFIG"])
        assert tfc == {"cluster": want_cluster, "task": {"type": rtype, "index": idx},
                       "environment": "cloud"}
        assert _env(c)["MX_CLUSTER_SPEC"] == _env(c)["TF_CONFIG"]
        port = 22225 if rtype == "ps" else 22222 + idx
        assert [p["containerPort"] for p in c["ports"]] == [port]
        assert svc["spec"]["ports"][0]["port"] == port
        gpus = (c.get("resources") or {}).get("limits", {}).get("amd.com/gpu")
        assert gpus == (None if rtype == "ps" else 2)
        assert tpl["spec"]["hostNetwork"] is True
        assert tpl["spec"]["dnsPolicy"] == "ClusterFirstWithHostNet"   # Service names resolve
        assert tpl["spec"]["restartPolicy"] == "Never"
        init = tpl["spec"].get("initContainers") or []
        assert init and any("GIT_SYNC_REPO" in str(i) for i in init)   # Q7 fixed: git sync works
    jm = by[("Job", "demo-tfjob-jobmon")]
    assert jm["metadata"]["namespace"] == "arena-system"
    jenv = _env(_containers(jm)[0])
    assert jenv["TFJOBNAME"] == "demo-tfjob" and jenv["CLEANPODPOLICY"] == "Running"
    assert jenv["RELEASE"] == "demo" and jenv["NAMESPACE"] == "team-a"
    (dep,) = [d for d in docs if d["kind"] == "Deployment"]
    aff = dep["spec"]["template"]["spec"]["affinity"]["podAffinity"]
    sel = aff["requiredDuringSchedulingIgnoredDuringExecution"][0]["labelSelector"]["matchLabels"]
    w0 = by[("Job", "demo-tfjob-worker-0")]["spec"]["template"]["metadata"]["labels"]
    assert all(w0[k] == v for k, v in sel.items())   # TensorBoard pinned next to worker-0


def test_tfjob_operator_mode_renders_crd():
    a = S.TFJobArgs()
    a.name, a.image, a.workers, a.ps_count, a.tf_operator = "op", "img", 2, 1, True
    a.prepare(["python", "x.py"])
    docs = charts.render(a.chart, "op", "default", a.values())
    (tf,) = [d for d in docs if d["kind"] == "TFJob"]
    reps = tf["spec"]["tfReplicaSpecs"]
    assert reps["PS"]["replicas"] == 1 and reps["Worker"]["replicas"] == 2
    assert not [d for d in docs if d["kind"] == "Job"]


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
        # 3 pods x 2 GPUs: one rank per GPU through the in-pod launcher
        assert env["WORLD_SIZE"] == "6" and env["MASTER_PORT"] == "29500"
        assert env["ARENA_RANKS_PER_POD"] == "2" and env["ARENA_PODS"] == "3"
        assert env["ARENA_RANK_COMMAND"] == "python train.py"
        assert env["MASTER_ADDR"] == "demo-tf-horovod-master"
        vols = d["spec"]["template"]["spec"]["volumes"]
        shm = [v for v in vols if v.get("emptyDir", {}).get("medium") == "Memory"]
        assert shm and shm[0]["emptyDir"]["sizeLimit"] == "4Gi"
        assert d["spec"]["template"]["spec"].get("hostIPC") is True
    assert "export ARENA_POD_INDEX=0" in " ".join(_containers(job)[0]["command"])
    assert "arena_amd.runtime.podlaunch" in " ".join(_containers(job)[0]["command"])
    # the worker pod index comes from the pod name (downward API), not $HOSTNAME (= node under
    # hostNetwork); tests/test_k8s_backend.py runs it on a fake node with several workers
    wc = _containers(ss)[0]
    assert "arena_amd.runtime.podlaunch" in " ".join(wc["command"])
    assert "HOSTNAME" not in " ".join(wc["command"])
    assert {"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}} \
        in wc["env"]
    # one rank per pod keeps the launcher-free form (any image, no arena_amd inside)
    a = S.MPIJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.ranks_per_pod = "one", "img", 2, 3, 1
    a.prepare(["python", "train.py"])
    one = {(d["kind"], d["metadata"]["name"]): d
           for d in charts.render(a.chart, "one", "default", a.values())}
    assert "export RANK=0" in " ".join(_containers(one[("Job", "one-tf-horovod-job")])[0]["command"])
    wc1 = _containers(one[("StatefulSet", "one-tf-horovod")])[0]
    assert "POD_NAME##*-" in " ".join(wc1["command"])
    assert {e["name"]: e.get("value") for e in wc1["env"]}["WORLD_SIZE"] == "3"
    for d in (job, ss):
        assert d["spec"]["template"]["spec"]["dnsPolicy"] == "ClusterFirstWithHostNet"


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
        env = _env(c)
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


def test_jobmon_image_runs_the_rendered_command():
    """The jobmon Job's command exists in the image deploy/jobmon.Dockerfile builds: the package
    is copied onto PYTHONPATH, the module imports without torch (the image has none), and the
    `arena-jobmon` console script is installed as well."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(GOLDEN))
    docker = open(os.path.join(root, "deploy", "jobmon.Dockerfile")).read()
    assert "COPY arena_amd /opt/arena/arena_amd" in docker and "PYTHONPATH=/opt/arena" in docker
    assert "/usr/local/bin/arena-jobmon" in docker and "kubectl" in docker
    for d in _render("mpijob"):
        if d["metadata"]["name"].endswith("jobmon"):
            cmd = _containers(d)[0]["command"]
            assert cmd == list(charts.JOBMON_COMMAND)
            assert _containers(d)[0]["image"] == charts.JOBMON_IMAGE
    mod = charts.JOBMON_COMMAND[2]
    probe = ("import sys; sys.modules['torch'] = None; import importlib; "
             f"importlib.import_module({mod!r}); import arena_amd.cluster.k8s")
    r = subprocess.run([sys.executable, "-c", probe], cwd=root, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # without its env it exits 2 with a clear message (no traceback, no hang)
    env = {k: v for k, v in os.environ.items()
           if k not in ("NAMESPACE", "JOBNAME", "STATEFULSETNAME", "TFJOBNAME")}
    env["PYTHONPATH"] = root
    r = subprocess.run([sys.executable, "-m", mod], cwd=root, env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 2 and "Failed to get namespace" in r.stderr


def test_mpijob_ranks_per_pod_validation():
    from arena_amd.jobs.spec import ValidationError
    for rpp, gpus in ((3, 2), (0, 1), (-2, 1)):
        a = S.MPIJobArgs()
        a.name, a.image, a.gpu_count, a.ranks_per_pod = "x", "img", gpus, rpp
        with pytest.raises(ValidationError):
            a.prepare(["true"])
    a = S.MPIJobArgs()
    a.name, a.image, a.gpu_count, a.ranks_per_pod = "x", "img", 0, 4   # CPU ranks: allowed
    a.prepare(["true"])
    assert a.values()["ranksPerPod"] == 4


def test_mpijob_jupyter_master():
    """--jupyter: the launcher pod serves a notebook on 8888 behind <fullname>-jupyter
    (charts/tf-horovod/templates/service.yaml:47-67, job.yaml:148-153)."""
    a = S.MPIJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.jupyter = "nb", "img", 1, 2, True
    a.prepare(["python", "train.py"])
    docs = {(d["kind"], d["metadata"]["name"]): d
            for d in charts.render(a.chart, "nb", "default", a.values())}
    svc = docs[("Service", "nb-tf-horovod-jupyter")]
    assert svc["spec"]["type"] == "NodePort" and svc["spec"]["ports"][0]["port"] == 8888
    assert svc["spec"]["selector"]["role"] == "mpimaster"
    mc = _containers(docs[("Job", "nb-tf-horovod-job")])[0]
    assert "jupyter notebook" in mc["command"][2] and "/run_jupyter.sh" in mc["command"][2]
    assert mc["ports"] == [{"name": "jupyter", "containerPort": 8888}]
    wc = _containers(docs[("StatefulSet", "nb-tf-horovod")])[0]
    assert "train.py" in " ".join(wc["command"])         # workers still start their ranks


def test_tfjob_eight_workers_fit_one_node():
    """hostNetwork PS/worker job with 8 workers + 1 PS: every task on one 8-GPU node binds its
    own port, and TF_CONFIG, the Services and the containerPorts agree."""
    import json
    a = S.TFJobArgs()
    a.name, a.image, a.gpu_count, a.workers, a.ps_count = "big", "img", 1, 8, 1
    a.prepare(["python", "dist.py"])
    docs = charts.render(a.chart, "big", "default", a.values())
    ports, cluster = {}, None
    for d in docs:
        if d["kind"] == "Job" and "tf-replica-type" in d["metadata"]["labels"]:
            c = _containers(d)[0]
            ports[d["metadata"]["name"]] = c["ports"][0]["containerPort"]
            tfc = json.loads(_env(c)["TF_CONFIG"])
            cluster = cluster or tfc["cluster"]
            assert tfc["cluster"] == cluster
    assert len(ports) == 9 and len(set(ports.values())) == 9        # no two tasks share a port
    svc = {d["metadata"]["name"]: d["spec"]["ports"][0]["port"] for d in docs
           if d["kind"] == "Service" and d["metadata"]["name"] in ports}
    assert svc == ports
    for t, addrs in cluster.items():
        for i, addr in enumerate(addrs):
            assert int(addr.rsplit(":", 1)[1]) == ports[f"big-tfjob-{t}-{i}"]
    # pod networking: every pod has its own IP, the base ports are kept
    v = dict(a.values(), useHostNetwork=False)
    assert set(charts.task_ports(v)["worker"]) == {22222}


def test_mpijob_default_ranks_per_pod_with_8_gpus_renders_launcher():
    """The default for ``--gpus 8``: 8 ranks per pod through the in-pod launcher (ADVICE r4:
    the behaviour change is explicit). The pod command checks that arena_amd is importable in
    the user's image and names the fixes (install it, or --ranksPerPod 1) before exec."""
    import subprocess
    a = S.MPIJobArgs()
    a.name, a.image, a.gpu_count, a.workers = "big", "rocm/pytorch:latest", 8, 2
    a.prepare(["python", "train.py"])
    assert a.values()["ranksPerPod"] == 8
    docs = {(d["kind"], d["metadata"]["name"]): d
            for d in charts.render(a.chart, "big", "default", a.values())}
    job, ss = docs[("Job", "big-tf-horovod-job")], docs[("StatefulSet", "big-tf-horovod")]
    for d in (job, ss):
        c = _containers(d)[0]
        env = _env(c)
        assert env["WORLD_SIZE"] == "16" and env["ARENA_RANKS_PER_POD"] == "8"
        assert c["resources"]["limits"]["amd.com/gpu"] == 8
        cmd = c["command"]
        assert cmd[:2] == ["sh", "-c"] and "import arena_amd.runtime.podlaunch" in cmd[2]
        assert "--ranksPerPod 1" in cmd[2] and cmd[2].rstrip().endswith(
            "exec python3 -m arena_amd.runtime.podlaunch")
    # an image without arena_amd: the pod command exits 127 with the message (run it here with a
    # python3 that cannot import it)
    cmd = _containers(ss)[0]["command"][2]
    r = subprocess.run(["sh", "-c", cmd], env={"PATH": os.environ["PATH"], "HOME": "/tmp",
                                               "PYTHONPATH": "/nonexistent", "PYTHONNOUSERSITE": "1"},
                       capture_output=True, text=True, timeout=60, cwd="/tmp")
    assert r.returncode == 127 and "--ranksPerPod 1" in r.stderr, (r.returncode, r.stderr)
