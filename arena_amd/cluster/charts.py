"""Chart renderers: job kind + values -> Kubernetes manifests (dicts), AMD-first.

Replaces the reference's three Helm charts (charts/training, charts/tfjob, charts/tf-horovod;
SURVEY §2.7) with plain functions. The object names, labels and env contract are preserved
(SURVEY §2.13); the resource model is MI355X-native:
  * GPUs are requested as ``amd.com/gpu`` (the ROCm device plugin exposes /dev/kfd + /dev/dri);
    no NVIDIA driver hostPath mount;
  * allreduce jobs rendezvous through a TCPStore (``MASTER_ADDR``/``MASTER_PORT``/``WORLD_SIZE``/
    ``RANK``) on a headless Service instead of sshd + hostfile + mpirun;
  * allreduce pods get a Memory-backed /dev/shm (RCCL's intra-node transport) and hostIPC;
  * TensorBoard renders for every job kind (quirk Q6 fixed); git sync works everywhere (Q7).
"""
from __future__ import annotations

import copy
from typing import Dict, List

from ..runtime.heartbeat import liveness_probe
from .objects import AMD_GPU

ARENA_SYSTEM_NS = "arena-system"
JOBMON_IMAGE = "arena-amd/jobmon:latest"


def fullname(release: str, chart: str) -> str:
    """<release>-<chart>, or <release> if it already contains the chart name; max 63 chars
    (charts/*/templates/_helpers.tpl:5-32)."""
    name = release if chart in release else f"{release}-{chart}"
    return name[:63].rstrip("-")


def _env_list(envs: Dict[str, str]) -> List[dict]:
    return [{"name": k, "value": str(v)} for k, v in sorted(envs.items())]


def _resources(values: dict, gpus: int, cpu: str = "", memory: str = "") -> dict:
    res: dict = {}
    limits, requests = {}, {}
    if gpus > 0:
        limits[values.get("gpuResource", AMD_GPU)] = gpus
        requests[values.get("gpuResource", AMD_GPU)] = gpus
    if cpu:
        limits["cpu"] = requests["cpu"] = cpu
    if memory:
        limits["memory"] = requests["memory"] = memory
    if limits:
        res["limits"] = limits
    if requests:
        res["requests"] = requests
    return res


def _volumes_and_mounts(values: dict, with_code: bool = True):
    vols, mounts = [], []
    wd = values.get("workingDir", "/root")
    if with_code and values.get("syncMode"):
        vols.append({"name": "code-sync", "emptyDir": {}})
        mounts.append({"name": "code-sync", "mountPath": f"{wd}/code"})
    for name, path in sorted((values.get("dataset") or {}).items()):
        vols.append({"name": name, "persistentVolumeClaim": {"claimName": name}})
        mounts.append({"name": name, "mountPath": path})
    for d in values.get("dataDirs") or []:
        vols.append({"name": d["name"], "hostPath": {"path": d["hostPath"]}})
        mounts.append({"name": d["name"], "mountPath": d["containerPath"]})
    return vols, mounts


def _sync_init_containers(values: dict) -> List[dict]:
    mode = values.get("syncMode")
    if not mode:
        return []
    if mode == "git":
        return [{"name": "git-sync", "image": values.get("syncImage", ""),
                 "env": [{"name": "GIT_SYNC_REPO", "value": values.get("syncSource", "")},
                         {"name": "GIT_SYNC_DEST", "value": values.get("syncGitProjectName", "")},
                         {"name": "GIT_SYNC_ROOT", "value": "/code"},
                         {"name": "GIT_SYNC_ONE_TIME", "value": "true"}],
                 "volumeMounts": [{"name": "code-sync", "mountPath": "/code"}]}]
    return [{"name": "rsync-code", "image": values.get("syncImage") or "rsync:latest",
             "command": ["rsync", "-avP", values.get("syncSource", ""), "/code"],
             "volumeMounts": [{"name": "code-sync", "mountPath": "/code"}]}]


def _container(name: str, values: dict, image: str, gpus: int, cpu="", memory="",
               extra_env=None, mounts=None, ports=None, command=None) -> dict:
    env = dict(values.get("envs") or {})
    env.update(extra_env or {})
    c = {"name": name, "image": image,
         "command": command or ["sh", "-c", values.get("command", "")],
         "workingDir": values.get("workingDir", "/root"),
         "env": _env_list(env), "resources": _resources(values, gpus, cpu, memory),
         "volumeMounts": list(mounts or [])}
    if ports:
        c["ports"] = ports
    hb = float(values.get("heartbeatTimeout", 0) or 0)
    if hb > 0 and name != "tensorboard":
        # hang detection (arena_amd/runtime/heartbeat.py): the kubelet restarts a container
        # whose training-progress file went stale
        path = "/tmp/arena-heartbeat"
        c["env"] = c["env"] + _env_list({"ARENA_HEARTBEAT_FILE": path})
        c["livenessProbe"] = liveness_probe(path, hb)
    return c


def _tensorboard(release: str, ns: str, values: dict, app: str, affinity_labels=None):
    if not values.get("useTensorboard"):
        return []
    name = f"{release}-tensorboard"
    logdir = values.get("trainingLogdir", "/training_logs")
    pod_spec = {"containers": [{
        "name": "tensorboard", "image": values.get("tensorboardImage", ""),
        "command": ["tensorboard", f"--logdir=/output{logdir}", "--host=0.0.0.0",
                    "--port=6006"],
        "ports": [{"containerPort": 6006}],
        "volumeMounts": [{"name": "training-logs", "mountPath": f"/output{logdir}"}]}],
        "volumes": [{"name": "training-logs", "hostPath": {"path": values.get("hostLogPath", "")}}]}
    if affinity_labels:
        pod_spec["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [{
            "labelSelector": {"matchLabels": affinity_labels},
            "topologyKey": "kubernetes.io/hostname"}]}}
    labels = {"app": app, "release": release, "role": "tensorboard"}
    return [
        {"apiVersion": "apps/v1", "kind": "Deployment",
         "metadata": {"name": name, "namespace": ns, "labels": labels},
         "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                  "template": {"metadata": {"labels": labels}, "spec": pod_spec}}},
        {"apiVersion": "v1", "kind": "Service",
         "metadata": {"name": name, "namespace": ns, "labels": labels},
         "spec": {"type": values.get("tensorboardServiceType", "NodePort"), "selector": labels,
                  "ports": [{"port": 6006, "targetPort": 6006, "name": "tensorboard"}]}},
    ]


def _log_mount(values: dict):
    if not values.get("useTensorboard"):
        return [], []
    return ([{"name": "training-logs", "hostPath": {"path": values.get("hostLogPath", "")}}],
            [{"name": "training-logs", "mountPath": values.get("trainingLogdir", "/training_logs")}])


# ---------------------------------------------------------------------------------------------
def render_training(release: str, ns: str, values: dict) -> List[dict]:
    """Standalone job: one batch/v1 Job `<release>-training` (charts/training/templates/job.yaml)."""
    name = f"{release}-training"
    labels = {"app": "training", "release": release}
    vols, mounts = _volumes_and_mounts(values)
    lv, lm = _log_mount(values)
    vols += lv
    mounts += lm
    pod = {"metadata": {"labels": dict(labels)},
           "spec": {"restartPolicy": "Never", "hostNetwork": values.get("useHostNetwork", True),
                    "initContainers": _sync_init_containers(values),
                    "containers": [_container("job", values, values.get("image", ""),
                                              int(values.get("gpuCount", 0)),
                                              values.get("cpu", ""), values.get("memory", ""),
                                              mounts=mounts)],
                    "volumes": vols}}
    out = [{"apiVersion": "batch/v1", "kind": "Job",
            "metadata": {"name": name, "namespace": ns, "labels": {**labels, "role": "job"}},
            "spec": {"backoffLimit": int(values.get("retry", 0)), "template": pod}}]
    return out + _tensorboard(release, ns, values, "training")


def render_tfjob(release: str, ns: str, values: dict) -> List[dict]:
    """PS/worker job: kubeflow.org/v1alpha2 TFJob `<release>-tfjob` (charts/tfjob/templates)."""
    name = f"{release}-tfjob"
    labels = {"app": "tfjob", "release": release}
    vols, mounts = _volumes_and_mounts(values)
    replicas = {}
    ps = int(values.get("ps", 0))
    if ps > 0:
        replicas["PS"] = {"replicas": ps, "restartPolicy": "Never", "template": {
            "metadata": {"labels": dict(labels)},
            "spec": {"hostNetwork": values.get("useHostNetwork", True),
                     "hostPID": values.get("useHostPID", True),
                     "hostIPC": values.get("useHostIPC", True),
                     "initContainers": _sync_init_containers(values),
                     "containers": [_container(
                         "tensorflow", values, values.get("psImage", ""), 0,
                         values.get("psCPU", ""), values.get("psMemory", ""), mounts=mounts,
                         ports=[{"name": "tfjob-port",
                                 "containerPort": int(values.get("psPort", 22223))}])],
                     "volumes": list(vols)}}}
    workers = int(values.get("workers", 1))
    if workers > 0:
        lv, lm = _log_mount(values)
        replicas["Worker"] = {"replicas": workers, "restartPolicy": "Never", "template": {
            "metadata": {"labels": dict(labels)},
            "spec": {"hostNetwork": values.get("useHostNetwork", True),
                     "hostPID": values.get("useHostPID", True),
                     "hostIPC": values.get("useHostIPC", True),
                     "initContainers": _sync_init_containers(values),
                     "containers": [_container(
                         "tensorflow", values, values.get("workerImage", ""),
                         int(values.get("gpuCount", 0)), values.get("workerCPU", ""),
                         values.get("workerMemory", ""), mounts=mounts + lm,
                         ports=[{"name": "tfjob-port",
                                 "containerPort": int(values.get("workerPort", 22222))}])],
                     "volumes": list(vols) + lv}}}
    out = [{"apiVersion": "kubeflow.org/v1alpha2", "kind": "TFJob",
            "metadata": {"name": name, "namespace": ns, "labels": labels},
            "spec": {"cleanPodPolicy": values.get("cleanPodPolicy", "Running"),
                     "tfReplicaSpecs": replicas}}]
    return out + _tensorboard(release, ns, values, "tfjob",
                              affinity_labels={"app": "tfjob", "release": release,
                                               "tf-replica-type": "worker",
                                               "tf-replica-index": "0"})


def render_tf_horovod(release: str, ns: str, values: dict) -> List[dict]:
    """Allreduce job (charts/tf-horovod/templates): launcher Job + worker StatefulSet + headless
    Services + jobmon. Ranks rendezvous on a TCPStore served by the launcher (rank 0) at
    `<fullname>-master:rdzvPort`; the StatefulSet ordinal i is rank i+1."""
    fn = fullname(release, "tf-horovod")
    labels = {"app": "tf-horovod", "release": release}
    world = int(values.get("workers", 0)) + 1
    port = int(values.get("rdzvPort", 29500))
    vols, mounts = _volumes_and_mounts(values)
    lv, lm = _log_mount(values)
    shm = [{"name": "dshm", "emptyDir": {"medium": "Memory",
                                          "sizeLimit": values.get("shmSize", "2Gi")}}]
    shm_m = [{"name": "dshm", "mountPath": "/dev/shm"}]
    rdzv = {"MASTER_ADDR": f"{fn}-master", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
            "HSA_ENABLE_IPC_MODE_LEGACY": "0", "NCCL_SOCKET_IFNAME": "^lo,docker"}
    gpus = int(values.get("gpuCount", 0))
    common_spec = {"hostNetwork": values.get("useHostNetwork", True),
                   "hostIPC": True, "volumes": vols + lv + shm}
    master_cmd = ["sh", "-c", "export RANK=0; " + values.get("command", "")]
    worker_cmd = ["sh", "-c", "export RANK=$(( ${HOSTNAME##*-} + 1 )); " + values.get("command", "")]
    out = [
        {"apiVersion": "v1", "kind": "Service",
         "metadata": {"name": fn, "namespace": ns, "labels": labels},
         "spec": {"clusterIP": "None", "selector": {**labels, "role": "mpiworker"},
                  "ports": [{"port": port, "name": "rdzv"}]}},
        {"apiVersion": "v1", "kind": "Service",
         "metadata": {"name": f"{fn}-master", "namespace": ns, "labels": labels},
         "spec": {"clusterIP": "None", "selector": {**labels, "role": "mpimaster"},
                  "ports": [{"port": port, "name": "rdzv"}]}},
    ]
    if world > 1:
        out.append({
            "apiVersion": "apps/v1", "kind": "StatefulSet",
            "metadata": {"name": fn, "namespace": ns, "labels": labels},
            "spec": {"replicas": world - 1, "podManagementPolicy": "Parallel",
                     "serviceName": fn, "selector": {"matchLabels": {**labels, "role": "mpiworker"}},
                     "template": {"metadata": {"labels": {**labels, "role": "mpiworker"}},
                                  "spec": {**copy.deepcopy(common_spec),
                                           "initContainers": _sync_init_containers(values),
                                           "containers": [_container(
                                               "tf-horovod", values, values.get("image", ""), gpus,
                                               values.get("cpu", ""), values.get("memory", ""),
                                               extra_env=rdzv, mounts=mounts + lm + shm_m,
                                               command=worker_cmd)]}}}})
    out.append({
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": f"{fn}-job", "namespace": ns, "labels": {**labels, "role": "mpimaster"}},
        "spec": {"backoffLimit": int(values.get("retry", 0)),
                 "template": {"metadata": {"labels": {**labels, "role": "mpimaster"}},
                              "spec": {**copy.deepcopy(common_spec), "restartPolicy": "Never",
                                       "initContainers": _sync_init_containers(values),
                                       "containers": [_container(
                                           "mpimaster", values, values.get("image", ""), gpus,
                                           values.get("cpu", ""), values.get("memory", ""),
                                           extra_env=rdzv, mounts=mounts + lm + shm_m,
                                           command=master_cmd)]}}}})
    out.append({
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": f"{fn}-jobmon", "namespace": ARENA_SYSTEM_NS,
                     "labels": {**labels, "role": "jobmon"}},
        "spec": {"template": {"metadata": {"labels": {**labels, "role": "jobmon"}},
                              "spec": {"serviceAccountName": "jobmon", "restartPolicy": "Never",
                                       "containers": [{
                                           "name": "jobmon", "image": JOBMON_IMAGE,
                                           "imagePullPolicy": values.get("jobmonPullPolicy",
                                                                         "IfNotPresent"),
                                           "command": ["arena-jobmon"],
                                           "env": _env_list({"NAMESPACE": ns,
                                                             "JOBNAME": f"{fn}-job",
                                                             "STATEFULSETNAME": fn})}]}}}})
    return out + _tensorboard(release, ns, values, "tf-horovod",
                              affinity_labels={**labels, "role": "mpimaster"})


RENDERERS = {"training": render_training, "tfjob": render_tfjob, "tf-horovod": render_tf_horovod}


def render(chart: str, release: str, ns: str, values: dict) -> List[dict]:
    try:
        fn = RENDERERS[chart]
    except KeyError:
        raise ValueError(f"unknown chart {chart!r} (known: {sorted(RENDERERS)})") from None
    return fn(release, ns, values)
