"""Kubernetes backend: the charts' manifests applied with ``kubectl`` (no helm, no Tiller).

Plays the roles of the reference's helm wrapper (install/check/delete/list
releases) and its client-go reads (K1/K2, §2.4 "K8s API surface"):

* a *release* is the rendered manifest set plus a record ConfigMap ``arena-release-<name>``
  (labels ``arena.amd.com/release=<name>``, ``arena.amd.com/owner=arena``) holding the values and
  manifests -- the same thing helm stores in its release ConfigMaps;
* install = ``kubectl apply -f -`` of the record + manifests; delete = ``kubectl delete`` of every
  object the record lists (all names, quirk Q7 fixed); list = record ConfigMaps in all namespaces;
* reads = ``kubectl get <kind> -o json`` parsed by :mod:`k8s_json`; logs = ``kubectl logs``
  streamed line by line (``--since``/``--since-time``/``--tail``/``--timestamps``/``-f``).

``kubectl`` is found on PATH or via ``$ARENA_KUBECTL``; ``--config``/``$KUBECONFIG`` is passed
through as ``--kubeconfig``.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import time
from typing import Dict, Iterator, List, Optional

import yaml

from ..utils.logs import get_logger
from ..utils.timefmt import rfc3339
from . import charts, k8s_json
from .backend import Backend, BackendError, Release
from .objects import POD_FAILED, POD_SUCCEEDED, matches

log = get_logger("k8s")
RECORD_PREFIX = "arena-release-"
OWNER_LABEL = "arena.amd.com/owner"
RELEASE_LABEL = "arena.amd.com/release"

# kind -> kubectl resource name (plural) used for delete/get
_RESOURCE = {"Job": "jobs.batch", "StatefulSet": "statefulsets.apps", "Service": "services",
             "TFJob": "tfjobs.kubeflow.org", "Deployment": "deployments.apps",
             "ConfigMap": "configmaps", "Pod": "pods"}


def _selector(sel: Optional[dict]) -> List[str]:
    return ["-l", ",".join(f"{k}={v}" for k, v in sel.items())] if sel else []


class K8sBackend(Backend):
    name = "k8s"

    def __init__(self, kubeconfig: str = "", home: str = "", kubectl: Optional[str] = None):
        self.kubectl = kubectl or os.environ.get("ARENA_KUBECTL") or shutil.which("kubectl")
        if not self.kubectl:
            raise BackendError("kubectl not found (install it or set $ARENA_KUBECTL); "
                               "the local backend needs no cluster: --backend local")
        self.kubeconfig = kubeconfig
        self.home = home

    # ----------------------------------------------------------------------------- kubectl
    def _cmd(self, *args: str) -> List[str]:
        cmd = [self.kubectl]
        if self.kubeconfig:
            cmd += ["--kubeconfig", self.kubeconfig]
        return cmd + list(args)

    def _run(self, *args: str, stdin: Optional[str] = None, check: bool = True) -> str:
        r = subprocess.run(self._cmd(*args), input=stdin, capture_output=True, text=True)
        if check and r.returncode != 0:
            raise BackendError(f"kubectl {' '.join(args[:3])}: {r.stderr.strip() or r.stdout.strip()}")
        return r.stdout

    def _get(self, resource: str, namespace: Optional[str], selector=None) -> List[dict]:
        ns = ["-A"] if namespace is None else ["-n", namespace]
        if resource == "nodes":
            ns = []
        try:
            out = self._run("get", resource, *ns, *_selector(selector), "-o", "json")
        except BackendError as e:
            if resource == "tfjobs" and "the server doesn't have a resource type" in str(e):
                return []  # tf-operator CRD not installed: no TFJobs
            raise
        return (json.loads(out or "{}").get("items")) or []

    def _get_one(self, resource: str, namespace: str, name: str) -> Optional[dict]:
        r = subprocess.run(self._cmd("get", resource, name, "-n", namespace, "-o", "json"),
                           capture_output=True, text=True)
        if r.returncode != 0:
            if "NotFound" in r.stderr or "not found" in r.stderr:
                return None
            raise BackendError(f"kubectl get {resource} {name}: {r.stderr.strip()}")
        return json.loads(r.stdout)

    # ------------------------------------------------------------------------ release store
    def _records(self) -> List[dict]:
        return self._get("configmaps", None, {OWNER_LABEL: "arena"})

    def _record(self, name: str) -> Optional[dict]:
        for cm in self._records():
            if cm["metadata"]["name"] == RECORD_PREFIX + name:
                return cm
        return None

    def release_exists(self, name) -> bool:
        return self._record(name) is not None

    def install_release(self, name, namespace, chart, values) -> Release:
        if self.release_exists(name):
            raise BackendError(f"the job {name} is already exist, please delete it first. "
                               f"use 'arena delete {name}'")
        manifests = charts.render(chart, name, namespace, values)
        created = time.time()
        record = {"apiVersion": "v1", "kind": "ConfigMap",
                  "metadata": {"name": RECORD_PREFIX + name, "namespace": namespace,
                               "labels": {OWNER_LABEL: "arena", RELEASE_LABEL: name,
                                          "chart": chart}},
                  "data": {"chart": chart, "created": rfc3339(created),
                           "values": json.dumps(values), "manifests": json.dumps(manifests)}}
        docs = yaml.safe_dump_all([record] + manifests, sort_keys=False)
        self._run("apply", "-f", "-", stdin=docs)
        return Release(name, namespace, chart, values, manifests, created)

    def get_release(self, name):
        cm = self._record(name)
        if cm is None:
            return None
        d = cm.get("data") or {}
        created = k8s_json._t(d.get("created")) or 0.0
        return Release(name, cm["metadata"].get("namespace", "default"), d.get("chart", ""),
                       json.loads(d.get("values") or "{}"), json.loads(d.get("manifests") or "[]"),
                       created)

    def delete_release(self, name) -> None:
        rel = self.get_release(name)
        if rel is None:
            raise BackendError(f"release: \"{name}\" not found")
        for m in reversed(rel.manifests):
            res = _RESOURCE.get(m["kind"], m["kind"].lower() + "s")
            ns = m["metadata"].get("namespace", rel.namespace)
            self._run("delete", res, m["metadata"]["name"], "-n", ns, "--ignore-not-found",
                      "--wait=false")
        self._run("delete", "configmaps", RECORD_PREFIX + name, "-n", rel.namespace,
                  "--ignore-not-found", "--wait=false")

    def list_releases(self) -> Dict[str, str]:
        return {cm["metadata"]["labels"][RELEASE_LABEL]: cm["metadata"].get("namespace", "default")
                for cm in self._records()}

    # --------------------------------------------------------------------------- cluster reads
    def list_pods(self, namespace=None, selector=None, active_only=False):
        pods = [k8s_json.pod_from(o) for o in self._get("pods", namespace, selector)]
        if active_only:
            pods = [p for p in pods if p.phase not in (POD_SUCCEEDED, POD_FAILED)]
        return pods

    def list_jobs(self, namespace=None, selector=None):
        return [k8s_json.job_from(o) for o in self._get("jobs.batch", namespace, selector)]

    def list_tfjobs(self, namespace=None, selector=None):
        return [k8s_json.tfjob_from(o) for o in self._get("tfjobs.kubeflow.org", namespace, selector)]

    def list_nodes(self):
        return [k8s_json.node_from(o) for o in self._get("nodes", None)]

    def list_services(self, namespace, selector=None):
        return [k8s_json.service_from(o) for o in self._get("services", namespace, selector)
                if matches(o.get("metadata", {}).get("labels") or {}, selector)]

    def get_endpoints(self, namespace, name):
        o = self._get_one("endpoints", namespace, name)
        return k8s_json.endpoints_from(o) if o else None

    def get_pod(self, namespace, name):
        o = self._get_one("pods", namespace, name)
        return k8s_json.pod_from(o) if o else None

    def get_job(self, namespace, name):
        o = self._get_one("jobs.batch", namespace, name)
        return k8s_json.job_from(o) if o else None

    def get_statefulset(self, namespace, name):
        o = self._get_one("statefulsets.apps", namespace, name)
        return k8s_json.statefulset_from(o) if o else None

    def delete_statefulset(self, namespace, name):
        self._run("delete", "statefulsets.apps", name, "-n", namespace, "--wait=false")

    def delete_service(self, namespace, name):
        self._run("delete", "services", name, "-n", namespace, "--wait=false")

    def delete_job(self, namespace, name):
        # background propagation: the Job's pods are garbage-collected with it
        self._run("delete", "jobs.batch", name, "-n", namespace, "--cascade=background",
                  "--wait=false")

    def ensure_namespace(self, namespace):
        if self._run("get", "namespace", namespace, check=False).strip():
            return
        r = subprocess.run(self._cmd("create", "namespace", namespace), capture_output=True,
                           text=True)
        if r.returncode != 0 and "AlreadyExists" not in r.stderr:
            raise BackendError(f"create namespace {namespace}: {r.stderr.strip()}")

    def pod_logs(self, namespace, pod, follow=False, since_seconds=None, since_time=None, tail=-1,
                 timestamps=False) -> Iterator[str]:
        args = ["logs", pod, "-n", namespace]
        if follow:
            args.append("--follow")
        if since_seconds is not None:
            args.append(f"--since={int(since_seconds)}s")
        if since_time is not None:
            args.append(f"--since-time={rfc3339(since_time)}")
        if tail is not None and tail >= 0:
            args.append(f"--tail={tail}")
        if timestamps:
            args.append("--timestamps")
        p = subprocess.Popen(self._cmd(*args), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True)
        try:
            for line in p.stdout:
                yield line if line.endswith("\n") else line + "\n"
        finally:
            if p.poll() is None:
                p.terminate()
            p.wait()
        if p.returncode not in (0, None, -15):
            raise BackendError(f"kubectl logs {pod}: {p.stderr.read().strip()}")
