"""In-memory cluster backend for tests (the role client-go's fake clientset would play; the
reference ships none -- SURVEY §4). Scheduling and pod lifecycle are driven explicitly by tests:
``schedule()`` binds pending pods to nodes with free GPUs; ``set_phase()`` moves a pod along.
"""
from __future__ import annotations

import time
from typing import Dict, Iterator, List, Optional

from . import charts
from .backend import Backend, BackendError, Release
from .controller import ClusterState
from .objects import (AMD_GPU, GPU_RESOURCES, MASTER_LABEL, Endpoints, Meta, Node, Pod,
                      POD_FAILED, POD_PENDING, POD_RUNNING, POD_SUCCEEDED, matches)


def make_node(name: str, ip: str, gpus: int = 0, master: bool = False,
              resource: str = AMD_GPU, extra_addresses=None) -> Node:
    labels = {"kubernetes.io/hostname": name}
    if master:
        labels[MASTER_LABEL] = ""
    addrs = list(extra_addresses or []) + [("InternalIP", ip), ("Hostname", name)]
    cap = {resource: gpus} if gpus else {}
    return Node(meta=Meta(name=name, namespace="", labels=labels), capacity=cap, addresses=addrs)


class FakeBackend(Backend):
    name = "fake"

    def __init__(self, nodes: Optional[List[Node]] = None, clock=time.time):
        self.clock = clock
        self.state = ClusterState(clock=clock)
        for n in nodes or []:
            self.state.nodes[n.name] = n
        self.releases: Dict[str, Release] = {}
        self.logs: Dict[tuple, List[tuple]] = {}  # (ns, pod) -> [(t, line)]
        self.deleted: List[str] = []

    # ---- releases --------------------------------------------------------------------------
    def install_release(self, name, namespace, chart, values) -> Release:
        if name in self.releases:
            raise BackendError(f"the job {name} is already exist, please delete it first. "
                               f"use 'arena delete {name}'")
        manifests = charts.render(chart, name, namespace, values)
        rel = Release(name, namespace, chart, values, manifests, self.clock())
        self.state.apply(manifests)
        self.state.reconcile()
        self.releases[name] = rel
        return rel

    def release_exists(self, name) -> bool:
        return name in self.releases

    def get_release(self, name):
        return self.releases.get(name)

    def delete_release(self, name) -> None:
        if name not in self.releases:
            raise BackendError(f"release {name} not found")
        self.state.delete_release_objects(name)
        del self.releases[name]
        self.deleted.append(name)

    def list_releases(self) -> Dict[str, str]:
        return {n: r.namespace for n, r in self.releases.items()}

    # ---- reads -----------------------------------------------------------------------------
    def list_pods(self, namespace=None, selector=None, active_only=False) -> List[Pod]:
        out = []
        for p in self.state.pods.values():
            if namespace and p.namespace != namespace:
                continue
            if not matches(p.meta.labels, selector):
                continue
            if active_only and p.phase in (POD_SUCCEEDED, POD_FAILED):
                continue
            out.append(p)
        return out

    def list_jobs(self, namespace=None, selector=None):
        return [j for j in self.state.jobs.values()
                if (not namespace or j.meta.namespace == namespace)
                and matches(j.meta.labels, selector)]

    def list_tfjobs(self, namespace=None, selector=None):
        return [t for t in self.state.tfjobs.values()
                if (not namespace or t.meta.namespace == namespace)
                and matches(t.meta.labels, selector)]

    def list_nodes(self):
        return list(self.state.nodes.values())

    def list_services(self, namespace, selector=None):
        return [s for s in self.state.services.values()
                if s.meta.namespace == namespace and matches(s.meta.labels, selector)]

    def get_endpoints(self, namespace, name):
        return self.state.endpoints.get((namespace, name))

    def get_pod(self, namespace, name):
        return self.state.pods.get((namespace, name))

    def get_job(self, namespace, name):
        return self.state.jobs.get((namespace, name))

    def get_statefulset(self, namespace, name):
        return self.state.statefulsets.get((namespace, name))

    def delete_statefulset(self, namespace, name):
        ss = self.state.statefulsets.pop((namespace, name), None)
        if ss is None:
            raise BackendError(f"statefulsets \"{name}\" not found")
        for key in [k for k, p in self.state.pods.items()
                    if k[0] == namespace and "StatefulSet" in p.meta.owner_kinds
                    and k[1].rsplit("-", 1)[0] == name]:
            del self.state.pods[key]

    def delete_service(self, namespace, name):
        if self.state.services.pop((namespace, name), None) is None:
            raise BackendError(f"services \"{name}\" not found")

    def delete_job(self, namespace, name):
        if self.state.jobs.pop((namespace, name), None) is None:
            raise BackendError(f"jobs.batch \"{name}\" not found")
        for key in [k for k, p in self.state.pods.items()
                    if k[0] == namespace and "Job" in p.meta.owner_kinds
                    and k[1].rsplit("-", 1)[0] == name]:
            del self.state.pods[key]

    def ensure_namespace(self, namespace):
        self.state.namespaces.add(namespace)

    def pod_logs(self, namespace, pod, follow=False, since_seconds=None, since_time=None,
                 tail=-1, timestamps=False) -> Iterator[str]:
        if (namespace, pod) not in self.state.pods:
            raise BackendError(f"pods \"{pod}\" not found")
        lines = list(self.logs.get((namespace, pod), []))
        now = self.clock()
        if since_seconds is not None:
            lines = [x for x in lines if x[0] >= now - since_seconds]
        if since_time is not None:
            lines = [x for x in lines if x[0] >= since_time]
        if tail is not None and tail >= 0:
            lines = lines[-tail:] if tail else []
        from ..utils.timefmt import rfc3339
        for t, line in lines:
            yield (f"{rfc3339(t)} {line}\n" if timestamps else f"{line}\n")

    # ---- test drivers ----------------------------------------------------------------------
    def add_endpoints(self, namespace, name, ip, port):
        self.state.endpoints[(namespace, name)] = Endpoints(
            meta=Meta(name=name, namespace=namespace), addresses=[ip], ports=[port])

    def add_log(self, namespace, pod, line, t=None):
        self.logs.setdefault((namespace, pod), []).append((self.clock() if t is None else t, line))

    def set_phase(self, namespace, pod, phase, node=None, exit_code=None):
        self.state.set_pod_phase(namespace, pod, phase, node, exit_code)

    def schedule(self) -> List[Pod]:
        """Bind every pending, unscheduled pod to the first node with enough free GPUs and mark
        it Running (a deterministic stand-in for kube-scheduler + kubelet)."""
        bound = []
        for pod in sorted(self.state.pods.values(), key=lambda p: (p.meta.creation_timestamp, p.name)):
            if pod.phase != POD_PENDING or pod.node_name:
                continue
            need = sum(c.limits.get(r, 0) for c in pod.containers for r in GPU_RESOURCES)
            for node in self.state.nodes.values():
                if MASTER_LABEL in node.meta.labels and need:
                    continue
                cap = sum(node.capacity.get(r, 0) for r in GPU_RESOURCES)
                used = sum(c.limits.get(r, 0) for p in self.state.pods.values()
                           if p.node_name == node.name and p.phase in (POD_PENDING, POD_RUNNING)
                           for c in p.containers for r in GPU_RESOURCES)
                if need == 0 or cap - used >= need:
                    self.state.set_pod_phase(pod.namespace, pod.name, POD_RUNNING, node.name)
                    bound.append(pod)
                    break
        return bound
