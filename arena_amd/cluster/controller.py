"""A tiny in-process "controller": manifests -> cluster objects.

Plays the roles of the K8s Job / StatefulSet / Deployment controllers and of the external
tf-operator (TFJob -> `<tfjob>-{ps,worker}-<i>` pods labelled `group_name`,
`tf-replica-type`, `tf-replica-index`; conditions Created/Running/Restarting/Succeeded/Failed).
Used by the Fake and Local backends so both see exactly the objects the K8s backend would create.
"""
from __future__ import annotations

import hashlib
import itertools
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .objects import (Condition, Container, Endpoints, Job, Meta, Node, Pod, POD_FAILED,
                      POD_PENDING, POD_RUNNING, POD_SUCCEEDED, Service, ServicePort, StatefulSet,
                      TFJob, matches)


def _suffix(seed: str, n: int = 5) -> str:
    alphabet = "bcdfghjklmnpqrstvwxz2456789"
    h = int(hashlib.sha1(seed.encode()).hexdigest(), 16)
    out = []
    for _ in range(n):
        h, r = divmod(h, len(alphabet))
        out.append(alphabet[r])
    return "".join(out)


def _env_value(e: dict, pod_fields: dict) -> str:
    """A literal env value, or a downward-API ``fieldRef`` resolved for this pod (as the kubelet
    does at container start)."""
    ref = ((e.get("valueFrom") or {}).get("fieldRef") or {}).get("fieldPath")
    if ref:
        return str(pod_fields.get(ref, ""))
    return e.get("value", "")


def containers_from_template(tpl: dict, pod_fields: Optional[dict] = None) -> List[Container]:
    out = []
    for c in (tpl.get("spec") or {}).get("containers", []):
        res = c.get("resources") or {}
        env = {e["name"]: _env_value(e, pod_fields or {}) for e in c.get("env", [])}
        out.append(Container(name=c.get("name", ""), image=c.get("image", ""),
                             command=list(c.get("command", [])), env=env,
                             limits={k: v for k, v in (res.get("limits") or {}).items()
                                     if isinstance(v, int)},
                             requests={k: v for k, v in (res.get("requests") or {}).items()
                                       if isinstance(v, int)},
                             working_dir=c.get("workingDir", "")))
    return out


@dataclass
class ClusterState:
    nodes: Dict[str, Node] = field(default_factory=dict)
    pods: Dict[tuple, Pod] = field(default_factory=dict)          # (ns, name)
    jobs: Dict[tuple, Job] = field(default_factory=dict)
    statefulsets: Dict[tuple, StatefulSet] = field(default_factory=dict)
    services: Dict[tuple, Service] = field(default_factory=dict)
    endpoints: Dict[tuple, Endpoints] = field(default_factory=dict)
    tfjobs: Dict[tuple, TFJob] = field(default_factory=dict)
    deployments: Dict[tuple, dict] = field(default_factory=dict)
    configmaps: Dict[tuple, dict] = field(default_factory=dict)
    namespaces: set = field(default_factory=lambda: {"default", "kube-system", "arena-system"})
    node_ports: itertools.count = field(default_factory=lambda: itertools.count(30000))
    clock: callable = time.time

    # ---------------------------------------------------------------------------------------
    def _meta(self, m: dict, extra_labels=None, owner=None, name=None) -> Meta:
        labels = dict(m.get("labels") or {})
        labels.update(extra_labels or {})
        return Meta(name=name or m["name"], namespace=m.get("namespace", "default"),
                    labels=labels, creation_timestamp=self.clock(),
                    owner_kinds=[owner] if owner else [])

    def _new_pod(self, name: str, ns: str, tpl: dict, owner: str, extra_labels=None) -> Pod:
        tmeta = dict(tpl.get("metadata") or {})
        tmeta["namespace"] = ns
        fields = {"metadata.name": name, "metadata.namespace": ns}
        pod = Pod(meta=self._meta(tmeta, extra_labels, owner, name=name),
                  containers=containers_from_template(tpl, fields),
                  host_network=bool((tpl.get("spec") or {}).get("hostNetwork", False)))
        self.pods[(ns, name)] = pod
        return pod

    def apply(self, manifests: List[dict]) -> List[object]:
        created = []
        for m in manifests:
            kind = m["kind"]
            md = m["metadata"]
            ns = md.get("namespace", "default")
            self.namespaces.add(ns)
            spec = m.get("spec") or {}
            if kind == "Job":
                job = Job(meta=self._meta(md), backoff_limit=int(spec.get("backoffLimit", 0)),
                          template=spec.get("template") or {})
                self.jobs[(ns, job.name)] = job
                pod = self._new_pod(f"{job.name}-{_suffix(job.name + str(job.meta.creation_timestamp))}",
                                    ns, job.template, "Job")
                created += [job, pod]
            elif kind == "StatefulSet":
                ss = StatefulSet(meta=self._meta(md), replicas=int(spec.get("replicas", 0)),
                                 template={**(spec.get("template") or {}),
                                           "serviceName": spec.get("serviceName", "")})
                self.statefulsets[(ns, ss.name)] = ss
                created.append(ss)
                for i in range(ss.replicas):
                    created.append(self._new_pod(f"{ss.name}-{i}", ns, ss.template,
                                                 "StatefulSet"))
            elif kind == "TFJob":
                tf = TFJob(meta=self._meta(md), clean_pod_policy=spec.get("cleanPodPolicy", "Running"))
                tf.conditions.append(Condition("Created", "True", self.clock()))
                self.tfjobs[(ns, tf.name)] = tf
                created.append(tf)
                for rtype, rspec in (spec.get("tfReplicaSpecs") or {}).items():
                    n = int(rspec.get("replicas", 1))
                    tf.replicas[rtype] = n
                    for i in range(n):
                        created.append(self._new_pod(
                            f"{tf.name}-{rtype.lower()}-{i}", ns, rspec.get("template") or {},
                            "TFJob", {"group_name": "kubeflow.org",
                                      "tf-replica-type": rtype.lower(),
                                      "tf-replica-index": str(i),
                                      "tf_job_name": tf.name}))
            elif kind == "Deployment":
                self.deployments[(ns, md["name"])] = m
                tpl = spec.get("template") or {}
                created.append(self._new_pod(f"{md['name']}-{_suffix(md['name'], 9)}-{_suffix(md['name'] + 'p')}",
                                             ns, tpl, "ReplicaSet"))
            elif kind == "Service":
                svc = Service(meta=self._meta(md), type=spec.get("type", "ClusterIP"),
                              selector=dict(spec.get("selector") or {}),
                              cluster_ip=spec.get("clusterIP", ""))
                for p in spec.get("ports", []):
                    sp = ServicePort(port=int(p["port"]), target_port=int(p.get("targetPort", p["port"])),
                                     name=p.get("name", ""))
                    if svc.type == "NodePort":
                        sp.node_port = next(self.node_ports)
                    svc.ports.append(sp)
                self.services[(ns, svc.name)] = svc
                created.append(svc)
            elif kind == "ConfigMap":
                self.configmaps[(ns, md["name"])] = m
            else:
                raise ValueError(f"unsupported manifest kind {kind}")
        return created

    # --------------------------------------------------------------------------------- state
    def set_pod_phase(self, ns: str, name: str, phase: str, node: Optional[str] = None,
                      exit_code: Optional[int] = None) -> None:
        pod = self.pods[(ns, name)]
        if node is not None:
            pod.node_name = node
            n = self.nodes.get(node)
            if n is not None:
                pod.host_ip = next((a for t, a in n.addresses if t == "InternalIP"),
                                   n.addresses[0][1] if n.addresses else "")
        if phase == POD_RUNNING and pod.start_time is None:
            pod.start_time = self.clock()
        pod.phase = phase
        if exit_code is not None:
            pod.exit_code = exit_code
        self.reconcile()

    def reconcile(self) -> None:
        """Derive Job counters and TFJob conditions from pod phases (the controllers' job)."""
        for (ns, name), job in self.jobs.items():
            pods = [p for p in self.pods.values()
                    if p.namespace == ns and "Job" in p.meta.owner_kinds
                    and matches(p.meta.labels, job.template.get("metadata", {}).get("labels"))
                    and p.name.startswith(name + "-")]
            job.active = sum(p.phase in (POD_PENDING, POD_RUNNING) for p in pods)
            job.succeeded = sum(p.phase == POD_SUCCEEDED for p in pods)
            job.failed = sum(p.phase == POD_FAILED for p in pods)
            if job.start_time is None and pods:
                job.start_time = min(p.meta.creation_timestamp for p in pods)
            if job.completion_time is None and job.succeeded > 0:
                job.completion_time = self.clock()
        for (ns, name), tf in self.tfjobs.items():
            pods = [p for p in self.pods.values()
                    if p.namespace == ns and p.meta.labels.get("tf_job_name") == name]
            types = {c.type for c in tf.conditions}
            workers = [p for p in pods if p.meta.labels.get("tf-replica-type") == "worker"]
            if any(p.phase == POD_RUNNING for p in pods):
                if tf.start_time is None:
                    tf.start_time = self.clock()
                if "Running" not in types:
                    # tf-operator flips Created off once the job runs
                    for c in tf.conditions:
                        if c.type == "Created":
                            c.status = "False"
                    tf.conditions.append(Condition("Running", "True", self.clock()))
            if workers and all(p.phase == POD_SUCCEEDED for p in workers) and "Succeeded" not in types:
                for c in tf.conditions:
                    c.status = "False"
                tf.conditions.append(Condition("Succeeded", "True", self.clock()))
            if any(p.phase == POD_FAILED for p in pods) and "Failed" not in types:
                for c in tf.conditions:
                    c.status = "False"
                tf.conditions.append(Condition("Failed", "True", self.clock()))

    def delete_release_objects(self, release: str) -> int:
        n = 0
        for store in (self.pods, self.jobs, self.statefulsets, self.services, self.tfjobs,
                      self.deployments, self.configmaps):
            for key in [k for k, v in store.items()
                        if (v.meta.labels if hasattr(v, "meta") else v["metadata"].get("labels", {})
                            ).get("release") == release]:
                del store[key]
                n += 1
        return n
