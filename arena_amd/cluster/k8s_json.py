"""Kubernetes JSON <-> object model codec (the fields the reference reads; SURVEY §2.4 API list).

``from_k8s`` parses ``kubectl get ... -o json`` items into :mod:`objects` dataclasses for the
K8s backend; ``to_k8s`` serialises them back (used by the fake kubectl in tests, and handy for
golden files). Times are RFC3339 strings on the wire and epoch floats in the model.
"""
from __future__ import annotations

from typing import Optional

from ..utils.timefmt import parse_rfc3339, rfc3339
from .objects import (Condition, Container, Endpoints, Job, Meta, Node, Pod, Service, ServicePort,
                      StatefulSet, TFJob)


def _t(s: Optional[str]) -> Optional[float]:
    if not s:
        return None
    try:
        return parse_rfc3339(s)
    except ValueError:
        return None


def _ts(t: Optional[float]) -> Optional[str]:
    return rfc3339(t) if t is not None else None


def _qty(v) -> int:
    """Resource quantity -> int (GPU counts are plain integers; CPU/memory are not modelled)."""
    if isinstance(v, int):
        return v
    try:
        return int(str(v))
    except ValueError:
        return 0


def meta_from(m: dict) -> Meta:
    return Meta(name=m.get("name", ""), namespace=m.get("namespace", ""),
                labels=dict(m.get("labels") or {}), annotations=dict(m.get("annotations") or {}),
                creation_timestamp=_t(m.get("creationTimestamp")) or 0.0,
                owner_kinds=[o.get("kind", "") for o in m.get("ownerReferences") or []],
                uid=m.get("uid", ""))


def meta_to(m: Meta, with_ns: bool = True) -> dict:
    out = {"name": m.name, "labels": dict(m.labels),
           "creationTimestamp": _ts(m.creation_timestamp)}
    if with_ns:
        out["namespace"] = m.namespace
    if m.annotations:
        out["annotations"] = dict(m.annotations)
    if m.owner_kinds:
        out["ownerReferences"] = [{"kind": k, "name": "", "apiVersion": "v1"} for k in m.owner_kinds]
    if m.uid:
        out["uid"] = m.uid
    return out


def container_from(c: dict) -> Container:
    res = c.get("resources") or {}
    return Container(name=c.get("name", ""), image=c.get("image", ""),
                     command=list(c.get("command") or []),
                     env={e["name"]: e.get("value", "") for e in c.get("env") or []},
                     limits={k: _qty(v) for k, v in (res.get("limits") or {}).items()},
                     requests={k: _qty(v) for k, v in (res.get("requests") or {}).items()},
                     working_dir=c.get("workingDir", ""))


def container_to(c: Container) -> dict:
    return {"name": c.name, "image": c.image, "command": list(c.command),
            "env": [{"name": k, "value": v} for k, v in c.env.items()],
            "resources": {"limits": dict(c.limits), "requests": dict(c.requests)},
            "workingDir": c.working_dir}


def pod_from(o: dict) -> Pod:
    st = o.get("status") or {}
    spec = o.get("spec") or {}
    cs = (st.get("containerStatuses") or [{}])[0]
    term = ((cs.get("state") or {}).get("terminated") or {})
    return Pod(meta=meta_from(o.get("metadata") or {}),
               containers=[container_from(c) for c in spec.get("containers") or []],
               node_name=spec.get("nodeName", ""), phase=st.get("phase", "Pending"),
               host_ip=st.get("hostIP", ""), pod_ip=st.get("podIP", ""),
               start_time=_t(st.get("startTime")),
               exit_code=term.get("exitCode"), restart_count=int(cs.get("restartCount", 0) or 0),
               host_network=bool(spec.get("hostNetwork", False)))


def pod_to(p: Pod) -> dict:
    st = {"phase": p.phase}
    if p.host_ip:
        st["hostIP"] = p.host_ip
    if p.pod_ip:
        st["podIP"] = p.pod_ip
    if p.start_time is not None:
        st["startTime"] = _ts(p.start_time)
    cs = {"name": p.containers[0].name if p.containers else "", "restartCount": p.restart_count,
          "state": {}}
    if p.exit_code is not None:
        cs["state"] = {"terminated": {"exitCode": p.exit_code}}
    st["containerStatuses"] = [cs]
    spec = {"containers": [container_to(c) for c in p.containers]}
    if p.host_network:
        spec["hostNetwork"] = True
    if p.node_name:
        spec["nodeName"] = p.node_name
    return {"apiVersion": "v1", "kind": "Pod", "metadata": meta_to(p.meta), "spec": spec,
            "status": st}


def job_from(o: dict) -> Job:
    st = o.get("status") or {}
    spec = o.get("spec") or {}
    return Job(meta=meta_from(o.get("metadata") or {}), active=int(st.get("active", 0) or 0),
               succeeded=int(st.get("succeeded", 0) or 0), failed=int(st.get("failed", 0) or 0),
               start_time=_t(st.get("startTime")), completion_time=_t(st.get("completionTime")),
               backoff_limit=int(spec.get("backoffLimit", 0) or 0),
               template=spec.get("template") or {})


def job_to(j: Job) -> dict:
    st = {"active": j.active, "succeeded": j.succeeded, "failed": j.failed}
    if j.start_time is not None:
        st["startTime"] = _ts(j.start_time)
    if j.completion_time is not None:
        st["completionTime"] = _ts(j.completion_time)
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": meta_to(j.meta),
            "spec": {"backoffLimit": j.backoff_limit, "template": j.template}, "status": st}


def statefulset_from(o: dict) -> StatefulSet:
    spec = o.get("spec") or {}
    return StatefulSet(meta=meta_from(o.get("metadata") or {}),
                       replicas=int(spec.get("replicas", 0) or 0),
                       template={**(spec.get("template") or {}),
                                 "serviceName": spec.get("serviceName", "")})


def statefulset_to(s: StatefulSet) -> dict:
    tpl = dict(s.template)
    svc = tpl.pop("serviceName", "")
    return {"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": meta_to(s.meta),
            "spec": {"replicas": s.replicas, "serviceName": svc, "template": tpl}}


def service_from(o: dict) -> Service:
    spec = o.get("spec") or {}
    return Service(meta=meta_from(o.get("metadata") or {}), type=spec.get("type", "ClusterIP"),
                   ports=[ServicePort(port=int(p.get("port", 0)),
                                      target_port=_qty(p.get("targetPort", p.get("port", 0))),
                                      node_port=int(p.get("nodePort", 0) or 0),
                                      name=p.get("name", ""))
                          for p in spec.get("ports") or []],
                   selector=dict(spec.get("selector") or {}), cluster_ip=spec.get("clusterIP", ""))


def service_to(s: Service) -> dict:
    ports = []
    for p in s.ports:
        d = {"port": p.port, "targetPort": p.target_port or p.port, "name": p.name}
        if p.node_port:
            d["nodePort"] = p.node_port
        ports.append(d)
    return {"apiVersion": "v1", "kind": "Service", "metadata": meta_to(s.meta),
            "spec": {"type": s.type, "ports": ports, "selector": dict(s.selector),
                     "clusterIP": s.cluster_ip}}


def endpoints_from(o: dict) -> Endpoints:
    subsets = o.get("subsets") or []
    addrs, ports = [], []
    if subsets:
        addrs = [a.get("ip", "") for a in subsets[0].get("addresses") or []]
        ports = [int(p.get("port", 0)) for p in subsets[0].get("ports") or []]
    return Endpoints(meta=meta_from(o.get("metadata") or {}), addresses=addrs, ports=ports)


def endpoints_to(e: Endpoints) -> dict:
    return {"apiVersion": "v1", "kind": "Endpoints", "metadata": meta_to(e.meta),
            "subsets": [{"addresses": [{"ip": a} for a in e.addresses],
                         "ports": [{"port": p} for p in e.ports]}]}


def tfjob_from(o: dict) -> TFJob:
    st = o.get("status") or {}
    spec = o.get("spec") or {}
    conds = [Condition(type=c.get("type", ""), status=c.get("status", "True"),
                       last_transition=_t(c.get("lastTransitionTime")) or 0.0)
             for c in st.get("conditions") or []]
    reps = {k: int((v or {}).get("replicas", 1) or 0)
            for k, v in (spec.get("tfReplicaSpecs") or {}).items()}
    return TFJob(meta=meta_from(o.get("metadata") or {}), replicas=reps, conditions=conds,
                 start_time=_t(st.get("startTime")),
                 clean_pod_policy=spec.get("cleanPodPolicy", "Running"))


def tfjob_to(t: TFJob) -> dict:
    st = {"conditions": [{"type": c.type, "status": c.status,
                          "lastTransitionTime": _ts(c.last_transition)} for c in t.conditions]}
    if t.start_time is not None:
        st["startTime"] = _ts(t.start_time)
    return {"apiVersion": "kubeflow.org/v1alpha2", "kind": "TFJob", "metadata": meta_to(t.meta),
            "spec": {"cleanPodPolicy": t.clean_pod_policy,
                     "tfReplicaSpecs": {k: {"replicas": v} for k, v in t.replicas.items()}},
            "status": st}


def node_from(o: dict) -> Node:
    st = o.get("status") or {}
    ready = any(c.get("type") == "Ready" and c.get("status") == "True"
                for c in st.get("conditions") or [])
    return Node(meta=meta_from(o.get("metadata") or {}),
                capacity={k: _qty(v) for k, v in (st.get("capacity") or {}).items()},
                addresses=[(a.get("type", ""), a.get("address", "")) for a in st.get("addresses") or []],
                ready=ready)


def node_to(n: Node) -> dict:
    return {"apiVersion": "v1", "kind": "Node", "metadata": meta_to(n.meta, with_ns=False),
            "status": {"capacity": dict(n.capacity),
                       "addresses": [{"type": t, "address": a} for t, a in n.addresses],
                       "conditions": [{"type": "Ready", "status": "True" if n.ready else "False"}]}}


PARSERS = {"pods": pod_from, "jobs": job_from, "statefulsets": statefulset_from,
           "services": service_from, "endpoints": endpoints_from, "tfjobs": tfjob_from,
           "nodes": node_from}
