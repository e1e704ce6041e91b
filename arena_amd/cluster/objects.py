"""Minimal Kubernetes-shaped object model.

Only the fields the reference actually reads are modelled (SURVEY §2.4 "K8s API surface"):
labels/namespace/owner kinds/creation time on every object; pod phase, host IP, node name and
container resource limits; batch Job active/succeeded/failed + start time; node capacity,
addresses and role label; Service ports/NodePorts; Endpoints; TFJob conditions; StatefulSet
replicas. Objects are built from manifests (dicts) by :mod:`arena_amd.cluster.controller`, so the
Fake and Local backends see exactly what the K8s backend would apply.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

AMD_GPU = "amd.com/gpu"
NVIDIA_GPU = "nvidia.com/gpu"                         # read for mixed clusters (gpu.go:8-79)
DEPRECATED_NVIDIA_GPU = "alpha.kubernetes.io/nvidia-gpu"
GPU_RESOURCES = (AMD_GPU, NVIDIA_GPU, DEPRECATED_NVIDIA_GPU)
MASTER_LABEL = "node-role.kubernetes.io/master"

POD_PENDING, POD_RUNNING, POD_SUCCEEDED, POD_FAILED, POD_UNKNOWN = (
    "Pending", "Running", "Succeeded", "Failed", "Unknown")


@dataclass
class Meta:
    name: str
    namespace: str = "default"
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)
    creation_timestamp: float = field(default_factory=time.time)
    owner_kinds: List[str] = field(default_factory=list)
    uid: str = ""


@dataclass
class Container:
    name: str
    image: str = ""
    command: List[str] = field(default_factory=list)
    env: Dict[str, str] = field(default_factory=dict)
    limits: Dict[str, int] = field(default_factory=dict)
    requests: Dict[str, int] = field(default_factory=dict)
    working_dir: str = ""


@dataclass
class Pod:
    meta: Meta
    containers: List[Container] = field(default_factory=list)
    node_name: str = ""
    phase: str = POD_PENDING
    host_ip: str = ""
    pod_ip: str = ""
    start_time: Optional[float] = None
    exit_code: Optional[int] = None
    restart_count: int = 0
    host_network: bool = False

    @property
    def name(self) -> str:
        return self.meta.name

    @property
    def hostname(self) -> str:
        """What ``$HOSTNAME`` is inside the pod: the node's name under hostNetwork (the charts'
        default), else the pod's own name."""
        return (self.node_name or "") if self.host_network else self.meta.name

    @property
    def namespace(self) -> str:
        return self.meta.namespace


@dataclass
class Job:
    meta: Meta
    active: int = 0
    succeeded: int = 0
    failed: int = 0
    start_time: Optional[float] = None
    completion_time: Optional[float] = None
    backoff_limit: int = 0
    template: dict = field(default_factory=dict)

    @property
    def name(self) -> str:
        return self.meta.name


@dataclass
class StatefulSet:
    meta: Meta
    replicas: int = 0
    template: dict = field(default_factory=dict)

    @property
    def name(self) -> str:
        return self.meta.name


@dataclass
class ServicePort:
    port: int
    target_port: int = 0
    node_port: int = 0
    name: str = ""


@dataclass
class Service:
    meta: Meta
    type: str = "ClusterIP"
    ports: List[ServicePort] = field(default_factory=list)
    selector: Dict[str, str] = field(default_factory=dict)
    cluster_ip: str = ""

    @property
    def name(self) -> str:
        return self.meta.name


@dataclass
class Endpoints:
    meta: Meta
    addresses: List[str] = field(default_factory=list)
    ports: List[int] = field(default_factory=list)


@dataclass
class Condition:
    type: str
    status: str = "True"
    last_transition: float = field(default_factory=time.time)


@dataclass
class TFJob:
    """kubeflow.org/v1alpha2 TFJob (types.go:107-209): replica specs + conditions."""
    meta: Meta
    replicas: Dict[str, int] = field(default_factory=dict)  # PS/Worker/Chief/Evaluator
    conditions: List[Condition] = field(default_factory=list)
    start_time: Optional[float] = None
    clean_pod_policy: str = "Running"

    @property
    def name(self) -> str:
        return self.meta.name


@dataclass
class Node:
    meta: Meta
    capacity: Dict[str, int] = field(default_factory=dict)
    addresses: List[Tuple[str, str]] = field(default_factory=list)  # (type, address)
    ready: bool = True

    @property
    def name(self) -> str:
        return self.meta.name


def matches(labels: Dict[str, str], selector: Optional[Dict[str, str]]) -> bool:
    if not selector:
        return True
    return all(labels.get(k) == v for k, v in selector.items())


def parse_selector(sel: Optional[str]) -> Optional[Dict[str, str]]:
    """'release=x,app=y' -> dict (equality selectors, the only kind the reference uses)."""
    if not sel:
        return None
    out = {}
    for part in sel.split(","):
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip()
    return out
