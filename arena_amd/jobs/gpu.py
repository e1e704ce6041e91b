"""GPU accounting (reference: cmd/arena/commands/gpu.go:8-79), AMD-first.

Node capacity and container limits are read from ``amd.com/gpu`` first, then the NVIDIA resource
names (mixed clusters). A pod's GPUs are the sum of its containers' LIMITS; an "active" pod is one
not in Succeeded/Failed.
"""
from __future__ import annotations

from typing import Iterable, List

from ..cluster.objects import GPU_RESOURCES, Node, Pod, POD_FAILED, POD_SUCCEEDED


def gpu_in_node(node: Node) -> int:
    for r in GPU_RESOURCES:
        if r in node.capacity:
            return int(node.capacity[r])
    return 0


def gpu_in_container(limits: dict) -> int:
    for r in GPU_RESOURCES:
        if r in limits:
            return int(limits[r])
    return 0


def gpu_in_pod(pod: Pod) -> int:
    return sum(gpu_in_container(c.limits) for c in pod.containers)


def gpu_in_active_pod(pod: Pod) -> int:
    if pod.phase in (POD_SUCCEEDED, POD_FAILED):
        return 0
    return gpu_in_pod(pod)


def gpu_pods(pods: Iterable[Pod]) -> List[Pod]:
    return [p for p in pods if gpu_in_pod(p) > 0]
