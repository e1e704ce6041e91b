"""Per-node GPU view (reference: top_node.go:57-250, NodeDescriber): pods grouped by node,
total = node capacity, allocated = Σ GPU limits of the node's active pods."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

from ..cluster.objects import MASTER_LABEL, Node, Pod
from .gpu import gpu_in_node, gpu_in_pod


@dataclass
class NodeInfo:
    node: Node
    pods: List[Pod] = field(default_factory=list)

    def total_gpu(self) -> int:
        return gpu_in_node(self.node)

    def allocated_gpu(self) -> int:
        return sum(gpu_in_pod(p) for p in self.pods)

    def role(self) -> str:
        return "master" if MASTER_LABEL in self.node.meta.labels else "worker"

    def internal_ip(self) -> str:
        # Q16 fixed: summary and details both show the InternalIP (fallback: first address)
        for t, a in self.node.addresses:
            if t == "InternalIP":
                return a
        return self.node.addresses[0][1] if self.node.addresses else "unknown"


def describe_nodes(backend) -> List[NodeInfo]:
    active = backend.list_pods(active_only=True)
    out = []
    for n in backend.list_nodes():
        out.append(NodeInfo(n, [p for p in active if p.node_name == n.name]))
    return out
