"""TensorBoard URL (reference: tensorboard.go:18-81): first Ready node's first address + the
NodePort of the Service labelled release=<name>, role=tensorboard."""
from __future__ import annotations

from typing import Optional


def tensorboard_url(backend, name: str, namespace: str) -> Optional[str]:
    node_ip = None
    for n in backend.list_nodes():
        if n.ready and n.addresses:
            node_ip = n.addresses[0][1]
            break
    if node_ip is None:
        return None
    for svc in backend.list_services(namespace, {"release": name, "role": "tensorboard"}):
        for p in svc.ports:
            if p.node_port:
                return f"http://{node_ip}:{p.node_port}"
    return None
