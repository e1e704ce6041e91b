"""Dashboard / log-viewer discovery (reference: dashboard_helper.go:12-47): the first address and
port of a Service's Endpoints in the arena namespace."""
from __future__ import annotations

from typing import Optional


def dashboard(backend, namespace: str, name: str) -> Optional[str]:
    ep = backend.get_endpoints(namespace, name)
    if ep is None or not ep.addresses or not ep.ports:
        return None
    return f"{ep.addresses[0]}:{ep.ports[0]}"
