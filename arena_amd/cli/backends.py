"""Backend selection: --backend / $ARENA_BACKEND (local | k8s); default local."""
from __future__ import annotations

import os


def arena_home(args=None) -> str:
    return (getattr(args, "home", None) or os.environ.get("ARENA_HOME")
            or os.path.join(os.path.expanduser("~"), ".arena"))


def make_backend(args):
    kind = getattr(args, "backend", None) or os.environ.get("ARENA_BACKEND", "local")
    if kind == "local":
        from ..cluster.local import LocalBackend
        return LocalBackend(arena_home(args))
    if kind == "k8s":
        from ..cluster.k8s import K8sBackend
        return K8sBackend(kubeconfig=getattr(args, "config", "") or os.environ.get("KUBECONFIG", ""),
                          home=arena_home(args))
    raise SystemExit(f"unknown backend {kind!r} (local | k8s)")
