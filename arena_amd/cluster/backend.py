"""Backend interface: what the CLI needs from "a cluster".

Replaces the reference's two integration adapters: the helm CLI wrapper
(install/check/delete/list releases, util/helm/helm.go:21-195) and the client-go read API
(pods/jobs/nodes/services/endpoints/TFJobs, logs). Implementations:
  * :class:`arena_amd.cluster.fake.FakeBackend`   -- in-memory cluster for tests;
  * :class:`arena_amd.cluster.local.LocalBackend` -- this machine: real processes on real GPUs;
  * :class:`arena_amd.cluster.k8s.K8sBackend`     -- renders manifests, applies with kubectl.
"""
from __future__ import annotations

import abc
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional

from .objects import Endpoints, Job, Node, Pod, Service, StatefulSet, TFJob


@dataclass
class Release:
    name: str
    namespace: str
    chart: str
    values: dict
    manifests: List[dict] = field(default_factory=list)
    created: float = 0.0


class BackendError(RuntimeError):
    pass


class Backend(abc.ABC):
    name = "abstract"

    # ---- release store (helm equivalent) --------------------------------------------------
    @abc.abstractmethod
    def install_release(self, name: str, namespace: str, chart: str, values: dict) -> Release:
        """Render and create every object of a job. Raises if the release exists."""

    @abc.abstractmethod
    def release_exists(self, name: str) -> bool: ...

    @abc.abstractmethod
    def get_release(self, name: str) -> Optional[Release]: ...

    @abc.abstractmethod
    def delete_release(self, name: str) -> None: ...

    @abc.abstractmethod
    def list_releases(self) -> Dict[str, str]:
        """release name -> namespace (helm.ListReleaseMap, helm.go:164-195)."""

    # ---- cluster reads (client-go equivalent) ---------------------------------------------
    @abc.abstractmethod
    def list_pods(self, namespace: Optional[str] = None, selector: Optional[dict] = None,
                  active_only: bool = False) -> List[Pod]: ...

    @abc.abstractmethod
    def list_jobs(self, namespace: Optional[str] = None,
                  selector: Optional[dict] = None) -> List[Job]: ...

    @abc.abstractmethod
    def list_tfjobs(self, namespace: Optional[str] = None,
                    selector: Optional[dict] = None) -> List[TFJob]: ...

    @abc.abstractmethod
    def list_nodes(self) -> List[Node]: ...

    @abc.abstractmethod
    def list_services(self, namespace: str, selector: Optional[dict] = None) -> List[Service]: ...

    @abc.abstractmethod
    def get_endpoints(self, namespace: str, name: str) -> Optional[Endpoints]: ...

    @abc.abstractmethod
    def get_pod(self, namespace: str, name: str) -> Optional[Pod]: ...

    @abc.abstractmethod
    def get_job(self, namespace: str, name: str) -> Optional[Job]: ...

    @abc.abstractmethod
    def get_statefulset(self, namespace: str, name: str) -> Optional[StatefulSet]: ...

    @abc.abstractmethod
    def delete_statefulset(self, namespace: str, name: str) -> None: ...

    @abc.abstractmethod
    def delete_service(self, namespace: str, name: str) -> None: ...

    @abc.abstractmethod
    def delete_job(self, namespace: str, name: str) -> None:
        """Delete a batch Job and its pods (jobmon's cleanPodPolicy for PS/worker jobs)."""

    @abc.abstractmethod
    def ensure_namespace(self, namespace: str) -> None: ...

    @abc.abstractmethod
    def pod_logs(self, namespace: str, pod: str, follow: bool = False,
                 since_seconds: Optional[float] = None, since_time: Optional[float] = None,
                 tail: int = -1, timestamps: bool = False) -> Iterator[str]:
        """Yield log lines (with a trailing newline). ``timestamps`` prefixes RFC3339 times."""

    # ---- optional telemetry (top node) -----------------------------------------------------
    def node_telemetry(self, node: str) -> Optional[dict]:
        """Live GPU utilisation/VRAM/power for a node, if the backend can measure it."""
        return None
