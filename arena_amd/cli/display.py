"""Table renderers with the reference's exact column layouts:
list.go:86-133, get.go:101-134, top_node.go:107-229 (tabwriter padding 2, pad ' ')."""
from __future__ import annotations

import time
from typing import List, Optional

from ..jobs.gpu import gpu_in_pod, gpu_pods
from ..jobs.nodes import NodeInfo
from ..jobs.trainer import TrainingJob
from ..utils.tabwriter import TabWriter

SEP = "-" * 89


def training_job_list(out, jobs: List[TrainingJob], display_gpu: bool, now=None) -> None:
    w = TabWriter(out)
    total_alloc = total_req = 0
    if display_gpu:
        w.write("NAME\tSTATUS\tTRAINER\tAGE\tNODE\tGPU(Requests)\tGPU(Allocated)\n")
    else:
        w.write("NAME\tSTATUS\tTRAINER\tAGE\tNODE\n")
    for j in jobs:
        status = j.get_status()
        host = j.host_ip_of_chief()
        if display_gpu:
            req, alloc = j.requested_gpu(), j.allocated_gpu()
            total_req += req
            total_alloc += alloc
            w.write(f"{j.name()}\t{status}\t{j.trainer().upper()}\t{j.age(now)}\t{host}\t{req}\t{alloc}\n")
        else:
            w.write(f"{j.name()}\t{status}\t{j.trainer().upper()}\t{j.age(now)}\t{host}\n")
    if display_gpu:
        w.write("\n\nTotal Allocated GPUs of Training Job:\n")
        w.write(f"{total_alloc} \t\n\n")
        w.write("Total Requested GPUs of Training Job:\n")
        w.write(f"{total_req} \t\n")
    w.flush()


def single_job(out, job: TrainingJob, tensorboard_url: Optional[str], now=None) -> None:
    w = TabWriter(out)
    w.write("NAME\tSTATUS\tTRAINER\tAGE\tINSTANCE\tNODE\n")
    for p in job.all_pods():
        host = p.host_ip if p.phase == "Running" and p.host_ip else "N/A"
        w.write(f"{job.name()}\t{p.phase.upper()}\t{job.trainer()}\t{job.age(now)}\t{p.name}\t{host}\n")
    if tensorboard_url:
        w.write("\nYour tensorboard will be available on:\n")
        w.write(f"{tensorboard_url} \t\n")
    w.flush()


def top_node_summary(out, infos: List[NodeInfo], telemetry=None) -> None:
    w = TabWriter(out)
    total = alloc = 0
    extra = telemetry is not None and any(telemetry.get(i.node.name) for i in infos)
    if extra:
        w.write("NAME\tIPADDRESS\tROLE\tGPU(Total)\tGPU(Allocated)\tGPU(Busy%)\tVRAM(Used/Total GiB)"
                "\tPower(W)\n")
    else:
        w.write("NAME\tIPADDRESS\tROLE\tGPU(Total)\tGPU(Allocated)\n")
    for i in infos:
        t, a = i.total_gpu(), i.allocated_gpu()
        total += t
        alloc += a
        row = f"{i.node.name}\t{i.internal_ip()}\t{i.role()}\t{t}\t{a}"
        if extra:
            tel = telemetry.get(i.node.name) or {}
            row += f"\t{tel.get('busy', 'N/A')}\t{tel.get('vram', 'N/A')}\t{tel.get('power', 'N/A')}"
        w.write(row + "\n")
    w.write(SEP + "\n")
    w.write("Allocated/Total GPUs In Cluster:\n")
    pct = int(alloc / total * 100) if total > 0 else 0
    w.write(f"{alloc}/{total} ({pct}%)\t\n")
    w.flush()


def top_node_details(out, infos: List[NodeInfo]) -> None:
    w = TabWriter(out)
    total = alloc = 0
    w.write("\n")
    for i in infos:
        t, a = i.total_gpu(), i.allocated_gpu()
        total += t
        alloc += a
        w.write("\n")
        w.write(f"NAME:\t{i.node.name}\n")
        w.write(f"IPADDRESS:\t{i.internal_ip()}\n")
        w.write(f"ROLE:\t{i.role()}\n")
        pods = gpu_pods(i.pods)
        if pods:
            w.write("\nNAMESPACE\tNAME\tGPU REQUESTS\tGPU LIMITS\n")
            for p in pods:
                g = gpu_in_pod(p)
                w.write(f"{p.namespace}\t{p.name}\t{g}\t{g}\n")
            w.write("\n")
        pct = 0
        if t > 0:
            pct = int(a / t * 100)
        else:
            w.write("\n")
        w.write(f"Total GPUs In Node {i.node.name}:\t{t} \t\n")
        w.write(f"Allocated GPUs In Node {i.node.name}:\t{a} ({pct}%)\t\n")
        w.write(SEP + "\n")
    w.write("\n\n")
    w.write("Allocated/Total GPUs In Cluster:\t")
    pct = int(alloc / total * 100) if total > 0 else 0
    w.write(f"{alloc}/{total} ({pct}%)\t\n")
    w.flush()


def release_summary(out, rel, now=None) -> None:
    """helm-install-style confirmation (util/helm/helm.go:66-70 prints helm's output)."""
    now = now or time.time()
    out.write(f"NAME:   {rel.name}\nNAMESPACE: {rel.namespace}\nSTATUS: DEPLOYED\n\nRESOURCES:\n")
    by_kind = {}
    for m in rel.manifests:
        by_kind.setdefault(f"{m['apiVersion']}/{m['kind']}", []).append(m["metadata"]["name"])
    for kind in sorted(by_kind):
        w = TabWriter(out)
        out.write(f"==> {kind}\n")
        w.write("NAME\tAGE\n")
        for n in by_kind[kind]:
            w.write(f"{n}\t0s\n")
        w.flush()
        out.write("\n")
