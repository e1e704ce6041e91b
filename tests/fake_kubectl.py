#!/usr/bin/env python3
"""A tiny stand-in for ``kubectl`` backed by a JSON file (``$FAKE_KUBE_STATE``), for testing the
K8s backend without a cluster. Objects created by ``apply`` go through the same in-process
controller as the Fake/Local backends (Job/StatefulSet/TFJob/Deployment -> pods), are stored as
Kubernetes JSON, and are served back by ``get -o json``.

Supported: get (list/one, -n/-A/-l, -o json), apply -f -, delete, create namespace, logs.
The endpoints controller is modelled too: a selector Service's Endpoints are the IPs of its
Running pods (the node's IP under hostNetwork) and its target port.
Test hooks (not kubectl): fake-node NAME IP GPUS, fake-phase NS POD PHASE [NODE] [EXIT],
fake-log NS POD TEXT..., fake-endpoints NS NAME IP PORT, fake-exec NS POD -- runs the pod's
container command the way the kubelet would start it: its env (downward-API fields resolved) plus
HOSTNAME = the node's name under hostNetwork, else the pod's name.
"""
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import yaml  # noqa: E402

from arena_amd.cluster import k8s_json as kj  # noqa: E402
from arena_amd.cluster.controller import ClusterState  # noqa: E402
from arena_amd.cluster.objects import AMD_GPU, Meta, Node, matches  # noqa: E402
from arena_amd.utils.timefmt import parse_rfc3339, rfc3339  # noqa: E402

STATE = os.environ.get("FAKE_KUBE_STATE", "/tmp/fake_kube.json")
KINDS = {"pods": "pods", "pod": "pods", "jobs.batch": "jobs", "jobs": "jobs",
         "statefulsets.apps": "statefulsets", "statefulsets": "statefulsets",
         "services": "services", "service": "services", "svc": "services",
         "endpoints": "endpoints", "tfjobs.kubeflow.org": "tfjobs", "tfjobs": "tfjobs",
         "nodes": "nodes", "configmaps": "configmaps", "deployments.apps": "deployments",
         "namespace": "namespaces", "namespaces": "namespaces", "ns": "namespaces"}
STORES = ("pods", "jobs", "statefulsets", "services", "endpoints", "tfjobs", "nodes",
          "configmaps", "deployments", "namespaces")


def load():
    if os.path.exists(STATE):
        with open(STATE) as f:
            s = json.load(f)
    else:
        s = {}
    for k in STORES:
        s.setdefault(k, {})
    s.setdefault("logs", {})
    s["namespaces"].setdefault("default", {"metadata": {"name": "default"}})
    return s


def save(s):
    tmp = STATE + ".tmp"
    with open(tmp, "w") as f:
        json.dump(s, f)
    os.replace(tmp, STATE)


def key(ns, name):
    return f"{ns}/{name}"


def reconcile(s):
    """Round-trip through the controller to recompute Job counters / TFJob conditions."""
    st = ClusterState()
    for k, o in s["pods"].items():
        p = kj.pod_from(o)
        st.pods[(p.namespace, p.name)] = p
    for k, o in s["jobs"].items():
        j = kj.job_from(o)
        st.jobs[(j.meta.namespace, j.name)] = j
    for k, o in s["tfjobs"].items():
        t = kj.tfjob_from(o)
        st.tfjobs[(t.meta.namespace, t.name)] = t
    st.reconcile()
    for (ns, name), j in st.jobs.items():
        s["jobs"][key(ns, name)] = kj.job_to(j)
    for (ns, name), t in st.tfjobs.items():
        s["tfjobs"][key(ns, name)] = kj.tfjob_to(t)
    # endpoints controller (manual fake-endpoints entries are left alone)
    for k, svc in s["services"].items():
        sel = (svc.get("spec") or {}).get("selector")
        if not sel or s["endpoints"].get(k, {}).get("manual"):
            continue
        ns = k.split("/", 1)[0]
        ips = []
        for pk, p in sorted(s["pods"].items()):
            st_ = p.get("status") or {}
            if (pk.startswith(ns + "/") and st_.get("phase") == "Running"
                    and matches((p.get("metadata") or {}).get("labels") or {}, sel)):
                ip = st_.get("podIP") or st_.get("hostIP")
                if ip:
                    ips.append(ip)
        ports = [int(p.get("targetPort") or p["port"]) for p in svc["spec"].get("ports") or []]
        s["endpoints"][k] = {"apiVersion": "v1", "kind": "Endpoints",
                             "metadata": {"name": k.split("/", 1)[1], "namespace": ns},
                             "subsets": [{"addresses": [{"ip": i} for i in ips],
                                          "ports": [{"port": p} for p in ports]}] if ips else []}


def apply(s, docs):
    st = ClusterState()
    for n in s["nodes"].values():
        node = kj.node_from(n)
        st.nodes[node.name] = node
    for d in docs:
        if not d:
            continue
        if d["kind"] in ("ServiceAccount", "ClusterRole", "ClusterRoleBinding", "Role",
                         "RoleBinding", "CustomResourceDefinition"):
            continue   # RBAC / API objects: accepted, nothing to reconcile
        if d["kind"] == "Namespace":
            s["namespaces"].setdefault(d["metadata"]["name"], {"metadata": d["metadata"]})
            continue
        ns = d["metadata"].setdefault("namespace", "default")
        s["namespaces"].setdefault(ns, {"metadata": {"name": ns}})
        if d["kind"] == "ConfigMap":
            s["configmaps"][key(ns, d["metadata"]["name"])] = d
            continue
        if d["kind"] == "Deployment":
            s["deployments"][key(ns, d["metadata"]["name"])] = d
        created = st.apply([d])
        for o in created:
            kind = type(o).__name__
            if kind == "Pod":
                s["pods"][key(o.namespace, o.name)] = kj.pod_to(o)
            elif kind == "Job":
                s["jobs"][key(o.meta.namespace, o.name)] = kj.job_to(o)
            elif kind == "StatefulSet":
                s["statefulsets"][key(o.meta.namespace, o.name)] = kj.statefulset_to(o)
            elif kind == "Service":
                s["services"][key(o.meta.namespace, o.name)] = kj.service_to(o)
            elif kind == "TFJob":
                s["tfjobs"][key(o.meta.namespace, o.name)] = kj.tfjob_to(o)
    reconcile(s)


def parse_flags(argv):
    flags, pos = {}, []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a in ("-n", "--namespace", "-l", "-o", "-f", "--kubeconfig"):
            flags[a] = argv[i + 1]
            i += 2
            continue
        if a.startswith("--") and "=" in a:
            k, v = a.split("=", 1)
            flags[k] = v
        elif a.startswith("-"):
            flags[a] = True
        else:
            pos.append(a)
        i += 1
    return flags, pos


def sel_of(flags):
    raw = flags.get("-l")
    if not raw:
        return None
    return dict(p.split("=", 1) for p in raw.split(","))


def main(argv):
    flags, pos = parse_flags(argv)
    s = load()
    if not pos:
        print("fake kubectl: no command", file=sys.stderr)
        return 1
    cmd = pos[0]
    ns = flags.get("-n", flags.get("--namespace", "default"))
    if cmd == "get":
        store = KINDS[pos[1]]
        if store == "tfjobs" and os.environ.get("FAKE_KUBE_NO_TFJOB_CRD"):
            print(f'error: the server doesn\'t have a resource type "{pos[1]}"', file=sys.stderr)
            return 1
        if len(pos) > 2:
            name = pos[2]
            o = s[store].get(name if store in ("nodes", "namespaces") else key(ns, name))
            if o is None:
                print(f'Error from server (NotFound): {pos[1]} "{name}" not found', file=sys.stderr)
                return 1
            print(json.dumps(o) if flags.get("-o") == "json" else name)
            return 0
        items = [o for k, o in sorted(s[store].items())
                 if (flags.get("-A") or store in ("nodes", "namespaces") or k.startswith(ns + "/"))
                 and matches((o.get("metadata") or {}).get("labels") or {}, sel_of(flags))]
        print(json.dumps({"items": items}))
        return 0
    if cmd == "apply":
        docs = list(yaml.safe_load_all(sys.stdin.read()))
        apply(s, docs)
        save(s)
        for d in docs:
            print(f"{d['kind'].lower()}/{d['metadata']['name']} created")
        return 0
    if cmd == "delete":
        store = KINDS[pos[1]]
        k = key(ns, pos[2])
        if k not in s[store]:
            if flags.get("--ignore-not-found"):
                return 0
            print(f'Error from server (NotFound): {pos[1]} "{pos[2]}" not found', file=sys.stderr)
            return 1
        obj = s[store].pop(k)
        # owned pods go with their controller (garbage collection)
        if store in ("jobs", "statefulsets", "tfjobs", "deployments"):
            rel = obj["metadata"].get("labels", {}).get("release")
            name = obj["metadata"]["name"]
            for pk in [pk for pk, p in s["pods"].items() if pk.startswith(ns + "/") and (
                    p["metadata"]["name"].startswith(name + "-")
                    and p["metadata"].get("labels", {}).get("release") == rel)]:
                del s["pods"][pk]
        save(s)
        print(f"{pos[1]} \"{pos[2]}\" deleted")
        return 0
    if cmd == "create" and pos[1] in ("namespace", "ns"):
        if pos[2] in s["namespaces"]:
            print(f'Error from server (AlreadyExists): namespaces "{pos[2]}" already exists',
                  file=sys.stderr)
            return 1
        s["namespaces"][pos[2]] = {"metadata": {"name": pos[2]}}
        save(s)
        return 0
    if cmd == "logs":
        lines = s["logs"].get(key(ns, pos[1]))
        if lines is None and key(ns, pos[1]) not in s["pods"]:
            print(f'Error from server (NotFound): pods "{pos[1]}" not found', file=sys.stderr)
            return 1
        lines = lines or []
        if "--since-time" in flags:
            cut = parse_rfc3339(flags["--since-time"])
            lines = [x for x in lines if x[0] >= cut]
        if "--since" in flags:
            cut = time.time() - float(flags["--since"].rstrip("s"))
            lines = [x for x in lines if x[0] >= cut]
        if "--tail" in flags:
            t = int(flags["--tail"])
            lines = lines[-t:] if t else []
        for ts, text in lines:
            print(f"{rfc3339(ts)} {text}" if flags.get("--timestamps") else text)
        return 0
    # ---- test hooks
    if cmd == "fake-node":
        name, ip, gpus = pos[1], pos[2], int(pos[3])
        n = Node(meta=Meta(name=name, namespace="", labels={"kubernetes.io/hostname": name}),
                 capacity={AMD_GPU: gpus} if gpus else {},
                 addresses=[("InternalIP", ip), ("Hostname", name)])
        s["nodes"][name] = kj.node_to(n)
        save(s)
        return 0
    if cmd == "fake-phase":
        pns, pod, phase = pos[1], pos[2], pos[3]
        o = s["pods"][key(pns, pod)]
        o["status"]["phase"] = phase
        if len(pos) > 4:
            node = pos[4]
            o["spec"]["nodeName"] = node
            n = s["nodes"].get(node)
            if n:
                o["status"]["hostIP"] = next(a["address"] for a in n["status"]["addresses"]
                                             if a["type"] == "InternalIP")
        if len(pos) > 5:
            o["status"]["containerStatuses"][0]["state"] = {"terminated": {"exitCode": int(pos[5])}}
        if phase == "Running" and "startTime" not in o["status"]:
            o["status"]["startTime"] = rfc3339(time.time())
        reconcile(s)
        save(s)
        return 0
    if cmd == "fake-log":
        s["logs"].setdefault(key(pos[1], pos[2]), []).append([time.time(), " ".join(pos[3:])])
        save(s)
        return 0
    if cmd == "fake-endpoints":
        e = {"apiVersion": "v1", "kind": "Endpoints", "manual": True,
             "metadata": {"name": pos[2], "namespace": pos[1]},
             "subsets": [{"addresses": [{"ip": pos[3]}], "ports": [{"port": int(pos[4])}]}]}
        s["endpoints"][key(pos[1], pos[2])] = e
        save(s)
        return 0
    if cmd == "fake-exec":
        o = s["pods"][key(pos[1], pos[2])]
        pod = kj.pod_from(o)
        c = pod.containers[0]
        # the image ships arena_amd (the in-pod rank launcher of several-ranks-per-pod jobs)
        env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"),
               "PYTHONPATH": os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
               **c.env, "HOSTNAME": pod.hostname}
        r = subprocess.run(c.command, env=env, capture_output=True, text=True)
        sys.stdout.write(r.stdout)
        sys.stderr.write(r.stderr)
        return r.returncode
    print(f"fake kubectl: unsupported command {argv}", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
