#!/usr/bin/env python3
"""Count the node types of a captured ResNet training step (hipGraphGetNodes via ctypes) and
list memcpy nodes whose source is host memory: a captured host->device copy reads its source at
REPLAY time, so a library that stages kernel arguments in a host buffer it later frees makes the
graph replay read whatever the host heap holds then.

    python tools/graph_nodes.py --mode auto
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
         6: "wait_event", 7: "event_record", 8: "ext_sem_signal", 9: "ext_sem_wait",
         10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class hipPitchedPtr(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("pitch", ctypes.c_size_t), ("xsize", ctypes.c_size_t),
                ("ysize", ctypes.c_size_t)]


class hipPos(ctypes.Structure):
    _fields_ = [("x", ctypes.c_size_t), ("y", ctypes.c_size_t), ("z", ctypes.c_size_t)]


class hipExtent(ctypes.Structure):
    _fields_ = [("width", ctypes.c_size_t), ("height", ctypes.c_size_t), ("depth", ctypes.c_size_t)]


class hipMemcpy3DParms(ctypes.Structure):
    _fields_ = [("srcArray", ctypes.c_void_p), ("srcPos", hipPos), ("srcPtr", hipPitchedPtr),
                ("dstArray", ctypes.c_void_p), ("dstPos", hipPos), ("dstPtr", hipPitchedPtr),
                ("extent", hipExtent), ("kind", ctypes.c_int)]


class hipPointerAttribute(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int),
                ("allocationFlags", ctypes.c_uint)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from arena_amd.examples import cnn_bench
    from arena_amd.ops import conv
    from arena_amd.parallel import hvd
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    hvd.init("gloo")
    conv.set_mode(a.mode)
    args = cnn_bench.parse(["--model", "resnet50", "--batch_size", str(a.batch)])
    model, opt, x, y = cnn_bench.build(args, dev, 1)
    for _ in range(3):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16)
    torch.cuda.synchronize()
    opt.zero_grad(set_to_none=True)
    g = torch.cuda.CUDAGraph(keep_graph=True)   # keeps the hipGraph_t after instantiation
    with torch.cuda.graph(g):
        cnn_bench.train_step(model, opt, x, y, torch.bfloat16, zero_grad=False)
    graph = ctypes.c_void_p(g.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
    kinds = collections.Counter()
    host_copies = []
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        kinds[TYPES.get(t.value, t.value)] += 1
        if t.value == 1:
            p = hipMemcpy3DParms()
            if hip.hipGraphMemcpyNodeGetParams(ctypes.c_void_p(nd), ctypes.byref(p)) == 0:
                src = p.srcPtr.ptr
                attr = hipPointerAttribute()
                r = hip.hipPointerGetAttributes(ctypes.byref(attr), ctypes.c_void_p(src))
                # memoryType 1 = host, 2 = device; an error means unregistered (pageable) host
                host_copies.append((p.kind, r, attr.type, p.extent.width, hex(src or 0)))
    print(f"mode {a.mode}: {n.value} nodes {dict(kinds)}", flush=True)
    for hc in host_copies[:20]:
        print(f"  memcpy kind {hc[0]} ptr-attr rc {hc[1]} memtype {hc[2]} bytes {hc[3]} src {hc[4]}")
    print(f"  {len(host_copies)} memcpy nodes", flush=True)
    hvd.shutdown()


if __name__ == "__main__":
    main()
