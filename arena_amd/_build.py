"""Build the native C++ runtime tools (no GPU needed): supervisor, GPU/topology probe, PS server.

Outputs go to ``arena_amd/bin/`` (git-ignored, shipped to the GPU box with the tree).
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BIN = os.path.join(HERE, "bin")

TOOLS = {
    # name: (sources, extra flags)
    "arena-supervisor": (["csrc/runtime/supervisor.cpp"], ["-Icsrc/runtime"]),
    "arena-probe": (["csrc/runtime/probe.cpp"], ["-Icsrc/runtime"]),
    "arena-ps": (["csrc/runtime/ps_server.cpp"], ["-pthread", "-O3", "-march=x86-64-v3"]),
}


def tool_path(name: str) -> str:
    return os.path.join(BIN, name)


def build_native_tools(force: bool = False) -> list[str]:
    os.makedirs(BIN, exist_ok=True)
    cxx = shutil.which("g++") or shutil.which("c++")
    built = []
    for name, (srcs, flags) in TOOLS.items():
        out = tool_path(name)
        paths = [os.path.join(ROOT, s) for s in srcs]
        deps = paths + [os.path.join(ROOT, "csrc", "runtime", "json.h")]
        if not force and os.path.exists(out) and all(
                os.path.getmtime(out) >= os.path.getmtime(p) for p in deps):
            built.append(out)
            continue
        subprocess.run([cxx, "-O2", "-std=c++17", "-Wall", "-Wextra", "-o", out, *paths,
                        *[f.replace("-Icsrc", "-I" + os.path.join(ROOT, "csrc")) for f in flags]],
                       check=True)
        built.append(out)
    return built


def ensure_tool(name: str) -> str:
    """Path to a native tool, building it on first use (g++ only, seconds)."""
    path = tool_path(name)
    if not os.path.exists(path):
        build_native_tools()
    return path
