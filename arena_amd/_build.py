"""Build the native C++ runtime tools (no GPU needed): supervisor, GPU/topology probe, PS server.

Outputs go to ``arena_amd/bin/`` (git-ignored, shipped to the GPU box with the tree).

Sanitized variants (SURVEY §5 "race detection / sanitizers": the reference has none -- no
``-race`` target, Makefile:55-62) are built on demand into ``arena_amd/bin/<variant>/``:

* ``asan``  -- AddressSanitizer + UndefinedBehaviorSanitizer (leaks, overflows, UB), host code;
* ``tsan``  -- ThreadSanitizer, for the multi-threaded PS server and the supervisor's pipes.

``ARENA_NATIVE_SANITIZE=asan|tsan`` makes :func:`ensure_tool` hand out the sanitized binary,
so every test / job that launches a native tool runs under the sanitizer unchanged
(``make test-asan`` / ``make test-tsan``). These are host-only builds: GPU code is never
sanitized here (no xnack+/GPU ASan on this pool).
"""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BIN = os.path.join(HERE, "bin")

TOOLS = {
    # name: (sources, extra flags)
    "arena-supervisor": (["csrc/runtime/supervisor.cpp"], ["-Icsrc/runtime"]),
    "arena-probe": (["csrc/runtime/probe.cpp"], ["-Icsrc/runtime"]),
    "arena-ps": (["csrc/runtime/ps_server.cpp"], ["-pthread", "-O3", "-march=x86-64-v3"]),
}

SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
             "-fno-omit-frame-pointer", "-g", "-O1"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer", "-g", "-O1"],
}
# Runtime options: fail the process (exit 66) on the first report so tests see it.
SANITIZER_ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=66",
             "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1:exitcode=66"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:exitcode=66:second_deadlock_stack=1"},
}


def _variant(sanitize: Optional[str]) -> Optional[str]:
    v = sanitize if sanitize is not None else os.environ.get("ARENA_NATIVE_SANITIZE", "")
    v = (v or "").strip().lower() or None
    if v is not None and v not in SANITIZERS:
        raise ValueError(f"unknown sanitizer variant {v!r} (expected one of {sorted(SANITIZERS)})")
    return v


def bin_dir(sanitize: Optional[str] = None) -> str:
    v = _variant(sanitize)
    return os.path.join(BIN, v) if v else BIN


def tool_path(name: str, sanitize: Optional[str] = None) -> str:
    return os.path.join(bin_dir(sanitize), name)


def build_native_tools(force: bool = False, sanitize: Optional[str] = None) -> list[str]:
    v = _variant(sanitize)
    out_dir = bin_dir(v)
    os.makedirs(out_dir, exist_ok=True)
    cxx = shutil.which("g++") or shutil.which("c++")
    built = []
    for name, (srcs, flags) in TOOLS.items():
        out = os.path.join(out_dir, name)
        paths = [os.path.join(ROOT, s) for s in srcs]
        deps = paths + [os.path.join(ROOT, "csrc", "runtime", "json.h")]
        if not force and os.path.exists(out) and all(
                os.path.getmtime(out) >= os.path.getmtime(p) for p in deps):
            built.append(out)
            continue
        flags = [f.replace("-Icsrc", "-I" + os.path.join(ROOT, "csrc")) for f in flags]
        if v:  # sanitized: drop the release optimisation flags, keep includes/-pthread
            flags = [f for f in flags if not f.startswith(("-O", "-march"))] + SANITIZERS[v]
        subprocess.run([cxx, "-O2", "-std=c++17", "-Wall", "-Wextra", "-o", out, *paths, *flags],
                       check=True)
        built.append(out)
    return built


def sanitizer_env(sanitize: Optional[str] = None) -> dict:
    """Environment for running a sanitized tool (empty for the release build)."""
    v = _variant(sanitize)
    return dict(SANITIZER_ENV[v]) if v else {}


def ensure_tool(name: str, sanitize: Optional[str] = None) -> str:
    """Path to a native tool, building it on first use (g++ only, seconds)."""
    path = tool_path(name, sanitize)
    if not os.path.exists(path):
        build_native_tools(sanitize=sanitize)
    return path
