"""Version / build metadata (reference: version.go:10-64, Makefile ldflags).

Semver from ``git describe``: a clean tree exactly at a tag -> the tag; otherwise
``v<VERSION>+<sha7>[.dirty]``, or ``+unknown`` outside a git checkout. Build-time values may be
baked into ``arena_amd/_buildinfo.json`` (written by setup/packaging); git is queried otherwise.
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import platform
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)


def base_version() -> str:
    try:
        with open(os.path.join(_ROOT, "VERSION")) as f:
            return f.read().strip()
    except OSError:
        return "0.1.0"


def _git(*args) -> str:
    try:
        return subprocess.run(["git", "-C", _ROOT, *args], capture_output=True, text=True,
                              timeout=5).stdout.strip()
    except Exception:  # noqa: BLE001
        return ""


def semver(tag: str, commit: str, tree_state: str, base: str) -> str:
    if tag and tree_state == "clean":
        return tag
    v = "v" + base
    if commit:
        v += "+" + commit[:7]
        if tree_state == "dirty":
            v += ".dirty"
    else:
        v += "+unknown"
    return v


def get_version() -> dict:
    info = {}
    bi = os.path.join(_HERE, "_buildinfo.json")
    if os.path.exists(bi):
        with open(bi) as f:
            info = json.load(f)
    commit = info.get("gitCommit") or _git("rev-parse", "HEAD")
    tag = info.get("gitTag") if "gitTag" in info else _git("describe", "--exact-match", "--tags")
    state = info.get("gitTreeState") or ("" if not commit else
                                         ("dirty" if _git("status", "--porcelain") else "clean"))
    try:
        import torch
        torch_v = torch.__version__
        rocm_v = getattr(torch.version, "hip", "") or ""
    except Exception:  # noqa: BLE001
        torch_v, rocm_v = "", ""
    return {
        "version": semver(tag, commit, state, base_version()),
        "buildDate": info.get("buildDate", _dt.datetime.now(_dt.timezone.utc).strftime(
            "%Y-%m-%dT%H:%M:%SZ")),
        "gitCommit": commit,
        "gitTreeState": state,
        "gitTag": tag,
        "pythonVersion": sys.version.split()[0],
        "torchVersion": torch_v,
        "rocmVersion": rocm_v,
        "platform": f"{platform.system().lower()}/{platform.machine()}",
    }
