"""Loader for the in-tree native extension ``arena_amd._C`` (HIP kernels for gfx950).

GPU tensors always go through the HIP kernels. If the extension is missing on a machine with a
GPU, every GPU op raises :class:`NativeExtensionMissing` instead of silently falling back to
PyTorch (the round-end GPU check records which ``.so`` files were actually loaded).
"""
from __future__ import annotations

import importlib
import os

_EXT = None
_ERR: Exception | None = None


class NativeExtensionMissing(RuntimeError):
    pass


def load():
    """Return the ``arena_amd._C`` module, importing it on first use."""
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    if _ERR is not None:
        raise NativeExtensionMissing(
            "arena_amd._C is not built (run `python setup.py build_ext --inplace` or "
            f"`python -c 'import __graft_entry__ as g; g.build()'`): {_ERR}")
    try:
        mod = importlib.import_module("arena_amd._C")
        csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
            os.path.abspath(__file__)))), "csrc")
        if os.path.isdir(os.path.join(csrc, "ops")):
            from ._srchash import source_hash
            want = source_hash(os.path.join(csrc, "ops"), os.path.join(csrc, "ccl"))
            if getattr(mod, "src_hash", None) != want:
                raise RuntimeError(f"stale build: extension built from sources {mod.src_hash}, "
                                   f"tree has {want}")
        _EXT = mod
    except Exception as e:  # noqa: BLE001 - report any import failure verbatim
        _ERR = e
        return load()
    return _EXT


def available() -> bool:
    try:
        load()
        return True
    except NativeExtensionMissing:
        return False


def so_path() -> str | None:
    try:
        return load().__file__
    except NativeExtensionMissing:
        return None
