"""Shared bits of the bundled examples: device choice, data, TensorBoard dirs, checkpoints."""
from __future__ import annotations

import os

import torch


def pick_device(flag: str = "auto") -> torch.device:
    if flag == "auto":
        if torch.cuda.is_available():
            return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        return torch.device("cpu")
    return torch.device(flag)


def default_log_dir(flag: str) -> str:
    return flag or os.environ.get("ARENA_TRAINING_LOGDIR") or os.path.join("/tmp", "arena_mnist_logs")


def save_checkpoint(path: str, state: dict) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str):
    if not path or not os.path.exists(path):
        return None
    return torch.load(path, map_location="cpu", weights_only=True)


def share_cpu_threads(local_procs: int) -> None:
    """CPU runs with several ranks on one host: split the cores instead of letting every rank's
    OpenMP pool spin on all of them (oversubscription makes each step ~100x slower)."""
    if local_procs > 1:
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // local_procs))
