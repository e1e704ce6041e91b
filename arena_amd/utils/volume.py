"""Dataset (PVC) and host data-dir argument parsing (reference: util/volume.go:16-126).

``--data name:/mount``     -> a named volume mounted at an absolute, non-root path;
``--dataDir /host[:/ctr]`` -> a host directory (both absolute, non-root, at most one ':').
"""
import posixpath
import re

from .validate import ValidationError

_NAME_CHARS = r"[a-zA-Z0-9][a-zA-Z0-9_.-]"
_NAME = re.compile(r"^" + _NAME_CHARS + r"+$")


def _check_volume_name(name: str) -> None:
    if len(name) == 1:
        raise ValidationError("volume name is too short, names should be at least two "
                              "alphanumeric characters")
    if not _NAME.match(name):
        raise ValidationError(
            f"{name!r} includes invalid characters for a local volume name, only "
            f"{_NAME_CHARS!r} are allowed. If you intended to pass a host directory, use "
            "absolute path")


def _check_not_root(p: str) -> None:
    if posixpath.normpath(p.replace("\\", "/")) == "/":
        raise ValidationError("invalid specification: dataDir can't be '/'")


def _check_absolute(p: str) -> None:
    p = p.replace("\\", "/")
    if not posixpath.isabs(p):
        raise ValidationError(f"invalid dataDir: '{p}' must be absolute")


def _check_mount_destination(dest: str) -> None:
    _check_not_root(dest)
    _check_absolute(dest)


def _check_host_path(path: str) -> None:
    if path == "":
        raise ValidationError(f"invalid DataDir: '{path}'")
    _check_mount_destination(path)


def validate_datasets(datasets) -> None:
    for ds in datasets:
        parts = ds.split(":")
        if len(parts) != 2:
            raise ValidationError(
                f"dataset {ds} has incorrect format, should like data_name:/data0")
        _check_volume_name(parts[0])
        _check_mount_destination(parts[1])


def parse_data_dir_raw(raw: str):
    """Returns (host_path, container_path)."""
    raw = raw.replace("\\", "/")
    if raw.count(":") > 1:
        raise ValidationError(f"invalid DataDir: '{raw}'")
    arr = raw.split(":")
    if arr[0] == "":
        raise ValidationError(f"invalid DataDir: '{raw}'")
    host, ctr = (arr[0], arr[0]) if len(arr) == 1 else (arr[0], arr[1])
    _check_host_path(host)
    _check_host_path(ctr)
    return host, ctr
