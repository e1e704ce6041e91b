"""Leveled logging (reference: util/logs.go:10-23, logrus). Unknown levels are fatal."""
import logging
import sys

_LEVELS = {"debug": logging.DEBUG, "info": logging.INFO, "warn": logging.WARNING,
           "warning": logging.WARNING, "error": logging.ERROR}
_ROOT = "arena"


def get_logger(name: str = "") -> logging.Logger:
    return logging.getLogger(_ROOT + ("." + name if name else ""))


def set_log_level(level: str) -> None:
    if level not in _LEVELS:
        sys.stderr.write(f"Unsupported log level: {level}\n")
        raise SystemExit(1)
    root = logging.getLogger(_ROOT)
    if not root.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(levelname)s[%(asctime)s] %(message)s",
                                         "%Y-%m-%dT%H:%M:%S"))
        root.addHandler(h)
    root.setLevel(_LEVELS[level])
