"""Durations (reference: util/duration.go:10-27) plus Go-style duration parsing.

``short_human_duration`` reproduces kubectl's age column boundaries exactly:
< -1s -> "<invalid>", < 0 -> "0s", then whole seconds / minutes / hours / days / years.
``parse_duration`` accepts Go syntax ("5s", "2m", "1h30m", "300ms") -- the reference's
``logs --since`` only took integer seconds despite documenting durations (quirk Q9, fixed; bare
integers are still accepted as seconds).
"""
import re

_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
_PART = re.compile(r"(\d+(?:\.\d*)?|\.\d+)(ns|us|µs|ms|s|m|h)")


def short_human_duration(seconds_f: float) -> str:
    seconds = int(seconds_f)  # Go truncates toward zero
    if seconds < -1:
        return "<invalid>"
    if seconds < 0:
        return "0s"
    if seconds < 60:
        return f"{seconds}s"
    minutes = int(seconds_f / 60)
    if minutes < 60:
        return f"{minutes}m"
    hours = int(seconds_f / 3600)
    if hours < 24:
        return f"{hours}h"
    if hours < 24 * 365:
        return f"{hours // 24}d"
    return f"{int(seconds_f / 3600 / 24 / 365)}y"


def parse_duration(text: str) -> float:
    """Seconds from a Go duration string ("1h2m3.5s"); a bare number means seconds."""
    t = text.strip()
    if not t:
        raise ValueError("empty duration")
    sign = 1.0
    if t[0] in "+-":
        sign = -1.0 if t[0] == "-" else 1.0
        t = t[1:]
    if re.fullmatch(r"\d+(\.\d+)?", t):
        return sign * float(t)
    pos, total = 0, 0.0
    for m in _PART.finditer(t):
        if m.start() != pos:
            break
        total += float(m.group(1)) * _UNITS[m.group(2)]
        pos = m.end()
    if pos != len(t) or pos == 0:
        raise ValueError(f"invalid duration {text!r}")
    return sign * total
