"""Minimal TensorBoard event-file writer/reader (no TensorFlow / tensorboard dependency).

Files are TFRecord streams of ``Event`` protos (hand-encoded protobuf wire format):
  record = u64 len | u32 masked_crc32c(len) | data | u32 masked_crc32c(data)
  Event  = {1: wall_time (double), 2: step (int64), 3: file_version (string), 5: Summary}
  Summary.Value = {1: tag (string), 2: simple_value (float)}
so TensorBoard itself can read what the bundled MNIST jobs write (the reference's demo workloads
log scalars for `--tensorboard`, docs/userguide/2-tfjob-tensorboard.md).
"""
from __future__ import annotations

import glob
import os
import socket
import struct
import time
from typing import Dict, List, Tuple

_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, file_version: str = None,
                 scalars: Dict[str, float] = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(step)
    if file_version is not None:
        ev += _ld(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = _ld(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
            summ += _ld(1, val)
        ev += _ld(5, summ)
    return ev


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", masked_crc(hdr)) + data + struct.pack("<I", masked_crc(data))


class SummaryWriter:
    """``SummaryWriter(logdir).add_scalar(tag, value, step)`` -> events.out.tfevents.* file."""

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(_record(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self._f.write(_record(encode_event(time.time(), int(step), scalars={tag: value})))

    def add_scalars(self, values: Dict[str, float], step: int) -> None:
        self._f.write(_record(encode_event(time.time(), int(step), scalars=values)))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        self._f.close()


# ----------------------------------------------------------------------------------- reader
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        x = b[i]
        i += 1
        n |= (x & 0x7F) << shift
        if not x & 0x80:
            return n, i
        shift += 7


def _fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _read_varint(b, i)
            v, i = b[i:i + ln], i + ln
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError("unsupported wire type")
        yield f, wt, v


def read_events(path: str):
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i + 12 <= len(data):
        (ln,) = struct.unpack("<Q", data[i:i + 8])
        if i + 12 + ln + 4 > len(data):
            break
        payload = data[i + 12:i + 12 + ln]
        (crc,) = struct.unpack("<I", data[i + 12 + ln:i + 16 + ln])
        i += 16 + ln
        if crc != masked_crc(payload):
            continue
        ev = {"wall_time": 0.0, "step": 0, "scalars": {}}
        for f, wt, v in _fields(payload):
            if f == 1 and wt == 1:
                ev["wall_time"] = struct.unpack("<d", v)[0]
            elif f == 2 and wt == 0:
                ev["step"] = v
            elif f == 5 and wt == 2:
                for vf, _, vv in _fields(v):
                    if vf != 1:
                        continue
                    tag, sv = None, None
                    for ff, wwt, x in _fields(vv):
                        if ff == 1:
                            tag = x.decode()
                        elif ff == 2 and wwt == 5:
                            sv = struct.unpack("<f", x)[0]
                    if tag is not None and sv is not None:
                        ev["scalars"][tag] = sv
        yield ev


def read_scalars(logdir: str) -> Dict[str, Dict[str, List[Tuple[int, float]]]]:
    """{run: {tag: [(step, value), ...]}} for every event file under ``logdir``."""
    out: Dict[str, Dict[str, List[Tuple[int, float]]]] = {}
    for path in sorted(glob.glob(os.path.join(logdir, "**", "events.out.tfevents.*"),
                                 recursive=True)):
        run = os.path.relpath(os.path.dirname(path), logdir) or "."
        tags = out.setdefault(run, {})
        for ev in read_events(path):
            for tag, v in ev["scalars"].items():
                tags.setdefault(tag, []).append((ev["step"], v))
    return out
