"""Scalar logging: TensorBoard-compatible event files without tensorboard.

Reference: ``getSummaryWriter(epochs, del_dir)`` (codes/datawriter.py:6-11) returns a
``torch.utils.tensorboard.SummaryWriter`` under ``./logs/<YYYY-mm-dd>/<HH-MM-SS>-epoch<N>/``
(optionally ``rmtree('./logs/')`` first); lab 1 logs the tag ``'Train Loss'``
(task1/pytorch/model.py:57-61).  ``tensorboard`` is not installed in this image,
so :class:`ScalarWriter` encodes the TFRecord/Event protobuf framing itself
(length + masked CRC32C + serialized ``Event{wall_time, step, summary{value{tag,
simple_value}}}``), which TensorBoard reads natively, and mirrors every scalar to
``scalars.jsonl`` for scripts.  :func:`read_events` decodes the files back (tests).
"""
from __future__ import annotations

import json
import os
import shutil
import socket
import struct
import time
from datetime import datetime
from pathlib import Path

# ---------------------------------------------------------------- crc32c (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf encoding
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


def _key(field, wire):
    return _varint((field << 3) | wire)


def _len_field(field, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _event(wall_time: float, step: int, *, file_version: str | None = None,
           tag: str | None = None, value: float | None = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _len_field(3, file_version.encode())
    if tag is not None:
        val = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
        ev += _len_field(5, _len_field(1, val))
    return ev


def _record(data: bytes) -> bytes:
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data))


class ScalarWriter:
    """Minimal SummaryWriter: ``add_scalar(tag, value, step)``, ``flush``, ``close``."""

    def __init__(self, log_dir: str | os.PathLike):
        self.log_dir = Path(log_dir)
        self.log_dir.mkdir(parents=True, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self._f = open(self.log_dir / name, "wb")
        self._j = open(self.log_dir / "scalars.jsonl", "a")
        self._f.write(_record(_event(time.time(), 0, file_version="brain.Event:2")))
        self.path = self.log_dir / name

    def add_scalar(self, tag: str, scalar_value, global_step: int = 0, walltime=None):
        wt = time.time() if walltime is None else walltime
        v = float(scalar_value)
        self._f.write(_record(_event(wt, global_step, tag=tag, value=v)))
        self._j.write(json.dumps({"tag": tag, "value": v, "step": int(global_step),
                                  "wall_time": wt}) + "\n")

    def flush(self):
        self._f.flush()
        self._j.flush()

    def close(self):
        if not self._f.closed:
            self.flush()
            self._f.close()
            self._j.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def getSummaryWriter(epochs: int, del_dir: bool, root: str = "./logs/") -> ScalarWriter:
    """Reference-compatible factory (codes/datawriter.py:6-11)."""
    if os.path.exists(root) and del_dir:
        shutil.rmtree(root)
    stamp = "{0:%Y-%m-%d/%H-%M-%S}-epoch{1}/".format(datetime.now(), epochs)
    return ScalarWriter(os.path.join(root, stamp))


# ---------------------------------------------------------------- reader (for tests/tools)
def _read_varint(b, i):
    shift = result = 0
    while True:
        c = b[i]
        i += 1
        result |= (c & 0x7F) << shift
        if not c & 0x80:
            return result, i
        shift += 7


def _parse(b):
    i, out = 0, []
    while i < len(b):
        key, i = _read_varint(b, i)
        f, w = key >> 3, key & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v = struct.unpack("<d", b[i:i + 8])[0]
            i += 8
        elif w == 5:
            v = struct.unpack("<f", b[i:i + 4])[0]
            i += 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"wire type {w}")
        out.append((f, v))
    return out


def read_events(path) -> list[dict]:
    """Decode scalar events; verifies both CRCs of every record."""
    data = Path(path).read_bytes()
    i, events = 0, []
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        assert hc == _masked_crc(hdr), "header crc mismatch"
        payload = data[i + 12:i + 12 + n]
        (dc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        assert dc == _masked_crc(payload), "data crc mismatch"
        i += 16 + n
        ev = {"wall_time": None, "step": 0}
        for f, v in _parse(payload):
            if f == 1:
                ev["wall_time"] = v
            elif f == 2:
                ev["step"] = v
            elif f == 3:
                ev["file_version"] = v.decode()
            elif f == 5:
                for f2, val in _parse(v):
                    if f2 == 1:
                        for f3, x in _parse(val):
                            if f3 == 1:
                                ev["tag"] = x.decode()
                            elif f3 == 2:
                                ev["value"] = x
        events.append(ev)
    return events
