"""TensorBoard event-file writer (no tensorflow / tensorboard needed).

Replaces ``keras.callbacks.TensorBoard`` of the reference (rank 0 only,
``/root/reference/train.py:119-131``): scalars ``loss``,
``regression_loss``, ``classification_loss``, ``lr`` (and evaluation metrics) per epoch.

Format: TFRecord framing (``uint64 len``, masked CRC32C of len, payload, masked CRC32C of
payload) of hand-encoded ``tensorflow.Event`` protobufs (wall_time=1, step=2, file_version=3,
summary=5 -> Summary.value=1 -> {tag=1, simple_value=2}).  CRC32C is the native C++ one.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Optional

from ..utils.cpu_native import crc32c


def _masked_crc(data: bytes) -> int:
    crc = crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


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


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, file_version: Optional[str] = None,
                 scalars: Optional[Dict[str, float]] = None, text: Optional[Dict[str, str]] = None) -> bytes:
    msg = _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    msg += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        msg += _field_bytes(3, file_version.encode())
    if scalars:
        summary = b""
        for tag, v in scalars.items():
            val = _field_bytes(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(v))
            summary += _field_bytes(1, val)
        msg += _field_bytes(5, summary)
    return msg


def frame(record: bytes) -> bytes:
    hdr = struct.pack("<Q", len(record))
    return hdr + struct.pack("<I", _masked_crc(hdr)) + record + struct.pack("<I", _masked_crc(record))


class EventFileWriter:
    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = "events.out.tfevents.{}.{}{}".format(int(time.time()), socket.gethostname(), filename_suffix)
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(frame(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalars(self, scalars: Dict[str, float], step: int) -> None:
        self._f.write(frame(encode_event(time.time(), step, scalars=scalars)))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self.add_scalars({tag: value}, step)

    def close(self) -> None:
        if self._f:
            self._f.close()
            self._f = None


def read_events(path: str):
    """Parse an event file back into [(step, {tag: value})] (tests / tooling)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    p = 0
    while p + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, p)
        if struct.unpack_from("<I", data, p + 8)[0] != _masked_crc(data[p:p + 8]):
            raise ValueError("bad length crc at {}".format(p))
        rec = data[p + 12:p + 12 + n]
        if struct.unpack_from("<I", data, p + 12 + n)[0] != _masked_crc(rec):
            raise ValueError("bad data crc at {}".format(p))
        p += 16 + n
        out.append(_decode_event(rec))
    return out


def _read_varint(b, i):
    shift = res = 0
    while True:
        c = b[i]
        i += 1
        res |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return res, i


def _fields(b):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError("wire type {}".format(wt))
        yield num, wt, v


def _decode_event(rec):
    step, scalars = 0, {}
    for num, wt, v in _fields(rec):
        if num == 2:
            step = v
        elif num == 5:
            for n2, _, val in _fields(v):
                if n2 == 1:
                    tag, sv = None, None
                    for n3, w3, x in _fields(val):
                        if n3 == 1:
                            tag = x.decode()
                        elif n3 == 2:
                            sv = struct.unpack("<f", x)[0]
                    if tag is not None:
                        scalars[tag] = sv
    return step, scalars
