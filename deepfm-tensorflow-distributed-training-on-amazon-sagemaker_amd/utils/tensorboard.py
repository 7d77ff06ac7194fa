"""TensorBoard scalar event files without TensorFlow.

The reference's ``tf.estimator.Estimator`` writes ``events.out.tfevents.*`` summaries into
``model_dir`` (training: ``loss``, ``global_step/sec``) and ``model_dir/eval`` (evaluation metrics)
(``DeepFM-dist-ps-multiInstance.py:494`` builds the Estimator with ``model_dir``; the summaries come
from TF itself).  This module writes the same file format so the same TensorBoard invocation works:

* framing: TFRecord records — u64 length, masked CRC32C of the length, payload, masked CRC32C of
  the payload (the same framing the input pipeline reads, ``data/tfrecord.py``);
* payload: a hand-encoded ``tensorflow.Event`` protobuf — ``wall_time`` (field 1, double), ``step``
  (field 2, int64), ``file_version`` (field 3, string; the first record) or ``summary`` (field 5)
  holding ``Summary.Value{tag (1), simple_value (2, float)}`` entries.

``read_scalars`` decodes such files back (tests; no TensorFlow needed).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Iterator, List, Optional, Tuple

_io = None


def _masked_crc(data: bytes) -> int:
    global _io
    if _io is None:
        try:
            from .. import _rocfm_io as m  # SSE4.2 CRC32C (csrc/io/tfrecord.cpp)
            _io = m
        except ImportError:
            _io = False
    if _io:
        return int(_io.masked_crc32c(data))
    from ..data.tfrecord import masked_crc32c_py

    return masked_crc32c_py(data)


def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int, scalars: Optional[Dict[str, float]] = None,
                 file_version: Optional[str] = None) -> bytes:
    ev = _varint(1 << 3 | 1) + struct.pack("<d", float(wall_time)) + _varint(2 << 3 | 0) + _varint(int(step))
    if file_version is not None:
        ev += _field_bytes(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, val in scalars.items():
            v = _field_bytes(1, str(tag).encode()) + _varint(2 << 3 | 5) + struct.pack("<f", float(val))
            summ += _field_bytes(1, v)
        ev += _field_bytes(5, summ)
    return ev


def frame(payload: bytes) -> bytes:
    n = struct.pack("<Q", len(payload))
    return n + struct.pack("<I", _masked_crc(n)) + payload + struct.pack("<I", _masked_crc(payload))


class EventWriter:
    """Appends scalar summaries to ``<logdir>/events.out.tfevents.<time>.<host>``."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        now = time.time()
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(now)}.{socket.gethostname()}{filename_suffix}")
        self._fh = open(self.path, "ab")
        self._fh.write(frame(encode_event(now, 0, file_version="brain.Event:2")))
        self._fh.flush()

    def scalars(self, step: int, values: Dict[str, float], wall_time: Optional[float] = None) -> None:
        vals = {k: float(v) for k, v in values.items() if v is not None}
        if not vals or self._fh is None:
            return
        self._fh.write(frame(encode_event(time.time() if wall_time is None else wall_time, step, vals)))
        self._fh.flush()

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None


# ---- decoding (tests / tooling) ------------------------------------------------------------------
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _fields(b: bytes) -> Iterator[Tuple[int, int, object]]:
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield num, wt, v


def read_scalars(path: str, verify: bool = True) -> List[Tuple[int, str, float]]:
    """(step, tag, value) of every scalar in an event file (CRCs checked when ``verify``)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        if verify and struct.unpack_from("<I", data, i + 8)[0] != _masked_crc(data[i:i + 8]):
            raise ValueError(f"{path}: bad length CRC at offset {i}")
        payload = data[i + 12:i + 12 + n]
        if verify and struct.unpack_from("<I", data, i + 12 + n)[0] != _masked_crc(payload):
            raise ValueError(f"{path}: bad payload CRC at offset {i}")
        i += 16 + n
        step = 0
        for num, _, v in _fields(payload):
            if num == 2:
                step = int(v)
            elif num == 5:
                for vn, _, val in _fields(v):
                    if vn != 1:
                        continue
                    tag, x = None, None
                    for fn, _, fv in _fields(val):
                        if fn == 1:
                            tag = fv.decode()
                        elif fn == 2:
                            (x,) = struct.unpack("<f", fv)
                    if tag is not None and x is not None:
                        out.append((step, tag, x))
    return out
