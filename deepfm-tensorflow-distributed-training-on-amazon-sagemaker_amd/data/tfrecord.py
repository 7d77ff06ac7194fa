"""TFRecord input pipeline (the reference's ``input_fn``, PS:112-169 / HVD:104-161).

* ``TFRecordDataset`` — batches of (ids int32 [B,F], vals f32 [B,F], labels f32 [B]) decoded by the
  C++ runtime (csrc/io: mmap + CRC32C + fixed-schema Example decoder + worker pool) into pinned
  host buffers; ``shard(count, index)`` = ``Dataset.shard``; ``drop_remainder`` and per-epoch
  repeat like ``batch(drop_remainder=True) … repeat(num_epochs)``; optional record shuffle buffer
  (the reference has none, Q6); pipe mode reads FIFOs / stdin sequentially (PipeModeDataset).
* ``read_records`` / ``parse_example`` — a tiny pure-Python reader used as a cross-check oracle in
  tests and as a fallback when the native module is unavailable.
* ``discover_files`` — ``glob('{dir}/**/tr*.tfrecords', recursive=True)`` etc. (PS:418-428).
"""
from __future__ import annotations

import glob
import os
import random
import struct
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import io as _io_mod

# --------------------------------------------------------------------------------------------
# file discovery (PS:418-428, HVD:352-361)
# --------------------------------------------------------------------------------------------


def discover_files(data_dir: str, prefix: str, shuffle: bool = False, seed: Optional[int] = None) -> List[str]:
    if not data_dir:
        return []
    files = sorted(glob.glob(os.path.join(data_dir, "**", f"{prefix}*.tfrecords"), recursive=True))
    if shuffle:  # the reference shuffles the training file order (PS:421)
        random.Random(seed).shuffle(files)
    return files


# --------------------------------------------------------------------------------------------
# pure-Python oracle
# --------------------------------------------------------------------------------------------
def _crc32c_py(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 & -(crc & 1))
    return crc ^ 0xFFFFFFFF


def masked_crc32c_py(data: bytes) -> int:
    c = _crc32c_py(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def read_records(path: str, verify: bool = False) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                return
            if len(hdr) < 12:
                raise ValueError("truncated TFRecord header")
            (n,) = struct.unpack("<Q", hdr[:8])
            body = f.read(n)
            (dcrc,) = struct.unpack("<I", f.read(4))
            if verify:
                if masked_crc32c_py(hdr[:8]) != struct.unpack("<I", hdr[8:])[0]:
                    raise ValueError("bad length crc")
                if masked_crc32c_py(body) != dcrc:
                    raise ValueError("bad data crc")
            yield body


def _varint(b: bytes, i: int) -> Tuple[int, int]:
    v = 0
    s = 0
    while True:
        x = b[i]
        i += 1
        v |= (x & 0x7F) << s
        if not x & 0x80:
            return v, i
        s += 7


def _fields(b: bytes):
    i = 0
    while i < len(b):
        tag, i = _varint(b, i)
        fno, wt = tag >> 3, tag & 7
        if wt == 2:
            n, i = _varint(b, i)
            yield fno, wt, b[i:i + n]
            i += n
        elif wt == 0:
            v, i = _varint(b, i)
            yield fno, wt, v
        elif wt == 5:
            yield fno, wt, b[i:i + 4]
            i += 4
        elif wt == 1:
            yield fno, wt, b[i:i + 8]
            i += 8
        else:
            raise ValueError("bad wire type")


def parse_example(payload: bytes) -> dict:
    """Decode a tf.train.Example into {name: list} (float_list → floats, int64_list → ints)."""
    out = {}
    for fno, _, feats in _fields(payload):
        if fno != 1:
            continue
        for f2, _, entry in _fields(feats):
            if f2 != 1:
                continue
            key, val = None, None
            for f3, _, x in _fields(entry):
                if f3 == 1:
                    key = x.decode()
                elif f3 == 2:
                    val = x
            values = []
            for kind, _, lst in _fields(val):
                for f5, wt, x in _fields(lst):
                    if kind == 2:  # float_list
                        if wt == 2:
                            values += list(struct.unpack(f"<{len(x) // 4}f", x))
                        else:
                            values.append(struct.unpack("<f", x)[0])
                    elif kind == 3:  # int64_list
                        if wt == 2:
                            j = 0
                            while j < len(x):
                                v, j = _varint(x, j)
                                values.append(v - (1 << 64) if v >= 1 << 63 else v)
                        else:
                            values.append(x - (1 << 64) if x >= 1 << 63 else x)
                    else:
                        values.append(x)
            out[key] = values
    return out


class RawGroup:
    """``n`` undecoded batches: ``bytes [n, cap]`` uint8 payloads and ``offs [n, B+1]`` int32
    offsets (batch k's record r is ``bytes[k, offs[k, r]:offs[k, r+1]]``), pinned host memory."""

    __slots__ = ("bytes", "offs", "n", "B")

    def __init__(self, bytes_: torch.Tensor, offs: torch.Tensor, n: int, B: int):
        self.bytes, self.offs, self.n, self.B = bytes_, offs, int(n), int(B)

    def used_bytes(self) -> int:
        """Bytes from the first batch's start to the end of the last batch's payloads."""
        return (self.n - 1) * self.bytes.shape[1] + int(self.offs[self.n - 1, self.B])

    def decode_host(self, field_size: int, feature_size: int = 0):
        """Decode on the host (tests / CPU fallback): (ids [n,B,F], vals [n,B,F], labels [n,B])."""
        io = _io_mod()
        n, B, F = self.n, self.B, int(field_size)
        ids = torch.zeros(n, B, F, dtype=torch.int32)
        vals = torch.zeros(n, B, F, dtype=torch.float32)
        labels = torch.zeros(n, B, dtype=torch.float32)
        raw = self.bytes.numpy()
        offs = self.offs.numpy()
        for k in range(n):
            for r in range(B):
                st, lab, i, v = io.decode_example(raw[k, offs[k, r]:offs[k, r + 1]].tobytes(), F, int(feature_size))
                if st != 0:
                    raise ValueError(f"decode error {st} in batch {k} record {r}")
                ids[k, r] = torch.from_numpy(i)
                vals[k, r] = torch.from_numpy(v)
                labels[k, r] = lab
        return ids, vals, labels


# --------------------------------------------------------------------------------------------
# native batch loader
# --------------------------------------------------------------------------------------------
class TFRecordDataset:
    """Iterable of host batches decoded by the C++ loader.

    Each yielded batch is a tuple of CPU tensors living in one of ``num_slots`` pinned buffers; the
    slot is recycled when the NEXT batch is requested, so consumers must copy (e.g. an async H2D
    copy followed by using the device tensor) before advancing the iterator twice.  ``hold=h``
    delays the recycling: a batch's slot is released when batch t+h is requested (consumers that
    keep ``h`` asynchronous copies in flight; the pool grows to keep 4 slots for the decoders).

    ``shard_policy="file"`` shards by file instead of by record: shard i reads ``files[i::count]``
    (needs ≥ count files), so the ranks of one host walk each byte once instead of every rank walking
    every file's framing (``profiles/r3_loader_aggregate.md``).
    """

    def __init__(self, files: Sequence[str], field_size: int, batch_size: int, feature_size: int = 0,
                 num_epochs: int = 1, shard_count: int = 1, shard_index: int = 0, drop_remainder: bool = True,
                 num_threads: int = 4, num_slots: int = 6, verify_crc: bool = True, skip_bad: bool = False,
                 shuffle_buffer: int = 0, seed: int = 0, stream_mode: bool = False, pin_memory: Optional[bool] = None,
                 hold: int = 1, shard_policy: str = "record", max_batches_per_epoch: int = 0):
        self.files = list(files)
        if shard_policy not in ("record", "file"):
            raise ValueError(f"shard_policy must be record or file, got {shard_policy!r}")
        if shard_policy == "file" and int(shard_count) > 1:
            if stream_mode:
                raise ValueError("shard_policy=file: file mode only (a pipe-mode channel is one stream)")
            if len(self.files) < int(shard_count):
                raise ValueError(f"shard_policy=file needs at least {shard_count} files, got {len(self.files)}")
            self.files = self.files[int(shard_index)::int(shard_count)]
            shard_count, shard_index = 1, 0
        self.F = int(field_size)
        self.B = int(batch_size)
        self.hold = max(1, int(hold))
        num_slots = max(int(num_slots), self.hold + 4)
        self.kw = dict(field_size=self.F, max_id=int(feature_size), batch_size=self.B, drop_remainder=drop_remainder,
                       num_epochs=int(num_epochs), shard_count=int(shard_count), shard_index=int(shard_index),
                       num_threads=int(num_threads), num_slots=int(num_slots), verify_crc=verify_crc,
                       skip_bad=skip_bad, shuffle_buffer=int(shuffle_buffer), seed=int(seed),
                       stream_mode=stream_mode, max_batches_per_epoch=int(max_batches_per_epoch))
        self.num_slots = int(num_slots)
        if pin_memory is None:
            pin_memory = torch.cuda.is_available()
        self.pin = pin_memory
        self.loader = None

    def __iter__(self):
        io = _io_mod()
        if io is None:
            raise RuntimeError("rocfm native IO module missing; run `python build.py`")
        self.loader = io.BatchLoader(self.files, **self.kw)
        bufs = []
        for i in range(self.num_slots):
            ids = torch.zeros(self.B, self.F, dtype=torch.int32, pin_memory=self.pin)
            vals = torch.zeros(self.B, self.F, dtype=torch.float32, pin_memory=self.pin)
            labels = torch.zeros(self.B, dtype=torch.float32, pin_memory=self.pin)
            self.loader.set_slot(i, ids.data_ptr(), vals.data_ptr(), labels.data_ptr())
            bufs.append((ids, vals, labels))
        self.loader.start()
        held = []
        try:
            while True:
                slot, rows, epoch = self.loader.next()
                while len(held) >= self.hold or (slot < 0 and held):
                    self.loader.release(held.pop(0))
                if slot < 0:
                    break
                held.append(slot)
                ids, vals, labels = bufs[slot]
                yield ids[:rows], vals[:rows], labels[:rows]
        finally:
            self.loader.stop()

    def groups(self, size: int, hold: int = 2, skip: int = 0, limit: Optional[int] = None):
        """Iterate over groups of ``size`` consecutive batches (fewer at the end of the data) as
        stacked views ``ids [n,B,F]``, ``vals [n,B,F]``, ``labels [n,B]`` of ONE pinned slot ring,
        so a consumer moves a whole group with one host→device copy per tensor.  The ring holds
        ``(hold + 2) · size`` batches; a group's slots are recycled when the group ``hold`` places
        later is requested.  ``skip`` batches are dropped undecoded by the C++ reader (resume);
        ``limit`` caps the number of batches yielded.  A trailing partial batch (drop_remainder
        False) is yielded on its own as a 2-D batch."""
        io = _io_mod()
        if io is None:
            raise RuntimeError("rocfm native IO module missing; run `python build.py`")
        size, hold = max(1, int(size)), max(1, int(hold))
        ns = (hold + 2) * size
        kw = dict(self.kw, num_slots=ns, skip_batches=int(skip))
        self.loader = io.BatchLoader(self.files, **kw)
        B, F = self.B, self.F
        ids = torch.zeros(ns, B, F, dtype=torch.int32, pin_memory=self.pin)
        vals = torch.zeros(ns, B, F, dtype=torch.float32, pin_memory=self.pin)
        labels = torch.zeros(ns, B, dtype=torch.float32, pin_memory=self.pin)
        for i in range(ns):
            self.loader.set_slot(i, ids[i].data_ptr(), vals[i].data_ptr(), labels[i].data_ptr())
        self.loader.start()
        held = []
        left = -1 if limit is None else int(limit)
        try:
            while left != 0:
                first, n, rows, epoch = self.loader.next_group(size if left < 0 else min(size, left))
                while len(held) >= hold or (n == 0 and held):
                    self.loader.release_group(*held.pop(0))
                if n == 0:
                    break
                held.append((first, n))
                left -= n if left > 0 else 0
                full = n if rows == B else n - 1
                if full:
                    yield ids[first:first + full], vals[first:first + full], labels[first:first + full]
                if full < n:
                    last = first + n - 1
                    yield ids[last, :rows], vals[last, :rows], labels[last, :rows]
        finally:
            self.loader.stop()

    def raw_groups(self, size: int, hold: int = 2, skip: int = 0, limit: Optional[int] = None,
                   record_bytes: int = 0):
        """Like ``groups`` but the batches stay undecoded: each item is a ``RawGroup`` of ``n``
        consecutive full batches whose Example payloads sit back to back in one pinned byte ring
        (``bytes [n, cap]``, batch k at row k) with their offsets (``offs [n, B+1]`` int32).  The
        host only resolves frames, checks CRCs and copies bytes; the GPU parses the Examples
        (``csrc/kernels/decode.hip``, rocfm.models.fused.FusedDeepFM.train_stream).  ``cap`` is
        ``B × record_bytes`` (default: the longest record of the files' indexes, rounded up to
        16 B).  Needs file mode with drop_remainder (a partial batch cannot be trained) and no
        skip_bad (a malformed record is only found on the device)."""
        io = _io_mod()
        if io is None:
            raise RuntimeError("rocfm native IO module missing; run `python build.py`")
        if self.kw["stream_mode"] or not self.kw["drop_remainder"] or self.kw["skip_bad"]:
            raise ValueError("raw_groups needs file mode, drop_remainder and no skip_bad")
        size, hold = max(1, int(size)), max(1, int(hold))
        B = self.B
        rb = int(record_bytes) or self.max_record_bytes()
        cap = B * ((rb + 15) // 16 * 16)
        ns = (hold + 2) * size
        kw = dict(self.kw, num_slots=ns, skip_batches=int(skip), raw=True, raw_cap=cap)
        self.loader = io.BatchLoader(self.files, **kw)
        raw = torch.zeros(ns, cap, dtype=torch.uint8, pin_memory=self.pin)
        offs = torch.zeros(ns, B + 1, dtype=torch.int32, pin_memory=self.pin)
        for i in range(ns):
            self.loader.set_raw_slot(i, raw[i].data_ptr(), offs[i].data_ptr())
        self.loader.start()
        held = []
        left = -1 if limit is None else int(limit)
        try:
            while left != 0:
                first, n, rows, epoch = self.loader.next_group(size if left < 0 else min(size, left))
                while len(held) >= hold or (n == 0 and held):
                    self.loader.release_group(*held.pop(0))
                if n == 0:
                    break
                held.append((first, n))
                left -= n if left > 0 else 0
                yield RawGroup(raw[first:first + n], offs[first:first + n], n, B)
        finally:
            self.loader.stop()

    def max_record_bytes(self) -> int:
        """Longest Example payload over the files (from their saved indexes; built when missing)."""
        io = _io_mod()
        m = 0
        for f in self.files:
            info = io.index_info(f)
            if info is None:
                io.build_index(f, bool(self.kw["verify_crc"]))
                info = io.index_info(f)
            if info is None:  # unwritable directory: walk the framing for the lengths
                m = max([m] + list(io.scan_file(f, False, False)[2]))
            else:
                m = max(m, int(info[1]))
        return max(m, 16)

    def num_batches(self) -> Optional[int]:
        """Batches this shard will yield over all epochs (file mode; None for a stream/FIFO source).

        Counts records from the files' saved indexes (or by walking the framing only, C++
        ``count_records``), then applies the record-index sharding, the per-epoch drop_remainder
        and the per-epoch cap of the loader.  Upper bound when ``skip_bad`` drops corrupt records."""
        if self.kw["stream_mode"]:
            return None
        return self.batches_per_epoch() * self.kw["num_epochs"]

    def batches_per_epoch(self) -> Optional[int]:
        if self.kw["stream_mode"]:
            return None
        io = _io_mod()
        if io is None:
            raise RuntimeError("rocfm native IO module missing; run `python build.py`")
        N = 0
        for f in self.files:
            info = io.index_info(f)
            N += int(info[0]) if info is not None else int(io.count_records(f))
        c, i = self.kw["shard_count"], self.kw["shard_index"]
        n = (N - i + c - 1) // c if N > i else 0
        per_epoch = n // self.B if self.kw["drop_remainder"] else (n + self.B - 1) // self.B
        cap = int(self.kw.get("max_batches_per_epoch", 0))
        return min(per_epoch, cap) if cap > 0 else per_epoch

    @property
    def bad_records(self) -> int:
        return 0 if self.loader is None else int(self.loader.bad_records)


def decode_file(path: str, field_size: int, feature_size: int = 0, verify_crc: bool = True, skip_bad: bool = False):
    """Whole file → (labels [N], ids [N,F] int32, vals [N,F]) tensors (small files / eval sets)."""
    io = _io_mod()
    if io is None:  # pure-Python fallback
        L, I, V = [], [], []
        for rec in read_records(path, verify=verify_crc):
            ex = parse_example(rec)
            L.append(ex["label"][0])
            I.append(ex["ids"])
            V.append(ex["values"])
        return (torch.tensor(L, dtype=torch.float32), torch.tensor(I, dtype=torch.int32),
                torch.tensor(V, dtype=torch.float32))
    L, I, V = io.decode_file(path, field_size, feature_size, verify_crc, skip_bad)
    return torch.from_numpy(L), torch.from_numpy(I), torch.from_numpy(V)


def write_tfrecord(path: str, labels, ids, vals, append: bool = False) -> int:
    io = _io_mod()
    return io.write_tfrecord(path, np.asarray(labels, np.float32), np.asarray(ids, np.int64),
                             np.asarray(vals, np.float32), append)
