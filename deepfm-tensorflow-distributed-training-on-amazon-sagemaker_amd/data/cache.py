"""Pre-decoded on-disk cache of a rank's training stream (SURVEY §1 L5 "binary cache", §7.4-3).

The reference's tf.data pipeline re-reads and re-parses every TFRecord every epoch (PS:147-165,
HVD:128-159).  At MI355X step rates one process decodes 27-36 M examples/s with 16 threads
(``profiles/r2_loader_fed_e2e.md``) — about what ONE GPU consumes — so eight ranks decoding at
once need most of a host's cores.  The decoded batches are tiny and regular (int32 ids [B,F],
f32 values [B,F], f32 labels [B]: 8F+4 bytes per example), so this cache stores one epoch of a
rank's shard raw, in three flat files plus a manifest, and later epochs (and later jobs on the
same files, shard and batch size) memory-map it: a read is a memcpy into the pinned staging
ring, with no CRC, varint or protobuf work.

Layout of ``<cache_dir>/<key>/``: ``ids.bin`` [N,B,F] int32, ``vals.bin`` [N,B,F] f32,
``labels.bin`` [N,B] f32, ``manifest.json`` (written last, atomically: its presence marks a
complete cache).  ``key`` hashes the file list (absolute paths, sizes, mtimes), the shard
(count, index), B, F, the id bound and the record-verification options.
"""
from __future__ import annotations

import hashlib
import json
import os
import threading
from typing import Iterable, Iterator, Optional

import numpy as np
import torch

VERSION = 1


class DecodedCache:
    def __init__(self, path: str, batch_size: int, field_size: int):
        self.path = path
        self.B, self.F = int(batch_size), int(field_size)

    # ---- construction ---------------------------------------------------------------------------
    @staticmethod
    def key_for(files, shard_count: int, shard_index: int, B: int, F: int, max_id: int, extra: str = "") -> str:
        h = hashlib.sha256()
        for f in files:
            st = os.stat(f)
            h.update(f"{os.path.abspath(f)}|{st.st_size}|{int(st.st_mtime_ns)}\n".encode())
        h.update(f"v{VERSION}|{shard_count}|{shard_index}|{B}|{F}|{max_id}|{extra}".encode())
        return h.hexdigest()[:24]

    @classmethod
    def for_dataset(cls, ds, cache_dir: str) -> "DecodedCache":
        """The cache of one epoch of ``ds`` (a rocfm.data.tfrecord.TFRecordDataset in file mode,
        drop_remainder, no record shuffle)."""
        kw = ds.kw
        if kw["stream_mode"] or kw["shuffle_buffer"] or not kw["drop_remainder"]:
            raise ValueError("decoded cache: file mode, drop_remainder and no record shuffle only")
        key = cls.key_for(ds.files, kw["shard_count"], kw["shard_index"], ds.B, ds.F, kw["max_id"],
                          extra=f"crc{int(kw['verify_crc'])}skip{int(kw['skip_bad'])}")
        return cls(os.path.join(cache_dir, key), ds.B, ds.F)

    def _manifest(self) -> Optional[dict]:
        try:
            with open(os.path.join(self.path, "manifest.json")) as f:
                m = json.load(f)
        except (OSError, ValueError):
            return None
        if m.get("version") != VERSION or m.get("B") != self.B or m.get("F") != self.F:
            return None
        return m

    def complete(self) -> bool:
        return self._manifest() is not None

    def num_batches(self) -> int:
        m = self._manifest()
        return int(m["batches"]) if m else 0

    # ---- write ----------------------------------------------------------------------------------
    def write_through(self, groups: Iterable) -> Iterator:
        """Yield ``groups`` (stacked [n,B,F] / single [B,F] host batches) unchanged while appending
        every full batch to the cache; the manifest is written once the source is exhausted, so a
        pass that stops early (max_steps, a failure) leaves no complete cache behind."""
        os.makedirs(self.path, exist_ok=True)
        tmp = {k: os.path.join(self.path, f"{k}.bin.part") for k in ("ids", "vals", "labels")}
        fh = {k: open(p, "wb") for k, p in tmp.items()}
        n = 0
        ok = False
        try:
            for g in groups:
                ids, vals, labels = g
                if ids.dim() == 2:
                    if ids.shape[0] == self.B:
                        fh["ids"].write(ids.numpy().tobytes())
                        fh["vals"].write(vals.numpy().tobytes())
                        fh["labels"].write(labels.numpy().tobytes())
                        n += 1
                else:
                    fh["ids"].write(ids.numpy().tobytes())
                    fh["vals"].write(vals.numpy().tobytes())
                    fh["labels"].write(labels.numpy().tobytes())
                    n += int(ids.shape[0])
                yield g
            ok = True
        finally:
            for f in fh.values():
                f.close()
            if ok:
                for k, p in tmp.items():
                    os.replace(p, os.path.join(self.path, f"{k}.bin"))
                m = {"version": VERSION, "B": self.B, "F": self.F, "batches": n}
                with open(os.path.join(self.path, "manifest.json.part"), "w") as f:
                    json.dump(m, f)
                os.replace(os.path.join(self.path, "manifest.json.part"), os.path.join(self.path, "manifest.json"))
            else:
                for p in tmp.values():
                    try:
                        os.remove(p)
                    except OSError:
                        pass

    # ---- read -----------------------------------------------------------------------------------
    def arrays(self):
        """Memory-mapped (ids [N,B,F] int32, vals [N,B,F] f32, labels [N,B] f32)."""
        n = self.num_batches()
        if n == 0:
            raise FileNotFoundError(f"no complete decoded cache at {self.path}")
        B, F = self.B, self.F
        mm = lambda k, dt, shape: np.memmap(os.path.join(self.path, f"{k}.bin"), dtype=dt, mode="c", shape=shape)  # copy-on-write: writable views, never written
        return mm("ids", np.int32, (n, B, F)), mm("vals", np.float32, (n, B, F)), mm("labels", np.float32, (n, B))

    def groups(self, size: int, hold: int = 2, skip: int = 0, limit: Optional[int] = None,
               pin_memory: Optional[bool] = None) -> Iterator:
        """Groups of ``size`` consecutive cached batches as stacked views of ONE pinned staging
        ring (same contract as TFRecordDataset.groups: a group's slots are reused when the group
        ``hold`` places later is requested).  A helper thread copies group g+1 out of the memory
        map while the consumer handles group g."""
        ids_m, vals_m, lab_m = self.arrays()
        n_all = ids_m.shape[0]
        lo = min(int(skip), n_all)
        hi = n_all if limit is None else min(n_all, lo + int(limit))
        if hi <= lo:
            return
        size, hold = max(1, int(size)), max(1, int(hold))
        pin = torch.cuda.is_available() if pin_memory is None else pin_memory
        nring = hold + 2  # groups in flight: `hold` held by the consumer, one being filled, one ready
        B, F = self.B, self.F
        ring = [(torch.empty(size, B, F, dtype=torch.int32, pin_memory=pin),
                 torch.empty(size, B, F, dtype=torch.float32, pin_memory=pin),
                 torch.empty(size, B, dtype=torch.float32, pin_memory=pin)) for _ in range(nring)]
        starts = list(range(lo, hi, size))

        def fill(j):
            a = starts[j]
            m = min(size, hi - a)
            r = ring[j % nring]
            r[0][:m].copy_(torch.from_numpy(np.asarray(ids_m[a:a + m])))
            r[1][:m].copy_(torch.from_numpy(np.asarray(vals_m[a:a + m])))
            r[2][:m].copy_(torch.from_numpy(np.asarray(lab_m[a:a + m])))
            return m

        res = {}
        th = None

        def launch(j):
            def run():
                res[j] = fill(j)
            t = threading.Thread(target=run, daemon=True)
            t.start()
            return t

        th = launch(0)
        for j in range(len(starts)):
            th.join()
            m = res.pop(j)
            # group j+1 goes to ring slot (j+1) % nring, last handed out as group j+1-nring ≤ j-hold-1:
            # released by the consumer when it requested group j-1 (it holds at most `hold` groups)
            th = launch(j + 1) if j + 1 < len(starts) else None
            r = ring[j % nring]
            yield r[0][:m], r[1][:m], r[2][:m]
        if th is not None:
            th.join()


def cached_epochs(cache: DecodedCache, make_groups, num_epochs: int, size: int, hold: int = 2, skip: int = 0,
                  limit: Optional[int] = None) -> Iterator:
    """``num_epochs`` passes over one epoch of a rank's training stream: the first from
    ``make_groups(skip)`` (the TFRecord loader, written through into ``cache``) unless the cache is
    already complete, the others from the cache.  ``skip`` / ``limit`` count batches over the
    concatenated epochs (resume / agreed step counts)."""
    left = None if limit is None else int(limit)
    skip = int(skip)
    for ep in range(int(num_epochs)):
        if left is not None and left <= 0:
            return
        if cache.complete():
            n = cache.num_batches()
            if skip >= n:
                skip -= n
                continue
            src = cache.groups(size, hold=hold, skip=skip, limit=left)
            took = min(n - skip, left) if left is not None else n - skip
            skip = 0
        else:
            if skip:  # cannot write a partial epoch: read this epoch from the TFRecords without caching
                src, took = make_groups(skip, left), None
                skip = 0
            else:
                src, took = cache.write_through(make_groups(0, None)), None
        got = 0
        for g in src:
            k = int(g[0].shape[0]) if g[0].dim() == 3 else 1
            cut = left is not None and got + k > left
            if cut:
                g = tuple(t[: left - got] for t in g)
                k = left - got
            if k > 0:
                got += k
                yield g
            if cut or (left is not None and got >= left):
                break
        if hasattr(src, "close"):
            src.close()  # a write-through stopped inside its epoch leaves no complete cache
        if left is not None:
            left -= got
