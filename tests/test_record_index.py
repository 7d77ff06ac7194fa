"""Persistent record index (csrc/io/record_index.h) and the loader's index / raw modes.

The index lets a record-sharded rank (the reference's ``dataset.shard(size, rank)``, HVD:132-133)
read only its own records; raw mode hands undecoded Example payloads to the GPU parser.  Every
mode must yield exactly the batches of the legacy framing walk + host decode."""
import os

import numpy as np
import pytest
import torch

from rocfm.data import tfrecord as T
from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.ops import io


def _files(tmp_path, n=3, per=1000, seed=0):
    out = []
    for i in range(n):
        p = str(tmp_path / f"tr{i}.tfrecords")
        write_synthetic_tfrecord(p, per + 37 * i, 50000, 39, seed=seed + i)
        out.append(p)
    return out


def _batches(files, use_index, **kw):
    ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=3, pin_memory=False, **kw)
    ds.kw["use_index"] = use_index
    return [tuple(x.clone() for x in b) for b in ds]


def test_writer_saves_a_valid_index(tmp_path):
    f = _files(tmp_path, 1)[0]
    assert os.path.exists(f + ".rfidx")
    n, mx = io().index_info(f)
    assert n == 1000 and n == io().count_records(f)
    assert mx == max(io().scan_file(f, True, False)[2])


@pytest.mark.parametrize("shards", [1, 3])
def test_index_mode_equals_legacy_walk(tmp_path, shards):
    files = _files(tmp_path)
    for idx in range(shards):
        kw = dict(shard_count=shards, shard_index=idx, num_epochs=2)
        a = _batches(files, True, **kw)
        b = _batches(files, False, **kw)
        assert len(a) == len(b) > 0
        for x, y in zip(a, b):
            for u, v in zip(x, y):
                assert torch.equal(u, v)


def test_stale_index_is_rebuilt_and_missing_index_is_written(tmp_path):
    files = _files(tmp_path, 1)
    f = files[0]
    ref = _batches(files, False)
    os.remove(f + ".rfidx")
    ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=2, pin_memory=False)
    got = [tuple(x.clone() for x in b) for b in ds]
    assert ds.loader.index_builds == 1 and os.path.exists(f + ".rfidx")
    assert all(torch.equal(u, v) for x, y in zip(got, ref) for u, v in zip(x, y))
    ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=2, pin_memory=False)
    list(ds)
    assert ds.loader.index_loads == 1 and ds.loader.index_builds == 0
    # the data file changes (append 10 records): the saved index no longer matches → rebuilt
    L, I, V = T.decode_file(f, 39)
    T.write_tfrecord(f, L[:10].numpy(), I[:10].numpy(), V[:10].numpy(), append=True)
    assert io().index_info(f) is None
    ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=2, pin_memory=False)
    n = sum(int(b[0].shape[0]) for b in ds)
    assert ds.loader.index_builds == 1 and n == (1010 // 64) * 64


def test_index_dir_env(tmp_path, monkeypatch):
    files = _files(tmp_path, 1)
    os.remove(files[0] + ".rfidx")
    d = tmp_path / "idx"
    d.mkdir()
    monkeypatch.setenv("ROCFM_INDEX_DIR", str(d))
    assert io().index_path(files[0]).startswith(str(d))
    assert io().build_index(files[0], True) == 1000
    assert len(os.listdir(d)) == 1 and not os.path.exists(files[0] + ".rfidx")
    assert io().index_info(files[0])[0] == 1000


def test_corrupt_data_crc_in_dropped_remainder_is_reported(tmp_path):
    """A record that no batch decodes (the drop_remainder tail) is still CRC-checked, like tf.data
    which reads every record before batch() drops the tail."""
    f = str(tmp_path / "tr.tfrecords")
    write_synthetic_tfrecord(f, 64 * 3 + 5, 50000, 39, seed=3)
    lens = io().scan_file(f, True, False)[2]
    off = sum(16 + x for x in lens[:64 * 3 + 2]) + 12 + 20  # inside record 194's payload
    with open(f, "r+b") as fh:
        fh.seek(off)
        b = fh.read(1)
        fh.seek(off)
        fh.write(bytes([b[0] ^ 0x5A]))
    io().build_index(f, False)  # framing is intact: the index stays valid
    ds = T.TFRecordDataset([f], 39, 64, 50000, num_threads=2, pin_memory=False)
    with pytest.raises(RuntimeError, match="data CRC.*remainder"):
        list(ds)


@pytest.mark.parametrize("shards", [1, 2])
def test_raw_groups_decode_to_the_host_batches(tmp_path, shards):
    files = _files(tmp_path, 2, per=700)
    for idx in range(shards):
        ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=2, pin_memory=False, shard_count=shards,
                               shard_index=idx)
        ref = [tuple(x.clone() for x in g) for g in ds.groups(4, hold=2)]
        ds = T.TFRecordDataset(files, 39, 64, 50000, num_threads=2, pin_memory=False, shard_count=shards,
                               shard_index=idx)
        raw = []
        for g in ds.raw_groups(4, hold=2):
            assert g.bytes.shape[1] % 16 == 0 and int(g.offs[0, 0]) == 0
            raw.append(g.decode_host(39, 50000))
        assert len(raw) == len(ref)
        for x, y in zip(raw, ref):
            for u, v in zip(x, y):
                assert torch.equal(u, v)


def test_raw_mode_rejects_skip_bad_and_stream(tmp_path):
    files = _files(tmp_path, 1)
    with pytest.raises(ValueError):
        next(iter(T.TFRecordDataset(files, 39, 64, skip_bad=True, pin_memory=False).raw_groups(4)))
    with pytest.raises(ValueError):
        next(iter(T.TFRecordDataset(files, 39, 64, stream_mode=True, pin_memory=False).raw_groups(4)))


def test_rewritten_file_with_a_stale_index_fails_loudly_without_crc_checks(tmp_path):
    """A file rewritten in place with the same size and mtime keeps a sidecar index whose interior
    offsets are wrong (only the size, the mtime and both framing ends are checked on load); with
    verify_crc off the loader still checks every frame's length CRC, so it raises instead of
    decoding garbage."""
    import shutil

    f = str(tmp_path / "tr.tfrecords")
    small = np.arange(1, 40).reshape(1, 39)           # 1-byte varints
    large = np.arange(200, 239).reshape(1, 39)        # 2-byte varints
    vals = np.ones((1, 39), np.float32)
    lab = np.zeros(1, np.float32)

    def write(order):
        for i, ids in enumerate(order):
            T.write_tfrecord(f, lab, ids, vals, append=i > 0)

    write([small, large, small])
    assert io().build_index(f, True) == 3
    st = os.stat(f)
    shutil.copy(f + ".rfidx", str(tmp_path / "old.rfidx"))
    size = os.path.getsize(f)
    write([large, small, small])  # same size, the second frame starts elsewhere
    assert os.path.getsize(f) == size
    shutil.copy(str(tmp_path / "old.rfidx"), f + ".rfidx")
    os.utime(f, ns=(st.st_atime_ns, st.st_mtime_ns))
    assert io().index_info(f) is not None  # the stale sidecar still passes the load checks
    ds = T.TFRecordDataset([f], 39, 1, 50000, num_threads=1, pin_memory=False, verify_crc=False)
    with pytest.raises(RuntimeError, match="TFRecord"):
        list(ds)
