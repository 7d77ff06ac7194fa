"""C++ TFRecord runtime: framing/CRC, Example decoding, loader sharding & batching, libsvm tool.

Golden statistics of the bundled data/val.tfrecords are from SURVEY.md §2.8 (10,000 records,
2,553 positives, ids in 1..117565, first record ids)."""
import os
import struct

import numpy as np
import pytest
import torch

from rocfm.data import tfrecord as T
from rocfm.ops import io

FIRST_IDS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 19, 586, 1079, 12368, 26191, 26341, 27172, 35362, 35613,
             36145, 47521, 51365, 63273, 65964, 66584, 71629, 84088, 84521, 86888, 88279, 88284, 100289, 100301,
             100316, 109930, 109982]


def test_golden_stats_of_bundled_data(ref_data_path):
    L, I, V = T.decode_file(ref_data_path, 39, 117581)
    assert L.shape == (10000,) and I.shape == (10000, 39) and V.shape == (10000, 39)
    assert int(L.sum()) == 2553
    assert int(I.min()) == 1 and int(I.max()) == 117565
    assert I[0].tolist() == FIRST_IDS and float(L[0]) == 1.0
    assert (I[:, :13] == torch.arange(1, 14, dtype=torch.int32)).all()  # numeric fields: fixed ids 1..13
    assert (V[:, 13:] == 1.0).all()
    assert len(torch.unique(I)) == 28116


def test_native_matches_python_oracle(ref_data_path):
    L, I, V = T.decode_file(ref_data_path, 39)
    for k, rec in enumerate(T.read_records(ref_data_path, verify=True)):
        ex = T.parse_example(rec)
        assert ex["ids"] == I[k].tolist()
        assert np.allclose(ex["values"], V[k].numpy())
        assert ex["label"][0] == float(L[k])
        if k == 50:
            break


def test_crc32c_known_vectors():
    m = io()
    assert m.crc32c(b"") == 0
    assert m.crc32c(b"123456789") == 0xE3069283  # standard CRC-32C check value
    assert m.masked_crc32c(b"abc") == T.masked_crc32c_py(b"abc")


def _write(path, n, F=5, seed=0, V=100):
    g = np.random.default_rng(seed)
    ids = g.integers(0, V, (n, F)).astype(np.int64)
    vals = g.random((n, F)).astype(np.float32)
    labels = (g.random(n) < 0.3).astype(np.float32)
    io().write_tfrecord(path, labels, ids, vals, False)
    return labels, ids, vals


def test_writer_roundtrip(tmp_path):
    p = str(tmp_path / "a.tfrecords")
    labels, ids, vals = _write(p, 300)
    L, I, V = T.decode_file(p, 5)
    assert np.array_equal(L.numpy(), labels) and np.array_equal(I.numpy(), ids) and np.array_equal(V.numpy(), vals)
    # the python oracle reads the C++ writer's bytes too
    ex = T.parse_example(next(T.read_records(p, verify=True)))
    assert ex["ids"] == ids[0].tolist()


def test_corrupt_record_fail_and_skip(tmp_path):
    p = str(tmp_path / "c.tfrecords")
    _write(p, 10)
    data = bytearray(open(p, "rb").read())
    (n0,) = struct.unpack("<Q", data[:8])
    data[12 + 5] ^= 0xFF  # corrupt the first record's payload
    open(p, "wb").write(bytes(data))
    with pytest.raises(RuntimeError):
        T.decode_file(p, 5)
    L, _, _ = T.decode_file(p, 5, skip_bad=True)
    assert len(L) == 9


def test_wrong_field_count_is_an_error(tmp_path):
    p = str(tmp_path / "w.tfrecords")
    _write(p, 4, F=5)
    with pytest.raises(RuntimeError, match="decode error"):
        T.decode_file(p, 6)


def _collect(ds):
    out = []
    for ids, vals, labels in ds:
        out.append((ids.clone(), vals.clone(), labels.clone()))
    return out


@pytest.mark.parametrize("threads", [1, 4])
def test_loader_batches_shards_epochs(tmp_path, threads):
    p1, p2 = str(tmp_path / "tr1.tfrecords"), str(tmp_path / "tr2.tfrecords")
    l1, i1, v1 = _write(p1, 250, seed=1)
    l2, i2, v2 = _write(p2, 170, seed=2)
    all_ids = np.concatenate([i1, i2])
    # shard(3, 1) over the concatenated files, batch 16, drop remainder, 2 epochs
    ds = T.TFRecordDataset([p1, p2], 5, 16, num_epochs=2, shard_count=3, shard_index=1, num_threads=threads,
                           num_slots=3, pin_memory=False)
    got = _collect(ds)
    kept = all_ids[1::3]
    nb = len(kept) // 16
    assert len(got) == 2 * nb
    for e in range(2):
        for b in range(nb):
            assert np.array_equal(got[e * nb + b][0].numpy(), kept[b * 16:(b + 1) * 16])
    # no drop_remainder: the tail batch is emitted
    ds = T.TFRecordDataset([p1], 5, 64, drop_remainder=False, pin_memory=False)
    sizes = [len(b[0]) for b in _collect(ds)]
    assert sizes == [64, 64, 64, 58]


def test_loader_shuffle_buffer_is_a_permutation(tmp_path):
    p = str(tmp_path / "tr.tfrecords")
    _, ids, _ = _write(p, 200, seed=3)
    ds = T.TFRecordDataset([p], 5, 10, shuffle_buffer=50, seed=7, pin_memory=False)
    got = torch.cat([b[0] for b in _collect(ds)]).numpy()
    assert got.shape == ids.shape
    assert sorted(map(tuple, got.tolist())) == sorted(map(tuple, ids.tolist()))
    assert not np.array_equal(got, ids)


def test_pipe_mode_stream(tmp_path):
    p = str(tmp_path / "pipe.tfrecords")
    _, ids, _ = _write(p, 40, seed=4)
    fifo = str(tmp_path / "fifo")
    os.mkfifo(fifo)
    import threading

    def feed():
        with open(fifo, "wb") as f:
            f.write(open(p, "rb").read())

    th = threading.Thread(target=feed)
    th.start()
    ds = T.TFRecordDataset([fifo], 5, 8, stream_mode=True, pin_memory=False)
    got = torch.cat([b[0] for b in _collect(ds)]).numpy()
    th.join()
    assert np.array_equal(got, ids)


def test_libsvm_converter_roundtrip(tmp_path):
    src = tmp_path / "tr.libsvm"
    src.write_text("1 1:0.5 2:0.03519 3:1\n0 4:0.25 5:1 6:1\n\n1 7:2 8:3 9:4\n")
    out = str(tmp_path / "tr.tfrecords")
    n = io().convert_libsvm(str(src), out, 2)
    assert n == 3
    L, I, V = T.decode_file(out, 3)
    assert L.tolist() == [1.0, 0.0, 1.0]
    assert I.tolist() == [[1, 2, 3], [4, 5, 6], [7, 8, 9]]
    assert np.allclose(V.numpy(), [[0.5, 0.03519, 1], [0.25, 1, 1], [2, 3, 4]])


def test_discover_files(tmp_path):
    (tmp_path / "a").mkdir()
    for n in ["tr1.tfrecords", "a/tr2.tfrecords", "va.tfrecords", "te.tfrecords", "other.txt"]:
        (tmp_path / n).write_bytes(b"")
    tr = T.discover_files(str(tmp_path), "tr")
    assert [os.path.basename(x) for x in tr] == ["tr2.tfrecords", "tr1.tfrecords"] or len(tr) == 2
    assert len(T.discover_files(str(tmp_path), "va")) == 1 and len(T.discover_files(str(tmp_path), "te")) == 1


def _big(tmp_path, n=30000, seed=5, name="big.tfrecords"):
    """≈9.5 MB of 39-field records: the loader indexes it with ≥2 parallel framing walks."""
    p = str(tmp_path / name)
    labels, ids, vals = _write(p, n, F=39, seed=seed, V=1_000_000)
    assert os.path.getsize(p) >= 8 << 20
    return p, labels, ids, vals


def test_parallel_index_matches_sequential_scan(tmp_path):
    p, labels, ids, vals = _big(tmp_path)
    for threads in (1, 3, 8):
        ds = T.TFRecordDataset([p], 39, 1000, num_threads=threads, pin_memory=False)
        got = _collect(ds)
        assert len(got) == 30
        assert np.array_equal(torch.cat([g[0] for g in got]).numpy(), ids)
        assert np.array_equal(torch.cat([g[2] for g in got]).numpy(), labels)
        assert ds.loader.index_fallbacks == 0
    assert io().count_records(p) == 30000


def test_parallel_index_corruption_falls_back_to_sequential_semantics(tmp_path):
    p, labels, ids, vals = _big(tmp_path)
    data = bytearray(open(p, "rb").read())
    # corrupt a payload byte of a record in the second half (a parallel walk's range)
    off, k = 0, 0
    while off < len(data) * 3 // 4:
        (n,) = struct.unpack("<Q", data[off:off + 8])
        off += 12 + n + 4
        k += 1
    data[off + 12 + 3] ^= 0xFF
    open(p, "wb").write(bytes(data))
    with pytest.raises(RuntimeError):
        _collect(T.TFRecordDataset([p], 39, 1000, num_threads=4, pin_memory=False))
    ds = T.TFRecordDataset([p], 39, 1000, num_threads=4, skip_bad=True, drop_remainder=False, pin_memory=False)
    got = _collect(ds)
    assert ds.loader.index_fallbacks == 0 and ds.bad_records == 1  # a bad data CRC is skipped in parallel
    keep = np.delete(ids, k, axis=0)
    assert np.array_equal(torch.cat([g[0] for g in got]).numpy(), keep)


@pytest.mark.parametrize("threads", [1, 4])
def test_sharded_loader_checks_data_crc_of_its_own_records(tmp_path, threads):
    """Sharded loaders walk the framing only and leave data CRCs to the decoders of the records they
    keep (loader.h): a corrupt record fails the rank whose shard holds it and no other; skip_bad
    keeps the full-walk semantics (the bad record is dropped before sharding)."""
    p, labels, ids, vals = _big(tmp_path)
    data = bytearray(open(p, "rb").read())
    off, k = 0, 0
    while k < 12345:
        (n,) = struct.unpack("<Q", data[off:off + 8])
        off += 12 + n + 4
        k += 1
    data[off + 12 + 3] ^= 0xFF  # record k's payload
    open(p, "wb").write(bytes(data))
    for r in range(3):
        ds = T.TFRecordDataset([p], 39, 1000, shard_count=3, shard_index=r, num_threads=threads, pin_memory=False)
        if r == k % 3:
            with pytest.raises(RuntimeError, match="corrupt data CRC"):
                _collect(ds)
        else:
            got = torch.cat([g[0] for g in _collect(ds)]).numpy()
            assert np.array_equal(got, ids[r::3][: len(got)]) and len(got) == (len(ids[r::3]) // 1000) * 1000
    keep = np.delete(ids, k, axis=0)
    for r in range(3):
        ds = T.TFRecordDataset([p], 39, 1000, shard_count=3, shard_index=r, num_threads=threads, skip_bad=True,
                               drop_remainder=False, pin_memory=False)
        got = torch.cat([g[0] for g in _collect(ds)]).numpy()
        assert np.array_equal(got, keep[r::3]) and ds.bad_records == 1


def test_file_shard_policy(tmp_path):
    files, per = [], []
    for i in range(5):
        f = str(tmp_path / f"tr{i}.tfrecords")
        per.append(_write(f, 40 + 8 * i, seed=30 + i)[1])
        files.append(f)
    for r in range(2):
        ds = T.TFRecordDataset(files, 5, 8, shard_count=2, shard_index=r, shard_policy="file", pin_memory=False)
        got = torch.cat([b[0] for b in _collect(ds)]).numpy()
        want = np.concatenate(per[r::2])
        assert np.array_equal(got, want[: len(want) // 8 * 8])
    with pytest.raises(ValueError, match="at least 6 files"):
        T.TFRecordDataset(files, 5, 8, shard_count=6, shard_index=0, shard_policy="file")
    from rocfm.config import Config
    with pytest.raises(ValueError, match="shard_policy"):
        Config(shard_policy="bytes", field_size=39, feature_size=100).validate()


def test_groups_match_batches_skip_limit_tail(tmp_path):
    p = str(tmp_path / "g.tfrecords")
    _, ids, _ = _write(p, 1000, seed=6)
    ref = torch.tensor(ids[: 1000 // 16 * 16], dtype=torch.int32).view(-1, 16, 5)  # 62 batches
    ds = T.TFRecordDataset([p], 5, 16, num_threads=3, pin_memory=False)
    got = [(g[0].clone(), g[2].clone()) for g in ds.groups(8, hold=2)]
    assert [g[0].shape[0] for g in got] == [8] * 7 + [6]
    assert torch.equal(torch.cat([g[0] for g in got]), ref)
    # skip 5 batches (dropped undecoded by the reader), then at most 20
    got = [g[0].clone() for g in ds.groups(8, skip=5, limit=20)]
    assert [g.shape[0] for g in got] == [8, 8, 4]
    assert torch.equal(torch.cat(got), ref[5:25])
    # drop_remainder=False: the partial tail batch comes alone, 2-D
    ds = T.TFRecordDataset([p], 5, 16, drop_remainder=False, pin_memory=False)
    got = list(ds.groups(8))
    assert got[-1][0].shape == (1000 - 62 * 16, 5)
    assert sum(g[0].shape[0] for g in got[:-1]) == 62


def test_libsvm_cli_sharded(tmp_path):
    """python -m rocfm.tools.libsvm_to_tfrecord with --shards: contiguous shards, input order kept,
    every record decodes to the libsvm line it came from (TOOL:22-61 schema)."""
    import subprocess
    import sys

    lines = []
    for i in range(103):
        feats = " ".join(f"{i * 7 + f}:{(f + 1) * 0.5:g}" for f in range(5))
        lines.append(f"{i % 2} {feats}")
    src = tmp_path / "train.libsvm"
    src.write_text("\n".join(lines) + "\n")
    out = tmp_path / "o" / "tr.tfrecords"
    r = subprocess.run([sys.executable, "-m", "rocfm.tools.libsvm_to_tfrecord", str(src), str(out), "--shards", "4",
                        "--threads", "3"], capture_output=True, text=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert r.returncode == 0, r.stderr
    from rocfm.tools.libsvm_to_tfrecord import shard_paths

    paths = shard_paths(str(out), 4)
    assert [os.path.basename(p) for p in paths] == [f"tr-0000{k}-of-00004.tfrecords" for k in range(4)]
    got = []
    for p in paths:
        L, I, V = T.decode_file(p, 5)
        got += [(float(l), i.tolist(), v.tolist()) for l, i, v in zip(L, I, V)]
    assert len(got) == 103
    for i, (l, ids, vals) in enumerate(got):
        assert l == float(i % 2) and ids == [i * 7 + f for f in range(5)]
        assert vals == [(f + 1) * 0.5 for f in range(5)]
    sizes = [len(T.decode_file(p, 5)[0]) for p in paths]
    assert sizes == [25, 26, 26, 26]


def test_decoded_cache_epochs_equal_loader(tmp_path):
    """rocfm.data.cache: the first pass is written through, later passes (and a later job) read
    the raw memory-mapped cache; over several epochs with skip / limit the batches equal the C++
    loader's multi-epoch stream exactly, and an interrupted first pass leaves no complete cache."""
    import torch

    from rocfm.data.cache import DecodedCache, cached_epochs
    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.data.tfrecord import TFRecordDataset

    files = []
    for i in range(2):
        p = str(tmp_path / f"tr{i}.tfrecords")
        write_synthetic_tfrecord(p, 1500, 5000, 39, seed=i)
        files.append(p)
    B, S, E = 128, 4, 3

    def ds(epochs):
        return TFRecordDataset(files, 39, B, 5000, num_epochs=epochs, shard_count=2, shard_index=1, num_threads=2,
                               pin_memory=False)

    def flat(groups):
        out = []
        for g in groups:
            if g[0].dim() == 2:
                g = tuple(t.unsqueeze(0) for t in g)
            out += [tuple(t[i].clone() for t in g) for i in range(g[0].shape[0])]
        return out

    ref = flat(ds(E).groups(S, hold=2))
    nb = len(ref) // E
    d = str(tmp_path / "cache")
    first = lambda sk, lim: ds(1).groups(S, hold=2, skip=sk, limit=lim)
    # an interrupted first pass (limit inside epoch 1) leaves no complete cache
    part = flat(cached_epochs(DecodedCache.for_dataset(ds(1), d), first, E, S, limit=nb - 2))
    assert len(part) == nb - 2 and not DecodedCache.for_dataset(ds(1), d).complete()
    for skip, limit in ((0, None), (0, None), (nb + 3, 2 * nb - 5)):  # write-through, then from the cache
        dc = DecodedCache.for_dataset(ds(1), d)
        got = flat(cached_epochs(dc, first, E, S, skip=skip, limit=limit))
        exp = ref[skip:] if limit is None else ref[skip:skip + limit]
        assert len(got) == len(exp)
        assert all(all(torch.equal(a, b) for a, b in zip(x, y)) for x, y in zip(got, exp))
        assert dc.complete() and dc.num_batches() == nb


@pytest.mark.parametrize("threads,shards", [(1, 1), (4, 1), (4, 3)])
def test_piecewise_index_matches_decode_file(tmp_path, threads, shards):
    """The loader indexes a file's first 2 MB as its own piece (the decoders start before the whole
    file is walked) and the rest as a second piece: the piece boundary falls inside a record, and
    the batches (every shard, skip, epochs) still equal the whole-file decode in record order."""
    from rocfm.data.synthetic import write_synthetic_tfrecord

    p1, p2 = str(tmp_path / "big.tfrecords"), str(tmp_path / "small.tfrecords")
    write_synthetic_tfrecord(p1, 9000, 50000, 39, seed=3)  # ≈2.8 MB: two pieces
    write_synthetic_tfrecord(p2, 700, 50000, 39, seed=4)
    assert os.path.getsize(p1) > (2 << 20)
    Ls, Is, Vs = zip(*(T.decode_file(p, 39, 50000) for p in (p1, p2)))
    L, I, V = torch.cat(Ls), torch.cat(Is), torch.cat(Vs)
    for r in range(shards):
        ds = T.TFRecordDataset([p1, p2], 39, 256, 50000, num_epochs=2, shard_count=shards, shard_index=r,
                               num_threads=threads, pin_memory=False)
        got = [(ids.clone(), vals.clone(), lab.clone()) for ids, vals, lab in ds]
        sel = torch.arange(r, len(L), shards)
        n = len(sel) // 256 * 256
        exp_i = I[sel][:n].reshape(-1, 256, 39)
        assert len(got) == 2 * len(exp_i)
        for k, (ids, vals, lab) in enumerate(got):
            e = k % len(exp_i)
            assert torch.equal(ids, exp_i[e])
            assert torch.equal(vals, V[sel][:n].reshape(-1, 256, 39)[e])
            assert torch.equal(lab, L[sel][:n].reshape(-1, 256)[e])
