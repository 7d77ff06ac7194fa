"""Device-side Example parsing (csrc/kernels/decode.hip) against the host decoder.

The host decoder (csrc/io/tfrecord.cpp decode_example, itself checked against the pure-Python
oracle on the bundled data) is the reference: every record must give the same status, and on
success the same ids / values / label bit for bit.  Then a streamed training run fed undecoded
batches must equal the same run fed host-decoded batches."""
import struct

import numpy as np
import pytest
import torch

from rocfm.data import tfrecord as T
from rocfm.ops import io
from rocfm.ops.decode import decode_on_device, pack_payloads

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _vi(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(fno, body):
    return _vi(fno << 3 | 2) + _vi(len(body)) + body


def _floats(vals, packed=True):
    if packed:
        return _ld(1, struct.pack(f"<{len(vals)}f", *vals))
    return b"".join(_vi(1 << 3 | 5) + struct.pack("<f", v) for v in vals)


def _ints(vals, packed=True):
    if packed:
        return _ld(1, b"".join(_vi(v) for v in vals))
    return b"".join(_vi(1 << 3 | 0) + _vi(v) for v in vals)


def _example(entries, extra=b""):
    """entries: [(key, feature_kind, list_body)] → serialized Example (map entry order as given)."""
    feats = b""
    for key, kind, body in entries:
        feats += _ld(1, _ld(1, key.encode()) + _ld(2, _ld(kind, body)))
    return _ld(1, feats) + extra


def _host(payload, F, max_id):
    st, lab, ids, vals = io().decode_example(payload, F, max_id)
    return st, lab, ids, vals


def _check(payloads, F, max_id, B=None):
    B = B or len(payloads)
    raw, offs, n = pack_payloads(payloads, B)
    ids, vals, labels, err = decode_on_device(raw, offs, n, B, F, DEV, max_id)
    ids, vals, labels = ids.cpu(), vals.cpu(), labels.cpu()
    first_bad = None
    for i, p in enumerate(payloads):
        k, r = divmod(i, B)
        st, lab, hi, hv = _host(p, F, max_id)
        if st == 0:
            assert torch.equal(ids[k, r], torch.from_numpy(hi)), (i, ids[k, r], hi)
            assert torch.equal(vals[k, r].view(torch.int32), torch.from_numpy(hv).view(torch.int32)), i
            assert float(labels[k, r]) == lab, i
        else:
            assert (ids[k, r] == 0).all() and (vals[k, r] == 0).all() and float(labels[k, r]) == 0.0, i
            first_bad = first_bad or (st, k, r)
    e = err.cpu().tolist()
    if first_bad is None:
        assert e[0] == 0, e
    else:
        assert e[0] != 0  # the first failing record by arrival order may be any failing one
        st, lab, _, _ = _host(payloads[e[1] * B + e[2]], F, max_id)
        assert st == e[0], (e, st)


def test_bundled_data_device_parse_equals_host(ref_data_path):
    recs = list(T.read_records(ref_data_path))
    B = 1000
    _check(recs, 39, 117581, B)


def test_synthetic_raw_groups_equal_host_groups(tmp_path):
    from rocfm.data.synthetic import write_synthetic_tfrecord

    files = []
    for i in range(2):
        files.append(str(tmp_path / f"tr{i}.tfrecords"))
        write_synthetic_tfrecord(files[-1], 3000, 1000000, 39, seed=i)
    ds = T.TFRecordDataset(files, 39, 256, 1000000, num_threads=2, pin_memory=True)
    ref = [tuple(x.clone() for x in g) for g in ds.groups(8, hold=2)]
    ds = T.TFRecordDataset(files, 39, 256, 1000000, num_threads=2, pin_memory=True)
    got = []
    for g in ds.raw_groups(8, hold=2):
        ids, vals, labels, err = decode_on_device(g.bytes, g.offs, g.n, 256, 39, DEV, 1000000)
        assert int(err[0]) == 0
        got.append((ids.cpu(), vals.cpu(), labels.cpu()))
    assert len(got) == len(ref)
    for x, y in zip(got, ref):
        for u, v in zip(x, y):
            assert torch.equal(u, v)


def test_wire_format_variants_and_errors():
    F = 5
    rng = np.random.default_rng(0)
    ids = [int(x) for x in rng.integers(0, 2000000, F)]
    vals = [float(np.float32(x)) for x in rng.normal(size=F)]
    good = [("label", 2, _floats([1.0])), ("ids", 3, _ints(ids)), ("values", 2, _floats(vals))]
    cases = [
        _example(good),
        _example(good[::-1]),  # map entries in another order
        _example([("label", 2, _floats([0.0], False)), ("ids", 3, _ints(ids, False)), ("values", 2, _floats(vals, False))]),
        _example([("label", 3, _ints([1]))] + good[1:]),  # int64 label
        _example([("other", 2, _floats([9.0] * 40))] + good + [("zzzzzzzzzzzzzzzzzzzz", 3, _ints([5]))]),
        _example(good, extra=_vi(2 << 3 | 0) + _vi(77) + _vi(3 << 3 | 5) + b"\0\0\0\0"),  # unknown Example fields
        _example(good[:2] + [("values", 2, _floats([0.5] * F)), ("values", 2, _floats(vals))]),  # last one wins
        _example([("label", 2, _floats([1.0])), ("ids", 1, _ld(1, b"abc")), ("values", 2, _floats(vals))]),  # bytes_list: missing ids
        _example(good[:1] + [("ids", 3, _ints(ids[:F - 1]))] + good[2:]),  # wrong length
        _example(good[:1] + [("ids", 3, _ints(ids + [7]))] + good[2:]),  # too long
        _example(good[:1] + [("ids", 3, _ints([ids[0], 2000000] + ids[2:]))] + good[2:]),  # id >= max_id
        _example(good[:1] + [("ids", 3, _ints([-3] + ids[1:]))] + good[2:]),  # negative (10-byte varint)
        _example(good[:2]),  # missing values
        _example(good)[:-3],  # truncated
        b"\x0a\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01",  # runaway length varint
        b"",
    ]
    _check(cases, F, 2000000, B=len(cases))
    _check([c for c in cases[:7]], F, 2000000)  # all-valid batch: no error flagged


def test_keys_and_long_records_from_global_memory():
    """Records too long for the LDS stage (> 512 B on average) are parsed from global memory."""
    F = 100
    rng = np.random.default_rng(1)
    pay = []
    for r in range(70):
        ids = [int(x) for x in rng.integers(0, 1 << 30, F)]
        vals = [float(np.float32(x)) for x in rng.normal(size=F)]
        pay.append(_example([("label", 2, _floats([float(r % 2)])), ("ids", 3, _ints(ids)),
                             ("values", 2, _floats(vals))], extra=_ld(9, b"x" * 400)))
    assert min(len(p) for p in pay) > 512
    _check(pay, F, 0, B=70)


def test_train_stream_raw_equals_host_decoded(tmp_path):
    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    V, B = 100000, 256
    files = []
    for i in range(2):
        files.append(str(tmp_path / f"tr{i}.tfrecords"))
        write_synthetic_tfrecord(files[-1], 5000, V, 39, seed=i)
    spec = ModelSpec(V, 39, 10, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4)
    out = []
    for raw in (False, True):
        eng = FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, DEV, params=init_params(spec, 0))
        ds = T.TFRecordDataset(files, 39, B, V, num_threads=2, num_epochs=2)
        src = ds.raw_groups(8, hold=2) if raw else ds.groups(8, hold=2)
        n = eng.train_stream(src, 8, hold=2)
        torch.cuda.synchronize()
        eng.check()
        out.append((n, eng.emb.clone(), eng.dense.clone(), eng.batch_loss()))
    assert out[0][0] == out[1][0] == 2 * (10000 // B)
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


def test_train_stream_raises_on_a_malformed_record(tmp_path):
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    V, B, F = 5000, 64, 39
    rng = np.random.default_rng(2)
    p = str(tmp_path / "tr.tfrecords")
    labels = rng.integers(0, 2, 64 * 20).astype(np.float32)
    ids = rng.integers(0, V, (64 * 20, F))
    ids[64 * 9 + 3, 7] = V + 5  # out of range in batch 9, record 3
    T.write_tfrecord(p, labels, ids, rng.normal(size=(64 * 20, F)).astype(np.float32))
    spec = ModelSpec(V, F, 10, [64, 32], [1.0, 1.0], l2_reg=1e-4)
    eng = FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, DEV, params=init_params(spec, 0))
    ds = T.TFRecordDataset([p], F, B, V, num_threads=2)
    with pytest.raises(RuntimeError, match="batch 9 record 3.*id out of range"):
        eng.train_stream(ds.raw_groups(4, hold=2), 4, hold=2)
        torch.cuda.synchronize()


def test_malformed_record_never_trains(tmp_path):
    """A malformed record halts every step the side chain prepares once the parser has flagged it
    (optim.h kHaltStepBit): the engine ends bitwise equal to a clean run over the batches of the
    graphs prepared before the flag — 4 or 8 steps here, by copy-stream timing — never past the
    bad batch (index 9), and its optimizer slots did not move in the halted steps."""
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    V, B, F, S = 5000, 64, 39, 4
    rng = np.random.default_rng(3)
    labels = rng.integers(0, 2, B * 20).astype(np.float32)
    ids = rng.integers(0, V, (B * 20, F))
    vals = rng.normal(size=(B * 20, F)).astype(np.float32)
    clean = str(tmp_path / "clean.tfrecords")
    T.write_tfrecord(clean, labels, ids, vals)
    bad_ids = ids.copy()
    bad_ids[B * 9 + 3, 7] = V + 5  # batch 9, record 3
    bad = str(tmp_path / "bad.tfrecords")
    T.write_tfrecord(bad, labels, bad_ids, vals)
    spec = ModelSpec(V, F, 10, [64, 32], [0.5, 0.5], l2_reg=1e-4)

    def engine():
        return FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, DEV, params=init_params(spec, 0))

    def state(e):
        return [e.emb.clone(), e.dense.clone()] + [s.clone() for s in e.emb_slots + e.dense_slots]

    e = engine()
    with pytest.raises(RuntimeError, match="batch 9 record 3.*id out of range"):
        e.train_stream(T.TFRecordDataset([bad], F, B, V, num_threads=2).raw_groups(S, hold=2), S, hold=2)
        torch.cuda.synchronize()
        e.check()
    torch.cuda.synchronize()
    got = state(e)
    matches = []
    for n in (4, 8):
        r = engine()
        done = r.train_stream(T.TFRecordDataset([clean], F, B, V, num_threads=2).raw_groups(S, hold=2, limit=n), S,
                              hold=2)
        torch.cuda.synchronize()
        assert done == n
        matches.append(all(torch.equal(x, y) for x, y in zip(got, state(r))))
    assert any(matches), "the engine state matches no clean prefix of the stream"


def test_estimator_writes_no_checkpoint_after_a_malformed_record(tmp_path):
    """save_checkpoints_steps=1 on a stream with a malformed record in batch 9: the job fails, and
    no checkpoint at or past the bad batch's step exists (state_dict checks the parser first)."""
    from rocfm import checkpoint as ckpt
    from rocfm.config import parse_flags
    from rocfm.estimator import Estimator

    V, B, F = 5000, 64, 39
    rng = np.random.default_rng(4)
    d = tmp_path / "data"
    d.mkdir()
    ids = rng.integers(0, V, (B * 24, F))
    ids[B * 9 + 3, 7] = V + 5
    T.write_tfrecord(str(d / "tr.tfrecords"), rng.integers(0, 2, B * 24).astype(np.float32), ids,
                     rng.normal(size=(B * 24, F)).astype(np.float32))
    md = str(tmp_path / "m")
    cfg = parse_flags(["--feature_size", str(V), "--field_size", str(F), "--embedding_size", "10",
                       "--deep_layers", "64,32", "--dropout", "1.0,1.0", "--batch_size", str(B), "--training_data_dir", str(d),
                       "--model_dir", md, "--engine", "fused", "--save_checkpoints_steps", "1",
                       "--save_checkpoints_secs", "0", "--keep_checkpoint_max", "100", "--log_steps", "0"])
    est = Estimator(cfg)
    with pytest.raises(RuntimeError, match="id out of range"):
        est.train([str(d / "tr.tfrecords")], num_epochs=1)
    prefix = ckpt.latest_checkpoint(md)
    assert prefix is None or ckpt.checkpoint_step(prefix) <= 9, prefix


def test_decode_lds_gate():
    """The parser's LDS stage fits every schema up to 192 fields on gfx950 (160 KiB opt-in); wider
    ones are refused before any launch (the Estimator then parses on the host)."""
    from rocfm.ops import hip

    H = hip()
    assert H.decode_fits(39) and H.decode_fits(192)
    assert not H.decode_fits(193) and not H.decode_fits(0)
    assert H.decode_lds_bytes(192) <= 160 * 1024
