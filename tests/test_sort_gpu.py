"""rocfm's segmented stable radix sort (csrc/kernels/seg_sort.hip) against torch.sort(stable=True)
(the plain-PyTorch reference of the same op) and against rocPRIM's radix sort on the multi-step
side chain's composite keys; and one engine run per sort library, bitwise equal."""
import numpy as np
import pytest
import torch

from rocfm.ops import require_hip

pytestmark = pytest.mark.gpu


def _keys(n, bits, gen, hot=True):
    hi = 1 << bits
    k = torch.randint(0, hi, (n,), generator=gen, dtype=torch.int64)
    if hot and n > 8:  # long runs of a few ids (Criteo's numeric fields) and the largest key
        k[torch.randint(0, n, (n // 3,), generator=gen)] = min(7, hi - 1)
        k[: n // 10] = hi - 1
    return k


def _seg_sort(H, keys_i64, nseg, seg_len, bits, first_val=0):
    dev = torch.device("cuda")
    kin = torch.from_numpy(keys_i64.numpy().astype(np.uint32).view(np.int32)).to(dev)
    n = nseg * seg_len
    ko = torch.full((n,), -5, dtype=torch.int32, device=dev)
    vo = torch.full((n,), -5, dtype=torch.int32, device=dev)
    temp = torch.zeros(max(H.seg_sort_temp_bytes(nseg, seg_len, bits), 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    H.seg_sort_iota(temp.data_ptr(), temp.numel(), kin.data_ptr(), ko.data_ptr(), vo.data_ptr(), nseg, seg_len, bits,
                    s, first_val)
    torch.cuda.synchronize()
    return (ko.cpu().numpy().view(np.uint32).astype(np.int64), vo.cpu().numpy().view(np.uint32).astype(np.int64))


def _ref(keys_i64, nseg, seg_len, bits, first_val=0):
    k = keys_i64.reshape(nseg, seg_len)
    mask = (1 << bits) - 1
    order = torch.sort(k & mask, dim=1, stable=True).indices
    ks = torch.gather(k, 1, order)
    vs = order + torch.arange(nseg).unsqueeze(1) * seg_len + first_val
    return ks.reshape(-1).numpy(), vs.reshape(-1).numpy()


@pytest.mark.parametrize("seg_len,bits,first_val", [
    (1, 1, 0), (100, 3, 0), (1024, 8, 0), (1025, 9, 5), (39936, 20, 0), (39936, 13, 11), (100003, 27, 0),
    (5000, 32, 0), (3000, 0, 2)])
def test_seg_sort_single_segment_matches_stable_sort(seg_len, bits, first_val):
    H = require_hip()
    g = torch.Generator().manual_seed(seg_len + bits)
    k = _keys(seg_len, max(bits, 1), g) if bits > 0 else torch.randint(0, 50, (seg_len,), generator=g)
    ko, vo = _seg_sort(H, k, 1, seg_len, bits, first_val)
    rk, rv = _ref(k, 1, seg_len, bits, first_val)
    np.testing.assert_array_equal(ko, rk)
    np.testing.assert_array_equal(vo, rv)


@pytest.mark.parametrize("nseg,seg_len,bits", [(16, 39936, 20), (7, 1500, 11), (33, 2048, 17), (2, 1, 4)])
def test_seg_sort_segments_sorted_on_their_own(nseg, seg_len, bits):
    """Keys carry unrelated bits above ``bits``: every segment is sorted by its low bits only."""
    H = require_hip()
    g = torch.Generator().manual_seed(nseg * 7 + bits)
    k = _keys(nseg * seg_len, bits, g) | (torch.randint(0, 8, (nseg * seg_len,), generator=g) << bits)
    ko, vo = _seg_sort(H, k, nseg, seg_len, bits)
    rk, rv = _ref(k, nseg, seg_len, bits)
    np.testing.assert_array_equal(ko, rk)
    np.testing.assert_array_equal(vo, rv)


def test_seg_sort_equals_rocprim_on_composite_keys():
    """The side chain's composite keys (step << id_bits | id): the segmented sort over the id bits
    is the permutation rocPRIM computes over all S·n keys."""
    H = require_hip()
    dev = torch.device("cuda")
    S, n, idbits = 16, 39936, 20
    g = torch.Generator().manual_seed(3)
    ids = _keys(S * n, idbits, g)
    comp = (torch.arange(S).repeat_interleave(n) << idbits) | ids
    ko, vo = _seg_sort(H, comp, S, n, idbits)
    kin = torch.from_numpy(comp.numpy().astype(np.uint32).view(np.int32)).to(dev)
    rk = torch.zeros(S * n, dtype=torch.int32, device=dev)
    rv = torch.zeros(S * n, dtype=torch.int32, device=dev)
    temp = torch.zeros(max(H.sort_pairs_temp_bytes(S * n, idbits + 4), 16), dtype=torch.uint8, device=dev)
    H.sort_pairs_iota(temp.data_ptr(), temp.numel(), kin.data_ptr(), rk.data_ptr(), rv.data_ptr(), S * n, idbits + 4,
                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(ko, rk.cpu().numpy().view(np.uint32).astype(np.int64))
    np.testing.assert_array_equal(vo, rv.cpu().numpy().view(np.uint32).astype(np.int64))


def test_engine_bitwise_equal_across_sort_libraries(monkeypatch):
    """40 Adam + dropout steps through 16-step graphs (segmented side-chain sort) and per-step
    launches: the same weights with rocPRIM's sort and with rocfm's."""
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    dev = torch.device("cuda")
    spec = ModelSpec(feature_size=20000, field_size=39, embedding_size=10, layers=[128, 64, 32],
                     keep_probs=[0.5, 0.5, 0.5], l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=1e-3)
    B = 256
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 20000, (8, B, 39), generator=g, dtype=torch.int32)
    ids[:, :, :13] = torch.arange(1, 14, dtype=torch.int32)
    vals = torch.rand(8, B, 39, generator=g)
    labels = (torch.rand(8, B, generator=g) < 0.3).float()
    out = {}
    for lib in ("rocprim", "rocfm"):
        monkeypatch.setenv("ROCFM_SORT_LIB", lib)
        for S in (16, 1):
            eng = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 1), seed=3)
            eng.attach_pool(ids.to(dev), vals.to(dev), labels.to(dev))
            eng.train_steps(40, S)
            torch.cuda.synchronize()
            out[(lib, S)] = {k: v.detach().cpu().clone() for k, v in eng.parameters_tf().items()}
            eng.check()
    ref = out[("rocprim", 16)]
    for key, sd in out.items():
        for name, v in ref.items():
            assert torch.equal(sd[name], v), f"{key} {name}"


@pytest.mark.parametrize("V,S", [(100_000_000, 16), (100_000_000, 64), (1_000_000_000, 64)])
def test_wide_vocabulary_streams_through_seg_sort(V, S, tmp_path):
    """100M- and 1B-row vocabularies through the streamed multi-step graphs: the side chain sorts
    every batch on its own 27-30 id bits (seg_sort.hip; plain per-batch keys where S << id_bits no
    longer fits 32 bits — no 64-bit keys, no rocPRIM) and the result is bitwise equal to per-step
    launches (one single-segment sort per step) — table rows and Adam slots of every touched id,
    and every dense parameter and slot."""
    import gc

    from rocfm.data import tfrecord as T
    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.models.deepfm import ModelSpec
    from rocfm.models.fused import FusedDeepFM, sort_lib
    from rocfm.optim import OptHParams

    assert sort_lib() == "rocfm"
    B, F, n = 256, 39, S + 9  # a full graph and a 9-step remainder graph
    f = str(tmp_path / "tr.tfrecords")
    write_synthetic_tfrecord(f, B * n, V, F, seed=4)
    spec = ModelSpec(V, F, 10, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=1e-3)
    dev = torch.device("cuda")
    host = [tuple(x.clone() for x in g) for g in T.TFRecordDataset([f], F, B, V, num_threads=2).groups(8, hold=2)]
    ids = torch.cat([g[0] for g in host]).to(dev)
    vals = torch.cat([g[1] for g in host]).to(dev)
    labels = torch.cat([g[2] for g in host]).to(dev)
    assert ids.shape[0] == n
    touched = torch.unique(ids.reshape(-1)).long()

    def snapshot(e):
        out = [e.emb[touched].cpu(), e.dense.cpu()]
        out += [s[touched].cpu() for s in e.emb_slots] + [s.cpu() for s in e.dense_slots]
        return out

    res = []
    for streamed in (True, False):
        e = FusedDeepFM(spec, hp, B, dev, params=None, seed=7, use_graph=streamed)
        if streamed:
            got = e.train_stream(T.TFRecordDataset([f], F, B, V, num_threads=2).raw_groups(S, hold=2), S, hold=2)
            assert got == n
            assert e.m_plain == ((S << e.m_idbits) > (1 << 32)) and e.m_keys64 is None
        else:
            e.attach_pool(ids, vals, labels)
            for _ in range(n):
                e.train_step()
        torch.cuda.synchronize()
        e.check()
        res.append(snapshot(e))
        del e
        gc.collect()
        torch.cuda.empty_cache()
    for a, b in zip(*res):
        assert torch.equal(a, b)
