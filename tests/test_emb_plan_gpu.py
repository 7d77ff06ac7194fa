"""The planned step tail (emb_plan.hip + emb_plan_body.h): the side chain's work plan equals its
sequential replica, and training through planned multi-step graphs is bit-identical to the per-step
path (which runs the unplanned body) — split runs included."""
import numpy as np
import pytest
import torch

from rocfm.data.synthetic import SyntheticCriteo
from rocfm.models.deepfm import ModelSpec, init_params
from rocfm.models.fused import FusedDeepFM
from rocfm.ops import reference as R
from rocfm.optim import OptHParams

pytestmark = pytest.mark.gpu


def _keysets():
    g = np.random.default_rng(5)
    out = []
    gen = SyntheticCriteo(1_000_000, 39, seed=1)
    ids, _, _ = gen.batch(1024, "cpu", torch.Generator().manual_seed(1))
    out.append(np.sort(ids.reshape(-1).numpy().astype(np.int64)))  # the bench shape (Zipf + hot runs)
    out.append(np.sort(g.integers(0, 50, 5000)))                    # every run long
    out.append(np.arange(3000))                                      # every entry a head
    out.append(np.zeros(4099, np.int64))                             # one run
    out.append(np.sort(np.r_[np.zeros(700), g.integers(1, 10**6, 2300), np.full(900, 10**6 + 1)]).astype(np.int64))
    return out


@pytest.mark.parametrize("beta,lsplit", [(4, 128), (0, 64), (9, 300)])
def test_emb_plan_kernel_matches_reference(beta, lsplit):
    from rocfm.ops._ext import require_hip

    H = require_hip()
    dev = torch.device("cuda")
    for keys in _keysets():
        n = keys.size
        for nw in (max(1, (n + 255) // 256), (n + 255) // 256 + 37):
            S = 2  # two batch segments: the second one is the same keys (segment offsets checked)
            kd = torch.from_numpy(np.tile(keys, S).astype(np.int32)).to(dev)
            items = torch.full((S, nw, 4), 7, dtype=torch.int32, device=dev)
            slots = torch.zeros(S, nw, 4, dtype=torch.int32, device=dev)
            runs = torch.zeros(S * (n + 1), dtype=torch.int32, device=dev)
            slab_w = H.plan_bounds()[2]
            hslab = torch.full((S, nw, slab_w), -5, dtype=torch.int32, device=dev)
            pp = H.EmbPlanParams()
            pp.skeys, pp.n, pp.S, pp.nw, pp.beta, pp.lsplit = kd.data_ptr(), n, S, nw, beta, lsplit
            pp.runs, pp.items, pp.slots = runs.data_ptr(), items.data_ptr(), slots.data_ptr()
            pp.hslab = hslab.data_ptr()
            H.emb_plan(pp, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            ri, rs = R.emb_plan_reference(keys, nw, beta, lsplit)
            ns = int((ri[:, 3] >= 0).sum())
            for k in range(S):
                np.testing.assert_array_equal(items[k].cpu().numpy(), ri, err_msg=f"n={n} nw={nw}")
                np.testing.assert_array_equal(slots[k, :ns].cpu().numpy(), rs[:ns])
            # the head-key slab: per item its run heads' count, then their keys in order
            head = np.ones(n, bool)
            head[1:] = keys[1:] != keys[:-1]
            hs = hslab.cpu().numpy()
            for k in range(S):
                for j in range(nw):
                    a, b = ri[j, 0], ri[j, 1]
                    hk = keys[a:b][head[a:b]] if b > a else keys[:0]
                    assert hs[k, j, 0] == hk.size, f"n={n} nw={nw} item {j}"
                    np.testing.assert_array_equal(hs[k, j, 1:1 + hk.size], hk.astype(np.int32))
            live = ri[:, 1] > ri[:, 0]
            e = ri[live][:, :2]
            assert e[0, 0] == 0 and e[-1, 1] == n and (e[1:, 0] == e[:-1, 1]).all()  # a partition


def _batch(B, F, V, gen):
    ids = torch.randint(0, V, (B, F), generator=gen, dtype=torch.int64)
    ids[:, :13] = torch.arange(1, 14)  # numeric-style fields: fixed ids in every example (long runs)
    ids[:, 13] = V - 1
    vals = torch.rand(B, F, generator=gen)
    vals[:, 13:] = 1.0
    labels = (torch.rand(B, generator=gen) < 0.3).float()
    return ids.to(torch.int32), vals, labels


def _engine(spec, hp, B, graph, **kw):
    return FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=graph, **kw)


@pytest.mark.parametrize("K,tbl,lsplit,beta,opt", [(10, "f32", "128", "4", "Adam"), (10, "f32", "64", "0", "Adam"),
                                                   (32, "f32", "64", "9", "Adam"), (10, "bf16", "64", "4", "Adam"),
                                                   (32, "f32", "128", "4", "Adagrad")])
def test_planned_tail_equals_per_step(K, tbl, lsplit, beta, opt, monkeypatch):
    """Multi-step graphs with the planned tail (items of equal cost, split runs combined by the last
    arrival) ≡ per-step training (fixed 256-entry chunks with in-workgroup continuation), bitwise,
    on hot-run batches (13 ids in every example) where lsplit = 64 splits many runs."""
    monkeypatch.setenv("ROCFM_EMB_LSPLIT", lsplit)
    monkeypatch.setenv("ROCFM_EMB_BETA", beta)
    spec = ModelSpec(feature_size=5000, field_size=39, embedding_size=K, layers=[64, 32], keep_probs=[0.7, 0.8],
                     l2_reg=1e-3)
    hp = OptHParams(name=opt, lr=2e-3)
    g = torch.Generator().manual_seed(9)
    NB, B = 6, 512
    pool = [_batch(B, 39, 5000, g) for _ in range(NB)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    a = _engine(spec, hp, B, True, table_dtype=tbl)
    b = _engine(spec, hp, B, False, table_dtype=tbl)
    a.attach_pool(ids, vals, labels)
    b.attach_pool(ids, vals, labels)
    a.train_steps(13, 4)
    assert a.m_eplan
    for _ in range(13):
        b.train_step()
    torch.cuda.synchronize()
    a.check()
    assert int((a.m_pitems.view(2, -1, a.m_plan_nw, 4)[..., 3] >= 0).sum()) > 0  # split runs occurred
    assert torch.equal(a.emb, b.emb) and torch.equal(a.dense, b.dense)
    assert all(torch.equal(x, y) for x, y in zip(a.emb_slots, b.emb_slots))
    assert int(a.m_pctr[: a.m_plan_nw].abs().sum()) == 0  # every split run's counter was reset


def test_planned_tail_equals_unplanned_bench_shape(monkeypatch):
    """The bench shape (1M vocab, B = 1024, Zipf + 13 hot ids): planned ≡ ROCFM_EMB_PLAN=0 graphs."""
    spec = ModelSpec(feature_size=1_000_000, field_size=39, embedding_size=10, layers=[128, 64, 32],
                     keep_probs=[0.5, 0.5, 0.5], l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=5e-4)
    gen = SyntheticCriteo(1_000_000, 39, seed=1)
    gg = torch.Generator(device="cuda").manual_seed(1)
    pool = [gen.batch(1024, torch.device("cuda"), gg) for _ in range(6)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]) for i in range(3))
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("ROCFM_EMB_PLAN", flag)
        e = _engine(spec, hp, 1024, True)
        e.attach_pool(ids, vals, labels)
        e.train_steps(12, 4)
        torch.cuda.synchronize()
        assert e.m_eplan == (flag == "1")
        e.check()
        outs.append((e.emb.clone(), e.dense.clone(), e.emb_slots[1].clone()))
        del e
    assert all(torch.equal(x, y) for x, y in zip(*outs))
