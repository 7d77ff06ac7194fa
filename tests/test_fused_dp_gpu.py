"""Fused data-parallel step (2 ranks sharing one GPU over gloo) ≡ single-GPU step on the union batch."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


_LR = {"Adam": 1e-3, "Momentum": 0.02, "GD": 0.05}


def _cfg(opt="Momentum"):
    """Momentum by default: a linear optimizer, so DP ≡ single differs only by fp32 summation order
    and the comparison is element-tight (``_assert_tight``); Adam turns last-bit differences on
    ≈0-gradient rows into lr-sized steps and keeps one loose smoke case."""
    from rocfm.models.deepfm import ModelSpec
    from rocfm.optim import OptHParams

    spec = ModelSpec(feature_size=4000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)
    return spec, OptHParams(name=opt, lr=_LR[opt])


def _assert_tight(got, exp, rtol=1e-5, atol=1e-7):
    d = (got.float().cpu() - exp.float().cpu()).abs()
    lim = atol + rtol * exp.float().cpu().abs()
    bad = d > lim
    assert not bad.any(), (int(bad.sum()), d.max().item(), (d - lim).max().item())


def _batches(B, n, seed):
    from rocfm.data.synthetic import SyntheticCriteo

    g = torch.Generator().manual_seed(seed)
    gen = SyntheticCriteo(4000, 39, seed=seed)
    return [gen.batch(B, "cpu", g) for _ in range(n)]


def _worker(rank, world, port, mode, out_path, exchange="rccl", steps=3, spg=0, update=None, push="1",
            opt="Momentum", shadow=0, fault=""):
    # shadow: validated (collective-shadowed) first steps, 0 = off (the equivalence tests keep
    # their multi-step graph coverage); fault: ROCFM_FAULT of the validation tests
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), ROCFM_DP_PUSH=push, ROCFM_SHADOW_STEPS=str(shadow),
                      ROCFM_FAULT=fault)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.dp import FusedDataParallel

    spec, hp = _cfg(opt)
    B = 64
    update = update or ("exact" if mode == "dense_dp" else "sparse")
    eng = FusedDataParallel(spec, hp, B, torch.device("cuda", 0), params=init_params(spec, 3),
                            embedding_update=update, mode=mode,
                            use_graph=spg > 0, exchange=exchange)
    assert eng.exchange == exchange or mode == "dense_dp", eng.exchange
    # p2p dp: the tail's producers push into the peers' slots when forced (ranks share this GPU)
    want_fused = exchange == "p2p" and mode == "dp" and os.environ.get("ROCFM_DP_PUSH") == "1"
    assert eng.fused_push == want_fused, (eng.fused_push, want_fused)
    batches = _batches(world * B, steps, 11)
    pool = [(b[0][rank * B:(rank + 1) * B], b[1][rank * B:(rank + 1) * B], b[2][rank * B:(rank + 1) * B])
            for b in batches]
    eng.attach_pool(torch.stack([x[0] for x in pool]).cuda(), torch.stack([x[1] for x in pool]).cuda(),
                    torch.stack([x[2] for x in pool]).cuda())
    if spg:
        eng.train_steps(steps, spg)  # multi-step graphs (the p2p push is captured; gloo is not)
    else:
        for _ in range(steps):
            eng.train_step()
    torch.cuda.synchronize()
    eng.check(replicas=False)
    consistent = eng.verify_replicas()
    diverged = False
    try:
        eng.check()
    except RuntimeError as exc:
        diverged = "replicas diverged" in str(exc)
    if rank == 0:
        torch.save({"emb": eng.emb.cpu(), "dense": eng.dense.cpu(), "slots": [x.cpu() for x in eng.emb_slots],
                    "shadow": eng.shadow.status, "exchange": eng.exchange, "consistent": consistent,
                    "diverged": diverged, "merge_plan": bool(getattr(eng, "m_plan", False))}, out_path)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,exchange,steps,spg,update", [
    ("dp", "rccl", 3, 0, "sparse"), ("dense_dp", "rccl", 3, 0, "exact"), ("dp", "p2p", 3, 0, "sparse"),
    ("dp", "p2p", 11, 4, "sparse"), ("dp", "p2p", 3, 0, "exact"), ("dp", "p2p", 11, 4, "exact")])
def test_fused_dp_equals_single_gpu_union_batch(tmp_path, mode, exchange, steps, spg, update):
    """exchange=rccl runs the backend's collective (gloo here); p2p the IPC push kernel.  dp+exact
    merges the sparse exchange into the dense gradient table, then updates the whole table."""
    _check_dp_vs_single(tmp_path, 2, mode, exchange, steps, spg, update)


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_fused_dp_world4_p2p_graphs(tmp_path, update):
    """4 ranks on one GPU: the p2p push fans out to 3 peers and the merge sums 4 rank lists (the
    directory-narrowed search merge, SEARCH_DIR_MAX_W), through multi-step graphs."""
    _check_dp_vs_single(tmp_path, 4, "dp", "p2p", 11, 4, update)


@pytest.mark.parametrize("world,spg", [(2, 0), (4, 4)])
def test_fused_dp_p2p_unfused_push(tmp_path, world, spg):
    """ROCFM_DP_PUSH=0: the tail writes the local send buffer and the push launch copies all of it
    (the path before producer-side pushing) ≡ the single-GPU union batch."""
    _check_dp_vs_single(tmp_path, world, "dp", "p2p", 11 if spg else 3, spg, "sparse", push="0")


def test_fused_dp_adam_smoke(tmp_path):
    """Adam through the p2p exchange and multi-step graphs: the loose comparison."""
    _check_dp_vs_single(tmp_path, 2, "dp", "p2p", 11, 4, "sparse", opt="Adam")


@pytest.mark.parametrize("world,push", [(2, "1"), (4, "0")])
def test_dp_shadow_exchange_validates_p2p(tmp_path, world, push):
    """Self-validation: the first 8 steps shadow the p2p all-gather with the collective and compare
    bitwise (status ok, p2p kept), then multi-step graphs; replica digests agree and the result is
    the single-GPU one."""
    dp = _check_dp_vs_single(tmp_path, world, "dp", "p2p", 13, 4, "sparse", push=push, shadow=8)
    assert dp["shadow"] == "ok" and dp["exchange"] == "p2p" and dp["consistent"] and not dp["diverged"], dp


def test_dp_shadow_exchange_catches_corrupt_push(tmp_path):
    """ROCFM_FAULT=corrupt_push:1: rank 1 sees one flipped word per p2p exchange; the shadow
    detects it, every rank falls back to RCCL (agreed), the validated steps consumed the
    collective's data, so the replicas agree and the result is still the single-GPU one."""
    dp = _check_dp_vs_single(tmp_path, 2, "dp", "p2p", 13, 4, "sparse", shadow=8, fault="corrupt_push:1")
    assert dp["shadow"] == "mismatch" and dp["exchange"] == "rccl" and dp["consistent"], dp


def test_dp_replica_check_catches_divergence(tmp_path):
    """ROCFM_FAULT=corrupt_replica:1: one rank's MLP drifts; the collective digest check fails on
    every rank (check() raises)."""
    dp = _check_dp_vs_single(tmp_path, 2, "dp", "p2p", 3, 0, "sparse", fault="corrupt_replica:1", compare=False)
    assert not dp["consistent"] and dp["diverged"], dp


def _check_dp_vs_single(tmp_path, world, mode, exchange, steps, spg, update, push="1", opt="Momentum", shadow=0,
                        fault="", compare=True):
    # ranks share this GPU, where the fused push is off by default: the workers force it (small
    # batches keep the spinning producers from starving a peer) unless the copy push is asked for
    out = str(tmp_path / "dp.pt")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out, exchange, steps, spg, update, push, opt, shadow,
                                      fault), nprocs=world, join=True, start_method="spawn")
    dp = torch.load(out, weights_only=True)
    if not compare:
        return dp
    assert dp["consistent"] and not dp["diverged"], dp
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM

    spec, hp = _cfg(opt)
    single = FusedDeepFM(spec, hp, 64 * world, torch.device("cuda"), params=init_params(spec, 3), use_graph=False,
                         embedding_update=update)
    batches = _batches(64 * world, steps, 11)
    single.attach_pool(torch.stack([b[0] for b in batches]).cuda(), torch.stack([b[1] for b in batches]).cuda(),
                       torch.stack([b[2] for b in batches]).cuda())
    for _ in range(steps):
        single.train_step()
    torch.cuda.synchronize()
    if opt != "Momentum":
        # rank-partial sums reorder fp32 additions; Adam amplifies that for near-zero gradients
        # (m/√v), so the tolerance grows with the number of steps
        atol = 2e-5 if steps <= 3 else 1e-4
        torch.testing.assert_close(dp["dense"], single.dense.cpu(), rtol=2e-3, atol=atol)
        torch.testing.assert_close(dp["emb"], single.emb.cpu(), rtol=2e-3, atol=atol)
        return dp
    _assert_tight(dp["dense"], single.dense)
    _assert_tight(dp["emb"], single.emb)
    for got, exp in zip(dp["slots"], single.emb_slots):  # the momentum accumulators too
        _assert_tight(got, exp)
    return dp


def test_fused_dp_world8_rehearsal(tmp_path):
    """Eight ranks on one GPU (the node's rank count): the push fans out to 7 peers (the copy push:
    eight ranks' spinning producers would compete for one GPU's CUs), the merge takes the
    plan-ahead path DP runs from PLAN_MIN_W ranks (the ids exchanged and the plan built on the side
    chain), multi-step graphs; ≡ the single-GPU union batch, replicas bit-identical."""
    _check_dp_vs_single(tmp_path, 8, "dp", "p2p", 11, 4, "sparse", push="0")


def test_fused_dp_world8_rehearsal_node_default(tmp_path, monkeypatch):
    """Eight ranks on one GPU in the 8-GPU node's DEFAULT combination: the fused producer push (every
    rank's tail stores its gradients straight into the 7 peers' receive slots) together with the
    plan-ahead merge (PLAN_MIN_W ≤ 8), at 64 examples per rank so that the spinning producers of
    eight processes cannot starve a lagging peer of CUs; ≡ the single-GPU union batch."""
    from rocfm.parallel.dp import PLAN_MIN_W

    assert PLAN_MIN_W <= 8
    monkeypatch.setenv("ROCFM_MERGE", "auto")
    dp = _check_dp_vs_single(tmp_path, 8, "dp", "p2p", 11, 4, "sparse", push="1")
    assert dp["merge_plan"]


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_fused_dp_world4_direct_maps(tmp_path, monkeypatch, update):
    """The position-map merge (scatter + apply launches) that DP runs beyond SEARCH_DIR_MAX_W ranks
    (the 8-GPU node), forced at 4 ranks (ROCFM_MERGE=direct), multi-step graphs and the p2p push ≡
    the single-GPU union batch."""
    monkeypatch.setenv("ROCFM_MERGE", "direct")
    _check_dp_vs_single(tmp_path, 4, "dp", "p2p", 11, 4, update)


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_fused_dp_world4_hash_merge(tmp_path, monkeypatch, update):
    """The O(W·cap) step-tagged hash merge (ROCFM_MERGE=hash; what 1B-row vocabularies use) through
    4 ranks, multi-step graphs and the p2p push ≡ the single-GPU union batch."""
    monkeypatch.setenv("ROCFM_MERGE", "hash")
    _check_dp_vs_single(tmp_path, 4, "dp", "p2p", 11, 4, update)


@pytest.mark.parametrize("world,update", [(2, "sparse"), (4, "sparse"), (4, "exact")])
def test_fused_dp_plan_merge(tmp_path, monkeypatch, world, update):
    """The plan-ahead merge (ROCFM_MERGE=plan; the default from PLAN_MIN_W ranks): every rank's
    unique ids of the next graph's batches go over a p2p exchange of their own on the side chain,
    where every rank builds the union + positions plan; the step merges by the plan — multi-step
    graphs ≡ the single-GPU union batch, replicas bit-identical."""
    monkeypatch.setenv("ROCFM_MERGE", "plan")
    _check_dp_vs_single(tmp_path, world, "dp", "p2p", 11, 4, update)


@pytest.mark.parametrize("merge", ["direct", "hash"])
@pytest.mark.parametrize("mode,upd", [("dp", "sparse"), ("dense_dp", "exact"), ("dp", "exact")])
def test_dp_multistep_graphs_world1_equal_single(mode, upd, merge, monkeypatch):
    """Single-process DP (no process group: the exchange is a copy) through the multi-step graph
    pipeline (export → exchange → merge / dense apply inside the graph) ≡ the single-GPU engine."""
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.parallel.dp import FusedDataParallel

    monkeypatch.setenv("ROCFM_MERGE", merge)
    spec, hp = _cfg()
    batches = _batches(128, 5, 11)
    pool = [torch.stack([b[i] for b in batches]).cuda() for i in range(3)]
    dp = FusedDataParallel(spec, hp, 128, torch.device("cuda"), params=init_params(spec, 3), embedding_update=upd,
                           mode=mode, use_graph=True)
    one = FusedDeepFM(spec, hp, 128, torch.device("cuda"), params=init_params(spec, 3), embedding_update=upd,
                      use_graph=True)
    dp.attach_pool(*pool)
    one.attach_pool(*pool)
    dp.train_steps(21, 8)
    one.train_steps(21, 8)
    torch.cuda.synchronize()
    assert dp.global_step() == one.global_step() == 21
    # same math; only fma contraction differs between the merge and the single-GPU update
    _assert_tight(dp.emb, one.emb)
    _assert_tight(dp.dense, one.dense)
    dp.check()
    if mode == "dp":
        assert dp.maps.hashed == (merge == "hash")


@pytest.mark.parametrize("kind", ["dp", "rowshard"])
def test_fp8_weight_copies_through_dense_apply(kind):
    """compute_dtype=fp8 where the MLP weights are refreshed by the dense apply (DP merge launch /
    row-shard owner update) instead of the tail's wgrad epilogue: after multi-step graphs the delayed
    per-tensor amax slot holds max |W0| of the current weights, and training tracks the single-GPU
    fp8 engine (same batches)."""
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.parallel.dp import FusedDataParallel
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg()
    batches = _batches(128, 5, 11)
    pool = [torch.stack([b[i] for b in batches]).cuda() for i in range(3)]
    dev = torch.device("cuda")
    if kind == "dp":
        drv = FusedDataParallel(spec, hp, 128, dev, params=init_params(spec, 3), use_graph=True, compute_dtype="fp8")
    else:
        drv = FusedRowShard(spec, hp, 128, dev, params=init_params(spec, 3), use_graph=True, compute_dtype="fp8")
    one = FusedDeepFM(spec, hp, 128, dev, params=init_params(spec, 3), use_graph=True, compute_dtype="fp8")
    drv.attach_pool(*pool)
    one.attach_pool(*pool)
    n = 13
    drv.train_steps(n, 4)
    one.train_steps(n, 4)
    torch.cuda.synchronize()
    e = drv.eng
    L = e.layout
    W0 = e.dense[L.offW[0]: L.offW[0] + L.dims[0] * L.dims[1]]
    assert e.w8[2][n & 1].item() == W0.abs().max().item()
    assert abs(e.w8[3].item() * 448.0 / W0.abs().max().item() - 1) < 0.05
    torch.testing.assert_close(e.dense, one.dense, rtol=2e-3, atol=2e-4)


def _stream_worker(rank, world, port, kind, out_path, shadow):
    """Streamed (host groups → HBM ring → multi-step graphs, exchange inline) vs pool-fed
    training of the same batches, both through the p2p exchange, with a shadow-validation window
    that ends inside the first group."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), ROCFM_DP_PUSH="1", ROCFM_SHADOW_STEPS=str(shadow))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.models.deepfm import init_params

    spec, hp = _cfg("Adam")
    B, n, S = 64, 13, 4
    batches = _batches(world * B, n, 11)
    mine = [(b[0][rank * B:(rank + 1) * B], b[1][rank * B:(rank + 1) * B], b[2][rank * B:(rank + 1) * B])
            for b in batches]

    def build():
        if kind == "rowshard":
            from rocfm.parallel.emb_shard import FusedRowShard

            return FusedRowShard(spec, hp, B, torch.device("cuda", 0), params=init_params(spec, 3), use_graph=True,
                                 exchange="p2p")
        from rocfm.parallel.dp import FusedDataParallel

        return FusedDataParallel(spec, hp, B, torch.device("cuda", 0), params=init_params(spec, 3), use_graph=True,
                                 exchange="p2p")

    res = {}
    a = build()
    groups = [tuple(torch.stack([m[j] for m in mine[i:i + S]]).pin_memory() for j in range(3))
              for i in range(0, n, S)]
    seen = []
    assert a.train_stream(iter(groups), S, after_steps=lambda s, k: seen.append((s, k)), hold=2) == n
    torch.cuda.synchronize()
    a.check()
    res["stream"] = (a.emb.cpu() if kind != "rowshard" else a.eng.emb.cpu(), a.dense.cpu(), a.global_step(),
                     a.shadow.status, sum(k for _, k in seen))
    a.close()
    b = build()
    b.attach_pool(*(torch.stack([m[j] for m in mine]).cuda() for j in range(3)))
    b.train_steps(n, S)
    torch.cuda.synchronize()
    b.check()
    res["pool"] = (b.emb.cpu() if kind != "rowshard" else b.eng.emb.cpu(), b.dense.cpu(), b.global_step(),
                   b.shadow.status, n)
    b.close()
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("dp", 2), ("dp", 4), ("rowshard", 2)])
def test_streamed_multi_gpu_equals_pool_fed(tmp_path, kind, world):
    """Multi-GPU loader path: DP / row-shard train_stream (what the Estimator runs at world > 1)
    ≡ the pool-fed multi-step path, bitwise (Adam), with the shadow window (3 steps) split off the
    first group."""
    out = str(tmp_path / "st.pt")
    mp.start_processes(_stream_worker, args=(world, _free_port(), kind, out, 3), nprocs=world, join=True,
                       start_method="spawn")
    r = torch.load(out, weights_only=True)
    (ea, da, sa, sha, na), (eb, db, sb, shb, nb) = r["stream"], r["pool"]
    assert sa == sb == 13 and na == 13 and sha == shb == "ok", (sa, sb, na, sha, shb)
    assert torch.equal(ea, eb) and torch.equal(da, db)


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_fused_dp_with_dedup(tmp_path, monkeypatch, update):
    """Per-tile dedup (ROCFM_DEDUP=1) under DP: compacted per-rank export lists through the p2p
    exchange and multi-step graphs ≡ the single-GPU engine (Momentum, element-tight)."""
    monkeypatch.setenv("ROCFM_DEDUP", "1")
    _check_dp_vs_single(tmp_path, 2, "dp", "p2p", 11, 4, update)
