"""Row-shard HIP path: routing kernels vs the numpy oracle; the fused row-shard step (1 rank, and 2 or 4
ranks sharing one GPU over gloo) ≡ the single-GPU fused step on the union batch."""
import os
import socket

import numpy as np
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


def _route(ids, W, V, cap):
    from rocfm.ops import require_hip

    H = require_hip()
    n = ids.numel()
    Vs = (V + W - 1) // W
    dev = ids.device
    i32 = dict(dtype=torch.int32, device=dev)
    keys, sk, sv = (torch.zeros(n, **i32) for _ in range(3))
    send = torch.zeros(W * cap, **i32)
    local = torch.zeros(n, **i32)
    skl = torch.zeros(n, **i32)
    counts = torch.zeros(W, **i32)
    ov = torch.zeros(1, **i32)
    bits = int(np.ceil(np.log2(max(W * Vs, 2))))
    temp = torch.zeros(max(H.sort_pairs_temp_bytes(n, bits), 16), dtype=torch.uint8, device=dev)
    kp = H.ShardKeysParams()
    kp.ids, kp.n, kp.W, kp.Vs, kp.keys = ids.data_ptr(), n, W, Vs, keys.data_ptr()
    s = torch.cuda.current_stream().cuda_stream
    H.shard_keys(kp, s)
    H.sort_pairs_iota(temp.data_ptr(), temp.numel(), keys.data_ptr(), sk.data_ptr(), sv.data_ptr(), n, bits, s)
    rp = H.ShardRouteParams()
    rp.skeys, rp.svals, rp.n, rp.W, rp.Vs, rp.cap = sk.data_ptr(), sv.data_ptr(), n, W, Vs, cap
    rp.send_ids, rp.local_idx, rp.skeys_local = send.data_ptr(), local.data_ptr(), skl.data_ptr()
    rp.counts, rp.overflow = counts.data_ptr(), ov.data_ptr()
    scratch = torch.zeros(H.route_scratch_ints(n), **i32)
    rp.scratch = scratch.data_ptr()
    H.shard_route(rp, s)
    torch.cuda.synchronize()
    return send.cpu().numpy(), local.cpu().numpy(), counts.cpu().numpy(), int(ov.item()), skl, sv, local


@pytest.mark.parametrize("W,n,V", [(1, 3000, 500), (3, 40000, 100003), (8, 39 * 1024, 1_000_000)])
def test_shard_route_matches_reference(W, n, V):
    from rocfm.ops.reference import shard_route_reference

    g = torch.Generator().manual_seed(W * 7 + 1)
    ids = torch.randint(0, V, (n,), generator=g, dtype=torch.int32)
    ids[::5] = 17  # hot id
    ids[1::7] = torch.randint(0, 50, (len(ids[1::7]),), generator=g, dtype=torch.int32)
    cap = n
    send, local, counts, ov, skl, sv, local_t = _route(ids.cuda(), W, V, cap)
    rs, rl, rc = shard_route_reference(ids.numpy(), W, (V + W - 1) // W, cap)
    assert ov == 0
    np.testing.assert_array_equal(counts, rc)
    np.testing.assert_array_equal(send.astype(np.int64).reshape(W, cap), rs)
    np.testing.assert_array_equal(local, rl)
    # sorted local keys are the lookup rows in sort order
    np.testing.assert_array_equal(skl.cpu().numpy(), local_t[sv.long()].cpu().numpy())


def test_shard_route_overflow_flag():
    ids = torch.arange(0, 4000, dtype=torch.int32).cuda()  # 2000 unique ids per owner
    _, _, counts, ov, *_ = _route(ids, 2, 4000, 1000)
    assert ov == 1 and counts.tolist() == [2000, 2000]


def _assert_params_close(got, exp, atol, frac_max=1e-3):
    """Every variable elementwise to ``atol`` (+ 2e-3 relative) except for at most 0.1 % of
    entries (``frac_max``; ≤ 5e-3): rank-partial and kernel-specific fma contraction reorder fp32 additions by a
    last bit, and Adam turns that into a full lr-sized step on the few rows whose summed gradient
    is ≈ 0.  A wrong merge or routing moves many rows, far beyond these bounds."""
    for k in exp:
        d = (got[k].float() - exp[k].float()).abs()
        frac = (d > atol + 2e-3 * exp[k].float().abs()).float().mean().item()
        if exp[k].numel() < 100:  # scalars / short bias vectors: bounded by the Adam step size only
            assert d.max().item() < 5e-3, (k, d.max().item())
        else:
            assert d.max().item() < 5e-3 and frac < frac_max, (k, d.max().item(), frac)


def _assert_params_tight(got, exp, rtol=1e-5, atol=1e-7):
    """Routing / merge check with a LINEAR optimizer (Momentum, GD): no Adam m/√v chaos, so the only
    differences are fp32 summation order (rank partials) — every element, no outlier allowance.
    Momentum at lr 0.02 moves a touched row by ≳1e-5 per step: a dropped, doubled or misrouted
    row gradient is orders of magnitude beyond these bounds."""
    for k in exp:
        e, g = exp[k].float().cpu(), got[k].float().cpu()
        d = (g - e).abs()
        lim = atol + rtol * e.abs()
        bad = (d > lim)
        assert not bad.any(), (k, int(bad.sum()), d.max().item(), (d - lim).max().item())


_LR = {"Adam": 1e-3, "Momentum": 0.02, "GD": 0.05}


def _cfg(opt="Adam"):
    from rocfm.models.deepfm import ModelSpec
    from rocfm.optim import OptHParams

    spec = ModelSpec(feature_size=4001, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)
    return spec, OptHParams(name=opt, lr=_LR[opt])


def _batches(B, n, seed, disjoint=False):
    """``disjoint``: consecutive batches look up disjoint id halves (even steps [0, 2000), odd
    [2000, 4000)), so a row served one step early (staleness 1) is never one the step before updated."""
    from rocfm.data.synthetic import SyntheticCriteo

    g = torch.Generator().manual_seed(seed)
    gen = SyntheticCriteo(4001, 39, seed=seed)
    out = [gen.batch(B, "cpu", g) for _ in range(n)]
    if disjoint:
        out = [((b[0] % 2000) + 2000 * (i % 2), b[1], b[2]) for i, b in enumerate(out)]
    return out


def _single(update, nsteps, B=128, opt="Adam", disjoint=False):
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM

    spec, hp = _cfg(opt)
    single = FusedDeepFM(spec, hp, B, torch.device("cuda"), params=init_params(spec, 3), use_graph=False,
                         embedding_update=update)
    batches = _batches(B, nsteps, 11, disjoint)
    single.attach_pool(torch.stack([b[0] for b in batches]).cuda(), torch.stack([b[1] for b in batches]).cuda(),
                       torch.stack([b[2] for b in batches]).cuda())
    for _ in range(nsteps):
        single.train_step()
    torch.cuda.synchronize()
    return single


def _world1(update, mode, n=11, opt="Momentum", hot=0, staleness=0, disjoint=False, replicate=False):
    """A 1-rank FusedRowShard trained eagerly, per-step graphs or multi-step graphs (4 per graph)."""
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg(opt)
    eng = FusedRowShard(spec, hp, 128, torch.device("cuda"), params=init_params(spec, 3), embedding_update=update,
                        use_graph=mode != "eager", hot_rows=hot, staleness=staleness, replicate_table=replicate)
    batches = _batches(128, n, 11, disjoint)
    eng.attach_pool(torch.stack([b[0] for b in batches]).cuda(), torch.stack([b[1] for b in batches]).cuda(),
                    torch.stack([b[2] for b in batches]).cuda())
    if hot:
        assert eng.n_hot == hot
    if mode == "multi":
        eng.train_steps(n, 4)  # 4 eager + 4 graph + 3 tail graph (≥ 2 multi-step graphs)
    else:
        for _ in range(n):
            eng.train_step()
    torch.cuda.synchronize()
    eng.check()
    return eng


def _tables(eng):
    """Parameters plus the tables' optimizer slots (replicated rows seen through their owners)."""
    sd = eng.state_dict()
    out = dict(eng.parameters_tf())
    out.update({k: v for k, v in sd.items() if k.startswith("fm_")})
    return out


@pytest.mark.parametrize("update,mode", [("sparse", "eager"), ("sparse", "graph"), ("exact", "eager"),
                                         ("sparse", "multi"), ("exact", "multi")])
def test_fused_rowshard_world1_equals_single(update, mode):
    """Routing at world 1 (eager, per-step graphs, multi-step graphs) with Momentum: every element
    of every variable and slot within fp32 reorder bounds of the single-GPU engine."""
    eng = _world1(update, mode)
    ref = _single(update, 11, opt="Momentum")
    _assert_params_tight(_tables(eng), _tables(ref))
    ids, vals, labels = _batches(100, 1, 5)[0]
    p, _ = eng.predict_batch(ids.cuda(), vals.cuda())
    pr, _ = ref.predict_batch(ids.cuda(), vals.cuda())
    torch.testing.assert_close(p, pr, rtol=1e-4, atol=1e-6)


def test_fused_rowshard_world1_adam_smoke():
    """Adam (m/√v turns last-bit reorder differences on ≈0-gradient rows into lr-sized steps): the
    loose outlier comparison, one case."""
    eng = _world1("sparse", "graph", n=10, opt="Adam")
    ref = _single("sparse", 10)
    _assert_params_close(eng.parameters_tf(), ref.parameters_tf(), 2e-5)


def _worker(rank, world, port, update, out_path, exchange="rccl", steps=3, spg=0, staleness=0, hot=0, opt="Momentum",
            shadow=0, fault="", replicate=False):
    # ROCFM_DP_PUSH=1: the X4 producer push is forced on although the ranks share this GPU (small
    # batches; the default keeps the copy push there).  shadow: collective-shadowed first steps
    # (0 = off, so the equivalence tests keep their graph coverage); fault: ROCFM_FAULT
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), ROCFM_DP_PUSH="1", ROCFM_SPIN_LIMIT=str(1 << 26),
                      ROCFM_SHADOW_STEPS=str(shadow),
                      ROCFM_FAULT=fault)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg(opt)
    B = 64
    eng = FusedRowShard(spec, hp, B, torch.device("cuda", 0), params=init_params(spec, 3), embedding_update=update,
                        use_graph=spg > 0, exchange=exchange, staleness=staleness, hot_rows=hot,
                        replicate_table=replicate)
    assert eng.exchange == exchange, eng.exchange
    assert eng.fused_push == (exchange == "p2p" and hot == 0), eng.fused_push
    fused = eng.fused_push
    batches = _batches(world * B, steps, 11, disjoint=staleness > 0)
    pool = [(b[0][rank * B:(rank + 1) * B], b[1][rank * B:(rank + 1) * B], b[2][rank * B:(rank + 1) * B])
            for b in batches]
    eng.attach_pool(torch.stack([x[0] for x in pool]).cuda(), torch.stack([x[1] for x in pool]).cuda(),
                    torch.stack([x[2] for x in pool]).cuda())
    if spg:
        eng.train_steps(steps, spg)  # multi-step graphs (p2p pushes captured; gloo is not)
    else:
        for _ in range(steps):
            eng.train_step()
    torch.cuda.synchronize()
    eng.check()
    P = eng.parameters_tf()
    status = {"shadow": eng.shadow.status, "exchange": eng.exchange, "fused": fused,
              "consistent": eng.verify_replicas()}
    # the streamed export's row ranges reassemble the gathered tables
    fw = torch.cat([c[1] for c in eng.iter_table_chunks(chunk_rows=700)])
    fv = torch.cat([c[2] for c in eng.iter_table_chunks(chunk_rows=700)])
    assert torch.equal(fw, P["fm_w"]) and torch.equal(fv, P["fm_v"])
    ids, vals, _ = _batches(100, 1, 5)[0]
    p, _ = eng.predict_batch(ids.cuda() if rank == 0 else ids[:0].cuda(), vals.cuda() if rank == 0 else vals[:0].cuda())
    if hot:
        assert eng.n_hot == hot
    if replicate:  # the full replica equals the owners' shards on every rank
        full = eng.emb_full.cpu()
        assert torch.equal(full[:, :spec.embedding_size], P["fm_v"]) and torch.equal(full[:, spec.embedding_size], P["fm_w"])
    if rank == 0:
        torch.save({"P": dict(P), "pred": p.cpu(), **status}, out_path)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _run_ranks(tmp_path, world, update, exchange, steps, spg, staleness=0, hot=0, opt="Momentum", shadow=0,
               fault="", replicate=False):
    out = str(tmp_path / f"rs{world}.pt")
    mp.start_processes(_worker, args=(world, _free_port(), update, out, exchange, steps, spg, staleness, hot, opt,
                                      shadow, fault, replicate), nprocs=world, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["consistent"], got["shadow"]
    return got


@pytest.mark.parametrize("world,update,staleness,hot,fault", [
    (2, "sparse", 0, 0, ""), (2, "exact", 0, 0, ""), (4, "sparse", 0, 32, ""), (2, "sparse", 1, 0, ""),
    (2, "sparse", 0, 0, "corrupt_push:1"), (2, "sparse", 0, 48, "corrupt_push:0")])
def test_rowshard_shadow_exchange(tmp_path, world, update, staleness, hot, fault):
    """Self-validation of the row-shard exchanges: the first 8 steps run X1-X4 through the p2p
    pushes (X3 / X4 from the step tail's producers when fused) AND the collective, compared
    bitwise; the step consumes the collective's copy.  Clean runs keep p2p (status ok); an
    injected corrupt word is detected and every rank falls back to the collective — the replicas
    (MLP, replicated rows) agree and the result equals the single-GPU engine either way."""
    steps = 13
    got = _run_ranks(tmp_path, world, update, "p2p", steps, 4, staleness, hot, shadow=8, fault=fault)
    if fault:
        assert got["shadow"] == "mismatch" and got["exchange"] == "rccl", got["shadow"]
    else:
        assert got["shadow"] == "ok" and got["exchange"] == "p2p", got["shadow"]
    ref = _single(update, steps, B=64 * world, opt="Momentum", disjoint=staleness > 0)
    _assert_params_tight(got["P"], ref.parameters_tf())


@pytest.mark.parametrize("update,exchange,steps,spg", [("sparse", "rccl", 3, 0), ("exact", "rccl", 3, 0),
                                                       ("sparse", "p2p", 3, 0), ("exact", "p2p", 3, 0),
                                                       ("sparse", "p2p", 10, 4)])
def test_fused_rowshard_2ranks_equals_single_gpu_union_batch(tmp_path, update, exchange, steps, spg):
    """exchange=rccl runs the backend's collectives (gloo here); p2p the IPC push kernels.  Momentum:
    every element within fp32 reorder bounds."""
    got = _run_ranks(tmp_path, 2, update, exchange, steps, spg)
    ref = _single(update, steps, opt="Momentum")
    _assert_params_tight(got["P"], ref.parameters_tf())
    ids, vals, _ = _batches(100, 1, 5)[0]
    pr, _ = ref.predict_batch(ids.cuda(), vals.cuda())
    torch.testing.assert_close(got["pred"], pr.cpu(), rtol=1e-4, atol=1e-6)


def test_fused_rowshard_2ranks_adam_smoke(tmp_path):
    got = _run_ranks(tmp_path, 2, "sparse", "p2p", 3, 0, opt="Adam")
    ref = _single("sparse", 3)
    _assert_params_close(got["P"], ref.parameters_tf(), 2e-5, frac_max=1e-2)


@pytest.mark.parametrize("update,merge,hot", [("sparse", "direct", 0), ("exact", "direct", 0), ("sparse", "hash", 32)])
def test_fused_rowshard_4ranks_p2p_graphs(tmp_path, update, merge, hot, monkeypatch):
    """4 ranks on one GPU: every table is split 4 ways and each all-to-all pushes to 3 peers (the
    W>2 routing the 8-GPU node runs), through multi-step graphs; beyond SEARCH_MAX_W ranks the
    owner merge scatters into direct maps or the O(W·cap) hash table (ROCFM_MERGE), with and
    without replicated hot rows."""
    monkeypatch.setenv("ROCFM_MERGE", merge)
    steps = 10
    got = _run_ranks(tmp_path, 4, update, "p2p", steps, 4, 0, hot)
    ref = _single(update, steps, B=256, opt="Momentum")
    _assert_params_tight(got["P"], ref.parameters_tf())
    ids, vals, _ = _batches(100, 1, 5)[0]
    pr, _ = ref.predict_batch(ids.cuda(), vals.cuda())
    torch.testing.assert_close(got["pred"], pr.cpu(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("mode", ["eager", "graph", "multi"])
def test_rowshard_staleness1_disjoint_batches_equal_sync(mode):
    """Bounded staleness (async-PS emulation): when consecutive batches share no rows, serving a
    step's rows during the previous update changes nothing — the synchronous result."""
    eng = _world1("sparse", mode, staleness=1, disjoint=True)
    ref = _single("sparse", 11, opt="Momentum", disjoint=True)
    _assert_params_tight(_tables(eng), _tables(ref))


def test_rowshard_staleness1_overlapping_batches_trains():
    """With shared rows the stale reads change the trajectory (so the mode is really asynchronous)
    but training stays finite and close to the synchronous run."""
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg()
    n = 12
    out = {}
    for st in (0, 1):
        eng = FusedRowShard(spec, hp, 128, torch.device("cuda"), params=init_params(spec, 3), use_graph=True,
                            staleness=st)
        batches = _batches(128, n, 11)
        eng.attach_pool(torch.stack([b[0] for b in batches]).cuda(), torch.stack([b[1] for b in batches]).cuda(),
                        torch.stack([b[2] for b in batches]).cuda())
        for _ in range(n):
            eng.train_step()
        torch.cuda.synchronize()
        eng.check()
        out[st] = (eng.parameters_tf(), eng.batch_loss())
    d = (out[0][0]["fm_v"] - out[1][0]["fm_v"]).abs().max().item()
    assert 0 < d < 1e-2
    assert np.isfinite(out[1][1]) and abs(out[1][1] - out[0][1]) < 0.05


def test_rowshard_staleness1_2ranks_p2p(tmp_path):
    """Two ranks, p2p pushes, double-buffered request lists, multi-step graphs: on disjoint
    consecutive batches ≡ the single-GPU engine on the union batch."""
    got = _run_ranks(tmp_path, 2, "sparse", "p2p", 10, 4, staleness=1)
    ref = _single("sparse", 10, opt="Momentum", disjoint=True)
    _assert_params_tight(got["P"], ref.parameters_tf())


@pytest.mark.parametrize("update,mode", [("sparse", "eager"), ("sparse", "graph"), ("sparse", "multi"),
                                         ("exact", "multi")])
def test_rowshard_hot_rows_world1_equals_single(update, mode):
    """Hot-row replication: the 64 most frequent ids live in the local replica (routed to the
    virtual owner W, updated from the X4 bucket) — with Momentum every element of every variable
    and table slot equals the single-GPU engine to fp32 reorder bounds; the checkpoint /
    prediction see the replica through the owners' rows."""
    eng = _world1(update, mode, hot=64)
    ref = _single(update, 11, opt="Momentum")
    _assert_params_tight(_tables(eng), _tables(ref))
    ids, vals, _ = _batches(100, 1, 5)[0]
    p, _ = eng.predict_batch(ids.cuda(), vals.cuda())
    pr, _ = ref.predict_batch(ids.cuda(), vals.cuda())
    torch.testing.assert_close(p, pr, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_rowshard_hot_rows_multistep_bitwise_reproducible(update):
    """Replicated rows through ≥ 2 multi-step graphs with each graph's side chain (next batches'
    fetch / sort / route) running BESIDE its main graph: two runs in one process are bitwise
    equal (Adam, the optimizer most sensitive to a partly-updated row).  Guards the replica update's
    touched-count hand-off (hot_apply_body reads and clears it in one thread)."""
    runs = [_tables(_world1(update, "multi", n=19, opt="Adam", hot=64)) for _ in range(2)]
    for k in runs[0]:
        assert torch.equal(runs[0][k], runs[1][k]), k


@pytest.mark.parametrize("exchange,spg", [("p2p", 4), ("rccl", 0)])
def test_rowshard_hot_rows_2ranks(tmp_path, exchange, spg):
    """Two ranks: replicated rows' sums travel in the X4 bucket (p2p rank segments summed in rank
    order / the backend's all-reduce) ≡ the single-GPU engine on the union batch (Momentum)."""
    got = _run_ranks(tmp_path, 2, "sparse", exchange, 10, spg, 0, 48)
    ref = _single("sparse", 10, opt="Momentum")
    _assert_params_tight(got["P"], ref.parameters_tf())
    ids, vals, _ = _batches(100, 1, 5)[0]
    pr, _ = ref.predict_batch(ids.cuda(), vals.cuda())
    torch.testing.assert_close(got["pred"], pr.cpu(), rtol=1e-4, atol=1e-6)


# ---- owner-sharded DP (parallelism=dp_owner: replicated table, owner-sharded embedding optimizer) ----
@pytest.mark.parametrize("mode", ["eager", "graph", "multi"])
def test_dp_owner_world1_equals_single(mode):
    """dp_owner at world 1: the forward reads the full replica, the owner merge broadcasts every
    updated row (X5) and row_scatter writes it back — Momentum, every element of every variable and
    slot within fp32 reorder bounds of the single-GPU engine; the replica equals the shard."""
    eng = _world1("sparse", mode, replicate=True)
    ref = _single("sparse", 11, opt="Momentum")
    _assert_params_tight(_tables(eng), _tables(ref))
    P = eng.parameters_tf()
    full = eng.emb_full.cpu()
    assert torch.equal(full[:, :10], P["fm_v"]) and torch.equal(full[:, 10], P["fm_w"])


@pytest.mark.parametrize("world,exchange,steps,spg", [(2, "rccl", 3, 0), (2, "p2p", 3, 0), (2, "p2p", 10, 4),
                                                     (4, "p2p", 10, 4)])
def test_dp_owner_ranks_equal_single_gpu_union_batch(tmp_path, world, exchange, steps, spg):
    """2 and 4 ranks on one GPU: X1 + X3 + X4 in one hand-off, the owner merge pushing its updated
    rows into every rank's X5 slot, row_scatter into every replica — equal to the single-GPU step on
    the union batch (Momentum, tight), replicas bit-identical (checked by the worker)."""
    got = _run_ranks(tmp_path, world, "sparse", exchange, steps, spg, replicate=True)
    ref = _single("sparse", steps, B=64 * world, opt="Momentum")
    _assert_params_tight(got["P"], ref.parameters_tf())


@pytest.mark.parametrize("fault", ["", "corrupt_push:1"])
def test_dp_owner_shadow_exchange(tmp_path, fault):
    """The first 8 steps shadow every p2p exchange (X1, X3, X4, X5) with the collective; a corrupt
    word is detected and every rank falls back to RCCL; the result equals the single GPU."""
    steps = 13
    got = _run_ranks(tmp_path, 2, "sparse", "p2p", steps, 4, shadow=8, fault=fault, replicate=True)
    if fault:
        assert got["shadow"] == "mismatch" and got["exchange"] == "rccl", got["shadow"]
    else:
        assert got["shadow"] == "ok" and got["exchange"] == "p2p", got["shadow"]
    ref = _single("sparse", steps, B=128, opt="Momentum")
    _assert_params_tight(got["P"], ref.parameters_tf())


def _owner_restore_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), ROCFM_SPIN_LIMIT=str(1 << 26), ROCFM_SHADOW_STEPS="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg("Momentum")
    B, n1, n2 = 64, 6, 5
    batches = _batches(world * B, n1 + n2, 11)
    pool = [torch.stack([b[i][rank * B:(rank + 1) * B] for b in batches]).cuda() for i in range(3)]

    def make(seed):
        return FusedRowShard(spec, hp, B, torch.device("cuda", 0), params=init_params(spec, seed), use_graph=True,
                             exchange="p2p", replicate_table=True)

    a = make(3)
    a.attach_pool(*pool)
    a.train_steps(n1, 4)
    torch.cuda.synchronize()
    sd = {k: v.clone() for k, v in a.state_dict().items()}
    b = make(99)  # other initial weights: everything must come from the checkpoint
    b.load_state_dict(sd)
    b.attach_pool(*pool)
    torch.cuda.synchronize()
    # the restored replica is the gathered owners' shards, on every rank (a stale replica would pass
    # verify_replicas — every rank equally stale — and silently feed the forward old rows)
    Pb = b.parameters_tf()
    full = b.emb_full.cpu()
    restored = (torch.equal(full[:, :spec.embedding_size], Pb["fm_v"]) and
                torch.equal(full[:, spec.embedding_size], Pb["fm_w"]) and torch.equal(full, a.emb_full.cpu()))
    for e in (a, b):
        e.train_steps(n2, 4)
        torch.cuda.synchronize()
        e.check()
    Pa, Pb = a.parameters_tf(), b.parameters_tf()
    same = all(torch.equal(Pa[k], Pb[k]) for k in Pa) and torch.equal(a.emb_full, b.emb_full)
    if rank == 0:
        torch.save({"restored": restored, "same": same, "step": b.global_step()}, out_path)
    a.close()
    b.close()
    dist.barrier()
    dist.destroy_process_group()


def test_dp_owner_checkpoint_restore_2ranks(tmp_path):
    """dp_owner restore: load_state_dict rebuilds every rank's full replica from the
    owners' shards (_sync_full); training on from the restored engine equals the uninterrupted run,
    bitwise."""
    out = str(tmp_path / "own.pt")
    mp.start_processes(_owner_restore_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["restored"] and got["same"] and got["step"] == 11, got
