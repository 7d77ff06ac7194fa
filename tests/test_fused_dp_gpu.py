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


def _cfg():
    from rocfm.models.deepfm import ModelSpec
    from rocfm.optim import OptHParams

    spec = ModelSpec(feature_size=4000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)
    return spec, OptHParams(name="Adam", lr=1e-3)


def _batches(B, n, seed):
    from rocfm.data.synthetic import SyntheticCriteo

    g = torch.Generator().manual_seed(seed)
    gen = SyntheticCriteo(4000, 39, seed=seed)
    return [gen.batch(B, "cpu", g) for _ in range(n)]


def _worker(rank, world, port, mode, out_path, exchange="rccl", steps=3, spg=0, update=None, push="1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), ROCFM_DP_PUSH=push)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.models.deepfm import init_params
    from rocfm.parallel.dp import FusedDataParallel

    spec, hp = _cfg()
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
    eng.check()
    if rank == 0:
        torch.save({"emb": eng.emb.cpu(), "dense": eng.dense.cpu()}, out_path)
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
    W>2 paths the 8-GPU node runs), through multi-step graphs."""
    _check_dp_vs_single(tmp_path, 4, "dp", "p2p", 11, 4, update)


@pytest.mark.parametrize("world,spg", [(2, 0), (4, 4)])
def test_fused_dp_p2p_unfused_push(tmp_path, world, spg):
    """ROCFM_DP_PUSH=0: the tail writes the local send buffer and the push launch copies all of it
    (the path before producer-side pushing) ≡ the single-GPU union batch."""
    _check_dp_vs_single(tmp_path, world, "dp", "p2p", 11 if spg else 3, spg, "sparse", push="0")


def _check_dp_vs_single(tmp_path, world, mode, exchange, steps, spg, update, push="1"):
    # ranks share this GPU, where the fused push is off by default: the workers force it (small
    # batches keep the spinning producers from starving a peer) unless the copy push is asked for
    out = str(tmp_path / "dp.pt")
    mp.start_processes(_worker, args=(world, _free_port(), mode, out, exchange, steps, spg, update, push), nprocs=world,
                       join=True, start_method="spawn")
    dp = torch.load(out, weights_only=True)
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM

    spec, hp = _cfg()
    single = FusedDeepFM(spec, hp, 64 * world, torch.device("cuda"), params=init_params(spec, 3), use_graph=False,
                         embedding_update=update)
    batches = _batches(64 * world, steps, 11)
    single.attach_pool(torch.stack([b[0] for b in batches]).cuda(), torch.stack([b[1] for b in batches]).cuda(),
                       torch.stack([b[2] for b in batches]).cuda())
    for _ in range(steps):
        single.train_step()
    torch.cuda.synchronize()
    # rank-partial sums reorder fp32 additions; Adam amplifies that for near-zero gradients
    # (m/√v), so the tolerance grows with the number of steps (a missed or stale row would be off
    # by a whole step, ≈lr = 1e-3)
    atol = 2e-5 if steps <= 3 else 1e-4
    torch.testing.assert_close(dp["dense"], single.dense.cpu(), rtol=2e-3, atol=atol)
    torch.testing.assert_close(dp["emb"], single.emb.cpu(), rtol=2e-3, atol=atol)


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_fused_dp_world4_hash_merge(tmp_path, monkeypatch, update):
    """The O(W·cap) step-tagged hash merge (ROCFM_MERGE=hash; what 1B-row vocabularies use) through
    4 ranks, multi-step graphs and the p2p push ≡ the single-GPU union batch."""
    monkeypatch.setenv("ROCFM_MERGE", "hash")
    _check_dp_vs_single(tmp_path, 4, "dp", "p2p", 11, 4, update)


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
    torch.testing.assert_close(dp.emb, one.emb, rtol=2e-3, atol=2e-5)
    torch.testing.assert_close(dp.dense, one.dense, rtol=2e-3, atol=2e-5)
    dp.check()
    if mode == "dp":
        assert dp.maps.hashed == (merge == "hash")
