"""Row-sharded (PS-equivalent) embedding on CPU (gloo, 2 ranks): the synchronous row-shard step ≡
the single-process step on the union batch; sharded checkpoints restore on any world size."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spec():
    from rocfm.models.deepfm import ModelSpec

    return ModelSpec(feature_size=301, field_size=8, embedding_size=4, layers=[16, 8], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)


def _batches(n, B, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 301, (B, 8), generator=g)
        ids[:, 0] = 5  # a hot row requested by both ranks
        ids[:, 1] = 300  # the last row (padding edge of the odd-sized table)
        out.append((ids, torch.rand(B, 8, generator=g), (torch.rand(B, generator=g) < 0.3).float()))
    return out


def _worker(rank, world, port, update, opt, out, ckpt_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rocfm import checkpoint as ckpt
    from rocfm.models.deepfm import init_params
    from rocfm.optim import OptHParams
    from rocfm.parallel.emb_shard import TorchRowShard

    spec = _spec()
    eng = TorchRowShard(spec, OptHParams(name=opt, lr=0.01), embedding_update=update, params=init_params(spec, 100))
    eng.set_lr_scale(float(world))
    B = 16
    for ids, vals, labels in _batches(3, world * B, 7):
        sl = slice(rank * B, (rank + 1) * B)
        eng.train_step(ids[sl], vals[sl], labels[sl])
    full = eng.parameters_tf()  # collective gather of the tables
    # sharded checkpoint: every rank writes its shard, rank 0 the manifest
    sd = eng.state_dict()
    rs = eng.row_sets()
    if rank != 0:
        ckpt.save_checkpoint(ckpt_dir, sd, 3, shard=(rank, world), row_sets=rs, write_index=False)
    dist.barrier()
    if rank == 0:
        ckpt.save_checkpoint(ckpt_dir, sd, 3, shard=(0, world), row_sets=rs, global_rows={k: spec.feature_size for k in rs})
    dist.barrier()
    # predict with unequal work per rank (rank 1 has no rows): collective must not deadlock
    ids, vals, labels = _batches(1, 8, 9)[0]
    p, _ = eng.predict_batch(ids if rank == 0 else ids[:0], vals if rank == 0 else vals[:0])
    if rank == 0:
        torch.save({"P": dict(full), "pred": p}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,update,opt", [(2, "sparse", "Adam"), (2, "exact", "Adam"), (2, "sparse", "Adagrad"),
                                              (4, "sparse", "Adam"), (4, "exact", "Adam"), (8, "sparse", "Adam"),
                                              (8, "exact", "Adagrad")])
def test_rowshard_equals_single_process_union_batch(tmp_path, world, update, opt):
    """the row-shard (PS-equivalent) path at 2, 4 and 8 ranks ≡ one process on the
    union batch; the W-shard checkpoint reassembles and restores on one process."""
    out = str(tmp_path / "p.pt")
    cdir = str(tmp_path / "ckpt")
    mp.start_processes(_worker, args=(world, _port(), update, opt, out, cdir), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(out, weights_only=True)
    from rocfm import checkpoint as ckpt
    from rocfm.models.deepfm import init_params
    from rocfm.models.torch_engine import TorchDeepFM
    from rocfm.optim import OptHParams

    spec = _spec()
    hp = OptHParams(name=opt, lr=0.01 * world)  # single process: lr × world (linear scaling)
    ref = TorchDeepFM(spec, hp, embedding_update=update, params=init_params(spec, 100))
    for ids, vals, labels in _batches(3, 16 * world, 7):
        ref.train_step(ids, vals, labels)
    for k in ref.P:
        torch.testing.assert_close(got["P"][k], ref.P[k], rtol=1e-5, atol=1e-6)
    ids, vals, _ = _batches(1, 8, 9)[0]
    pref, _ = ref.predict_batch(ids, vals)
    torch.testing.assert_close(got["pred"], pref, rtol=1e-5, atol=1e-6)
    # the 2-shard checkpoint reassembles into full tables (reshard 2 → 1)
    prefix = ckpt.latest_checkpoint(cdir)
    sd = ckpt.load_checkpoint(prefix)
    torch.testing.assert_close(sd["fm_v"], ref.P["fm_v"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sd["fm_w"], ref.P["fm_w"], rtol=1e-5, atol=1e-6)
    slot = "Adam" if opt == "Adam" else "Adagrad"
    torch.testing.assert_close(sd[f"fm_v/{slot}"], ref.slots["fm_v"][0], rtol=1e-5, atol=1e-6)
    # and restores into a 1-rank row-shard engine / a replicated engine
    from rocfm.parallel.emb_shard import TorchRowShard

    one = TorchRowShard(spec, OptHParams(name=opt, lr=0.01 * world), embedding_update=update)
    one.load_state_dict(sd)
    torch.testing.assert_close(one.base.P["fm_v"], ref.P["fm_v"], rtol=1e-5, atol=1e-6)


def test_shard_helpers():
    from rocfm.parallel.emb_shard import init_shard_params, shard_rows, shard_size, slice_rows

    assert shard_size(301, 2) == 151 and shard_size(300, 4) == 75
    assert shard_rows(10, 3, 1).tolist() == [1, 4, 7]
    t = torch.arange(10.0)
    assert slice_rows(t, 10, 3, 2).tolist() == [2.0, 5.0, 8.0, 0.0]
    spec = _spec()
    P = init_shard_params(spec, 3, 1, 2, "cpu")
    assert P["fm_v"].shape == (151, 4) and float(P["fm_v"][150].abs().sum()) == 0.0  # 301 = 2*150+1: rank 1 pads
    assert P["fm_v"][:150].abs().max() > 0 and "Deep-part/mlp0/weights" in P
