"""Distributed logic on CPU (gloo, 2 ranks): data parallelism ≡ single process on the union batch,
rank-0 broadcast, sharding policies."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rocfm.data.sharding import eval_shard, pipe_channel, train_shard
from rocfm.parallel.dist import RankInfo


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spec():
    from rocfm.models.deepfm import ModelSpec

    return ModelSpec(feature_size=300, field_size=8, embedding_size=4, layers=[16, 8], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)


def _batches(n, B, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 300, (B, 8), generator=g)
        ids[:, 0] = 5  # a hot row shared by all ranks
        out.append((ids, torch.rand(B, 8, generator=g), (torch.rand(B, generator=g) < 0.3).float()))
    return out


def _worker(rank, world, port, update, opt, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rocfm.models.deepfm import init_params
    from rocfm.models.torch_engine import TorchDeepFM
    from rocfm.optim import OptHParams
    from rocfm.parallel.dist import broadcast_tensors
    from rocfm.parallel.dp import attach_torch_dp

    spec = _spec()
    P = init_params(spec, 100 + rank)  # different init per rank: the broadcast must fix it
    eng = TorchDeepFM(spec, OptHParams(name=opt, lr=0.01), embedding_update=update, params=P)
    broadcast_tensors(list(eng.P.values()))
    attach_torch_dp(eng, update)
    B = 16
    for ids, vals, labels in _batches(3, world * B, 7):
        sl = slice(rank * B, (rank + 1) * B)
        eng.train_step(ids[sl], vals[sl], labels[sl])
    if rank == 0:
        torch.save(dict(eng.P), out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,update,opt", [(2, "sparse", "Adam"), (2, "exact", "Adam"), (2, "sparse", "Adagrad"),
                                              (4, "sparse", "Adam"), (4, "exact", "Adam"), (8, "sparse", "Adam"),
                                              (8, "exact", "Adagrad")])
def test_torch_dp_equals_single_process_union_batch(tmp_path, world, update, opt):
    """the DP path at 2, 4 and 8 ranks ≡ one process on the union batch."""
    out = str(tmp_path / "p.pt")
    mp.start_processes(_worker, args=(world, _port(), update, opt, out), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(out, weights_only=True)
    from rocfm.models.deepfm import init_params
    from rocfm.models.torch_engine import TorchDeepFM
    from rocfm.optim import OptHParams

    spec = _spec()
    ref = TorchDeepFM(spec, OptHParams(name=opt, lr=0.01), embedding_update=update, params=init_params(spec, 100))
    for ids, vals, labels in _batches(3, 16 * world, 7):
        ref.train_step(ids, vals, labels)
    for k in ref.P:
        torch.testing.assert_close(got[k], ref.P[k], rtol=1e-5, atol=1e-6)


def test_sharding_policy_table():
    r = RankInfo(rank=5, world=8, local_rank=1, local_world=4, host_index=1, num_hosts=2)
    assert train_shard(r, pipe_mode=0, enable_s3_shard=True) == (4, 1)  # HVD:131
    assert train_shard(r, pipe_mode=0, enable_s3_shard=False) == (8, 5)  # HVD:133
    assert train_shard(r, pipe_mode=1, enable_data_multi_path=True, enable_s3_shard=False) == (2, 1)  # HVD:141-144
    assert train_shard(r, pipe_mode=1, enable_data_multi_path=True, enable_s3_shard=True) == (1, 0)  # HVD:140
    assert train_shard(r, pipe_mode=1, enable_data_multi_path=False, enable_s3_shard=True) == (4, 1)  # HVD:146
    assert train_shard(r, pipe_mode=1, enable_data_multi_path=False, enable_s3_shard=False) == (8, 5)  # HVD:148
    assert train_shard(r, ps_mode=True) == (2, 1)  # PS:153-156
    assert eval_shard(r) == (8, 5)
    assert pipe_channel(["evaluation", "training", "training-1"], 1) == "training-1"
    assert pipe_channel(["evaluation", "training"], 0, training=False) == "evaluation"
