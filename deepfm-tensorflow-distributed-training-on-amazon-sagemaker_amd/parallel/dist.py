"""Process-group bootstrap and rank bookkeeping (replaces hvd.init / TF_CONFIG).

The reference distributes with either Horovod (``hvd.init()`` HVD:333, one process per GPU pinned
by ``visible_device_list = local_rank`` HVD:393-395) or a TF parameter-server cluster from
SageMaker's ``TF_CONFIG`` (PS:461-490).  Here every mode is one process per GPU under
``torch.distributed``: backend ``nccl`` (= RCCL over xGMI on ROCm) for GPU ranks, ``gloo`` for
CPU ranks (tests).  Rank info comes from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK/
LOCAL_WORLD_SIZE/MASTER_*); SageMaker's SM_HOSTS/SM_CURRENT_HOST are honoured for host indexing
when present (sharding policies, HVD:127-149).
"""
from __future__ import annotations

import datetime
import json
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class RankInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    local_world: int = 1
    host_index: int = 0
    num_hosts: int = 1

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


def rank_info_from_env(worker_per_host: Optional[int] = None, hosts: Optional[List[str]] = None,
                       current_host: Optional[str] = None) -> RankInfo:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(worker_per_host or world)))
    if worker_per_host:
        local_world = worker_per_host
    num_hosts = max(1, world // max(local_world, 1))
    host_index = rank // max(local_world, 1)
    if hosts is None and os.environ.get("SM_HOSTS"):
        try:
            hosts = json.loads(os.environ["SM_HOSTS"])
        except json.JSONDecodeError:
            hosts = None
    if hosts and len(hosts) > 1:
        num_hosts = len(hosts)
        cur = current_host or os.environ.get("SM_CURRENT_HOST")
        if cur in hosts:
            host_index = hosts.index(cur)
    return RankInfo(rank, world, local_rank, local_world, host_index, num_hosts)


def init_distributed(device_type: Optional[str] = None, timeout_s: int = 600) -> RankInfo:
    """Initialise the default process group if WORLD_SIZE > 1 (idempotent)."""
    info = rank_info_from_env()
    if info.world <= 1 or dist.is_initialized():
        return info
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    kw = dict(timeout=datetime.timedelta(seconds=timeout_s))
    if device_type == "cuda":
        torch.cuda.set_device(info.local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", info.local_rank), **kw)
    else:
        dist.init_process_group("gloo", **kw)
    return info


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


@torch.no_grad()
def broadcast_tensors(tensors, src: int = 0) -> None:
    """Rank-0 broadcast of every variable (hvd.BroadcastGlobalVariablesHook(0), HVD:418).

    Flattened into one bucket per dtype so it is a single collective.
    """
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    by_dtype = {}
    for t in tensors:
        if t.numel() * t.element_size() >= (64 << 20) and t.is_contiguous():
            dist.broadcast(t, src)  # large tables: in place, no concatenated copy
            continue
        by_dtype.setdefault(t.dtype, []).append(t)
    for _, ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def all_reduce_scalars(values, op=None, device="cpu"):
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t.tolist()
