"""Data-sharding policies of the reference (HVD:127-149, PS:153-156, README:87-92).

Returns ``(shard_count, shard_index)`` for ``Dataset.shard`` semantics (keep every count-th record
starting at index; record order runs over the concatenated file list), or ``(1, 0)`` for no shard.

=========  ======================  ===============  ============================================
mode       enable_data_multi_path  enable_s3_shard  shard
=========  ======================  ===============  ============================================
file       (ignored)               True             (worker_per_host, local_rank)   HVD:131
file       (ignored)               False            (world, rank)                   HVD:133
pipe       True                    False            (num_hosts, host) if hosts > 1  HVD:141-144
pipe       True                    True             none                            HVD:140-144
pipe       False                   True             (worker_per_host, local_rank)   HVD:146-147
pipe       False                   False            (world, rank)                   HVD:148-149
PS         —                       False            (num_hosts, host_rank)          PS:153-156
=========  ======================  ===============  ============================================

Evaluation data is sharded over ALL ranks and metrics are all-reduced (fix for Q7, where the
reference evaluates only rank 0's 1/N shard).
"""
from __future__ import annotations

from typing import Tuple

from ..parallel.dist import RankInfo


def train_shard(info: RankInfo, pipe_mode: int = 0, enable_s3_shard: bool = False,
                enable_data_multi_path: bool = False, ps_mode: bool = False) -> Tuple[int, int]:
    if ps_mode:
        if enable_s3_shard or info.num_hosts <= 1:
            return 1, 0
        return info.num_hosts, info.host_index
    if pipe_mode == 0:
        if enable_s3_shard:
            return max(info.local_world, 1), info.local_rank
        return max(info.world, 1), info.rank
    if enable_data_multi_path:
        if enable_s3_shard:
            return 1, 0
        if info.num_hosts > 1:
            return info.num_hosts, info.host_index
        return 1, 0
    if enable_s3_shard:
        return max(info.local_world, 1), info.local_rank
    return max(info.world, 1), info.rank


def eval_shard(info: RankInfo) -> Tuple[int, int]:
    return max(info.world, 1), info.rank


def pipe_channel(channels, local_rank: int, training: bool = True) -> str:
    """SageMaker pipe-mode channel binding (HVD:420-445): eval = channels[0], train = channels[1+local_rank]."""
    if not channels:
        raise ValueError("no pipe-mode channels")
    if not training:
        return channels[0]
    return channels[min(1 + local_rank, len(channels) - 1)]
