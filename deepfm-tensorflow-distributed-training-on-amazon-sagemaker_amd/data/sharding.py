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

import json
import os
from typing import List, Optional, Tuple

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


def sm_channels() -> List[str]:
    """SageMaker's channel list (env SM_CHANNELS, a JSON list; PS:391, HVD:420)."""
    raw = os.environ.get("SM_CHANNELS", "")
    if not raw:
        return []
    ch = json.loads(raw)
    if not isinstance(ch, list):
        raise ValueError(f"SM_CHANNELS must be a JSON list, got {raw!r}")
    return [str(c) for c in ch]


def pipe_mode_sources(num_epochs: int, local_rank: int, training_channel_name: str = "",
                      evaluation_channel_name: str = "", input_dir: Optional[str] = None):
    """Pipe-mode input (``pipe_mode=1``): the FIFOs SageMaker creates per channel and epoch,
    ``<SM_INPUT_DIR>/data/<channel>_<epoch>`` (what PipeModeDataset opens, PS:150 / HVD:136).

    Channel binding: the explicit ``training_channel_name`` / ``evaluation_channel_name`` flags
    (the PS script, PS:505-513), else SM_CHANNELS with the Horovod script's rule — evaluation =
    channels[0], training = channels[1 + local_rank] (HVD:420-445; SageMaker lists ``evaluation``
    first, README:81).  Returns (train FIFOs for every epoch in order, [eval FIFO])."""
    channels = sm_channels()
    tr = training_channel_name or (pipe_channel(channels, local_rank) if channels else "")
    ev = evaluation_channel_name or (pipe_channel(channels, local_rank, training=False) if len(channels) > 1 else "")
    if not tr:
        raise ValueError("pipe_mode=1 needs SM_CHANNELS or --training_channel_name")
    base = os.path.join(input_dir or os.environ.get("SM_INPUT_DIR", "/opt/ml/input"), "data")
    train = [os.path.join(base, f"{tr}_{e}") for e in range(max(1, int(num_epochs)))]
    evals = [os.path.join(base, f"{ev}_0")] if ev else []
    return train, evals
