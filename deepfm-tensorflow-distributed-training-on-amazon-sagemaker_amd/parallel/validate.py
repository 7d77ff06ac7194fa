"""Self-validation of a multi-GPU run: replica digests and the shadow exchange.

The reference trusts Horovod/NCCL (HVD:296, 418): every rank ends each step with the same
variables because the all-reduce is correct.  rocfm's default N>1 transport is its own p2p push
over IPC-mapped peer buffers (``rocfm.parallel.p2p``), with producers storing straight into the
peers' slots from the step tail.  A coherence bug there would give a fast but wrong number, so a
run checks itself:

* **Replica digest** (``replicas_agree``): an order-independent device-side hash of every
  replicated tensor (DP: MLP + tables + optimizer slots; row-shard: MLP + replicated hot rows),
  MIN/MAX-all-reduced.  DP replicas are bit-identical by construction (every rank sums the
  gathered rank segments in rank order), so ANY difference is a bug.  Engines run it in ``check()``.
* **Shadow exchange** (``Shadow``): for the first ``ROCFM_SHADOW_STEPS`` (default 8) steps of a p2p
  run, every exchange is ALSO done through the process group's collective (RCCL) from the data
  each rank holds locally — its send buffer, which producer-side pushes mirror during the window
  (DP export + MLP gradients, row-shard X3 / X4); the dp_owner X5 row broadcast has no local
  copy and is checked from the owner's own receive slot, i.e. for transfer and receiver
  agreement only — the two results are compared bitwise and the collective's result is what the
  step consumes.  After the window the ranks agree: any mismatch anywhere → every rank
  falls back to RCCL (replicas stay consistent, because the validated steps used RCCL's data).

``ROCFM_FAULT=corrupt_push:R`` makes rank R flip one received word of every shadowed p2p exchange
(test of the detection and the agreed fallback); ``corrupt_replica:R`` perturbs one MLP weight of
rank R before the first digest (test of the replica check).
"""
from __future__ import annotations

import logging
import os
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger("rocfm")

_SAMPLE_MAX = 1 << 22  # elements hashed per tensor (larger tensors: an evenly strided sample)


def _faults(kind: str) -> List[int]:
    """Ranks named by ``kind:R`` entries of ROCFM_FAULT (the validation faults)."""
    out = []
    for part in filter(None, (p.strip() for p in os.environ.get("ROCFM_FAULT", "").split(","))):
        k, _, r = part.partition(":")
        if k == kind and r.isdigit():
            out.append(int(r))
    return out


def fault_rank(kind: str, rank: int) -> bool:
    return rank in _faults(kind)


def tensor_digest(tensors: Iterable[torch.Tensor], sample_max: int = _SAMPLE_MAX) -> torch.Tensor:
    """[2·T] int64 on the tensors' device: per tensor, Σ_i lo16(bits_i)·(2i+1) and Σ_i hi16(bits_i)·(2i+1)
    over its raw bits (4-byte dtypes as int32, 2-byte as int16).  Exact integer sums (no overflow
    below 2^22 elements), so equal on two ranks iff the sampled bits are (up to hash collisions)."""
    outs = []
    for t in tensors:
        flat = t.detach().reshape(-1)
        n = flat.numel()
        if n == 0:
            outs.append(torch.zeros(2, dtype=torch.int64, device=t.device))
            continue
        if n > sample_max:
            flat = flat[:: (n + sample_max - 1) // sample_max]
        flat = flat.contiguous()
        es = flat.element_size()
        if es == 4:
            bits = flat.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        elif es == 2:
            bits = flat.view(torch.int16).to(torch.int64) & 0xFFFF
        elif es == 8:
            bits = flat.view(torch.int64) & 0xFFFFFFFF  # low words (int64 step counters)
        else:
            bits = flat.view(torch.uint8).to(torch.int64)
        w = torch.arange(bits.numel(), dtype=torch.int64, device=bits.device) * 2 + 1
        outs.append(torch.stack([((bits & 0xFFFF) * w).sum(), ((bits >> 16) * w).sum()]))
    return torch.cat(outs) if outs else torch.zeros(0, dtype=torch.int64)


def _coll_device(group, device) -> torch.device:
    return torch.device(device) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def replicas_agree(tensors: List[torch.Tensor], group=None) -> bool:
    """Collective: True iff every rank's ``tensor_digest`` of its replicated tensors is equal."""
    if not tensors:
        return True
    d = tensor_digest(tensors)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return True
    t = torch.cat([d, -d]).to(_coll_device(group, tensors[0].device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    n = d.numel()
    return bool(torch.equal(t[:n], -t[n:]))  # max == min for every component


def any_rank(flag: bool, device, group=None) -> bool:
    """Collective OR of a per-rank flag."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return flag
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=_coll_device(group, device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(int(t.item()))


class Shadow:
    """Bookkeeping of one engine's shadow-exchange window.

    ``compare(got, want)`` (device, no host sync): counts words whose bits differ, then copies
    ``want`` (the collective's result) over ``got`` so the step consumes validated data.
    ``finish()`` (collective, once the window has elapsed) returns whether any rank saw a mismatch.
    """

    def __init__(self, device, steps: Optional[int] = None):
        self.left = int(os.environ.get("ROCFM_SHADOW_STEPS", "8")) if steps is None else int(steps)
        self.device = torch.device(device)
        self.bad = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.compared = 0  # exchanges compared on this rank
        self.status = "pending" if self.left > 0 else "off"
        self.corrupt = False  # set by the engine from ROCFM_FAULT=corrupt_push:R

    @property
    def active(self) -> bool:
        return self.left > 0

    def corrupt_(self, got: torch.Tensor) -> None:
        """Fault injection: flip the low bit of one received word (as a bad transfer would)."""
        if self.corrupt and got.numel():
            w = got.reshape(-1).view(torch.int32)
            w[w.numel() // 2] ^= 1

    def compare(self, got: torch.Tensor, want: torch.Tensor) -> None:
        g = got.reshape(-1).view(torch.int32)
        w = want.reshape(-1).view(torch.int32)
        self.bad += (g != w).sum()
        got.reshape(-1).copy_(want.reshape(-1))
        self.compared += 1

    def step_done(self) -> bool:
        """Count one validated step; True when the window has just elapsed."""
        if self.left <= 0:
            return False
        self.left -= 1
        return self.left == 0

    def finish(self, group=None) -> bool:
        """Collective: True if any rank saw a mismatch in the window."""
        mism = any_rank(int(self.bad.item()) > 0, self.device, group)
        self.status = "mismatch" if mism else "ok"
        return mism
