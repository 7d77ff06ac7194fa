"""Data parallelism — the Horovod path of the reference (HVD:171, 296, 333, 393-418) on RCCL.

Every rank holds a full replica (rank-0 initial values, like BroadcastGlobalVariablesHook(0)),
trains on its own shard of the data and, each step, exchanges gradients:

``dense_dp`` (``parallelism=dense_dp``, always ``embedding_update=exact``)
    Horovod-faithful transport: the full-table L2 makes the fm_w/fm_v gradients dense,
    so the whole dense gradient — table + MLP in ONE flat bucket — is all-reduced and averaged
    (the 16.2 MB/step of the notebook config), then every rank applies the same
    dense optimizer update.

``dp`` (the default, either embedding update)
    Each rank reduces its lookups to (unique id, Σ grad row) pairs (emb_update.hip mode 2) and
    packs them next to its MLP gradient in one send buffer; ONE all-gather (the p2p push over
    xGMI, or RCCL) moves every rank's buffer to every rank; each rank then sums the MLP gradients
    over ranks in rank order and merges the gathered rows by direct addressing (rank order ⇒
    bitwise identical results on every rank).  ``sparse``: lazy L2 and the row optimizer on the
    touched rows.  ``exact``: the merged rows become this step's rows of the dense gradient table
    and every rank runs the dense full-table update (λ·θ on every row) — the same mathematics as
    dense_dp, because rows no rank touched have a zero data gradient on every rank, without
    moving the dense table.  Replicas stay bit-identical without a broadcast.

Gradients are averaged over ranks and the learning rate is scaled by the world size (HVD:171;
``lr_scaling``).  Both the fused HIP engine and the eager engine are supported.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..models.deepfm import ModelSpec
from ..optim import OptHParams


def collectives_capturable() -> bool:
    """RCCL collectives can be captured into HIP graphs (torch.distributed nccl backend); gloo's
    host-side collectives cannot.  ROCFM_GRAPH_COLLECTIVES=0 forces per-phase graphs."""
    if os.environ.get("ROCFM_GRAPH_COLLECTIVES", "1") == "0":
        return False
    return not dist.is_initialized() or dist.get_backend() == "nccl"


def _world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def force_collectives() -> bool:
    """ROCFM_FORCE_COLLECTIVES=1: with a process group of ONE rank, still run every exchange
    through the backend's collective (RCCL at world 1 copies through its own kernels) instead of
    the world-1 shortcut (alias / no-op).  Lets a one-GPU box capture and replay the exact RCCL
    calls (all_gather_into_tensor, all_to_all_single, all_reduce) the multi-GPU node runs."""
    return os.environ.get("ROCFM_FORCE_COLLECTIVES", "0") == "1" and dist.is_initialized()


def _all_gather_flat(out: torch.Tensor, inp: torch.Tensor) -> None:
    """all_gather into a [world*n] buffer; RCCL fast path, host-staged fallback for gloo."""
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, inp)
        return
    n = inp.numel()
    src = inp.detach().cpu()
    outs = [torch.empty_like(src) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, src)
    out.view(-1, n).copy_(torch.stack(outs))


def _all_reduce(t: torch.Tensor) -> None:
    if dist.get_backend() == "nccl" or t.device.type == "cpu":
        dist.all_reduce(t)
        return
    c = t.detach().cpu()
    dist.all_reduce(c)
    t.copy_(c)


# Up to this many ranks the merge binary-searches the sorted source lists (one launch, no maps);
# beyond it a scatter into position maps + apply is faster (tools/bench_merge.py on one MI355X,
# 7.5k keys per rank: W=1 3.9 vs 8.9 µs, W=2 9.8 vs 10.0, W=4 12.8 vs 10.0, W=8 20.6 vs 13.7)
SEARCH_MAX_W = 2
MERGE_MAP_BUDGET = 512 << 20  # bytes of direct-addressing merge maps ((W + 1) × V int32) before hashing


def range_merge_buckets(W: int, cap: int) -> int:
    """Key buckets of the range merge (merge.hip range mode, one workgroup each): ≈192 gathered
    entries per bucket on average, at least 64."""
    return max(64, -(-W * cap // 192))


# With bucket directories the search merge beats the position maps up to 4 ranks
# (tools/bench_merge.py, profiles/r3_session3_search_dir.md: W=2 7.6 vs maps 9.1 µs, W=4 9.5 vs
# 10.3, W=8 14.6 vs 14.2), so DP keeps the sorted export + search through W = 4.
SEARCH_DIR_MAX_W = 4


def merge_choice() -> str:
    """ROCFM_MERGE with ``noplan`` read as ``auto``: ``noplan`` is the automatic step-time merge
    (search ≤ 4 ranks, maps above) with the plan-ahead merge off — the A/B the N > 1 bench runs
    beside the default (``merge_noplan_*`` windows)."""
    m = os.environ.get("ROCFM_MERGE", "auto")
    return "auto" if m == "noplan" else m


def search_dir_buckets(W: int, V: int) -> int:
    """Key buckets of the directory the sorted DP export writes for the SEARCH merge (2 ≤ W ≤
    SEARCH_DIR_MAX_W): each entry's binary search in the other ranks' lists starts inside its
    key's bucket (≈log2(bucket) halvings instead of ≈log2(cap)): 10.2 → 7.6 µs at W = 2 with 8192
    buckets.  0 = off (ROCFM_SEARCH_DIR=0, one rank, or more than SEARCH_DIR_MAX_W ranks)."""
    if W < 2 or W > SEARCH_DIR_MAX_W or os.environ.get("ROCFM_SEARCH_DIR", "1") == "0":
        return 0
    if merge_choice() != "auto":  # a forced merge (direct / hash / range) is kept
        return 0
    return max(64, min(8192, V // 16))


# The plan-ahead merge (merge_plan.hip) from this many ranks on: the union of the ranks' exported
# ids and every id's position in every export are built on the side chain a graph ahead (the ids
# exchanged there), so the step's merge is one plan-driven gather-sum (ROCFM_MERGE=plan forces it,
# also over RCCL; any other forced merge keeps it off).  tools/bench_merge.py, uncached p2p
# memory: the step's apply 3.9 / 4.4 / 5.6 µs at W = 2 / 4 / 8 against 7.6 / 9.6 / 14.1 for the
# best step-time merge, for 2.9 / 3.5 / 5.7 µs per step of plan building on the side chain of a
# 16-step graph (profiles/r5_dp_plan_merge.md).  Default only beyond 4 ranks, where the step-time
# merge costs most (14 µs at W = 8): in the shared-GPU rehearsals (2 / 4 ranks on one GPU) the
# merge phase shrank but the headline loop ran slower with the plan's extra per-graph id exchange,
# and a shared GPU cannot say whether that carries over to one GPU per rank.
PLAN_MIN_W = 5


def plan_merge_enabled(W: int, exchange: str) -> bool:
    """By default with the p2p exchange (the ids ride a p2p exchange of their own); over RCCL (a
    side-chain all-gather in a process group of its own) only when forced."""
    m = os.environ.get("ROCFM_MERGE", "auto")
    return W >= 2 and (m == "plan" or (m == "auto" and W >= PLAN_MIN_W and exchange == "p2p"))


def range_merge_enabled(W: int) -> bool:
    """The range merge (bucket directories written by the sorted export; merge.hip range mode) for
    the multi-step DP path with ≥ 2 ranks — opt-in (ROCFM_MERGE=range).  Measured against the
    search / maps merges (profiles/r3_merge_range.md): no gain on Criteo-shape ids, whose
    field-clustered Zipf ids crowd a few key buckets; 8.6 vs 10.6 µs at W = 4 only when the keys
    are first spread by a bijective hash."""
    return W >= 2 and merge_choice() == "range"


class MergeMaps:
    """Row-merge lookup structures of merge.hip for W sources of ≤ cap unique keys over a table of
    ``rows`` rows.  Direct addressing ((W + 1) × rows int32 maps, the fastest: one load per source)
    while it fits MERGE_MAP_BUDGET, else a step-tagged linear-probing hash table of
    next_pow2(2·W·cap) slots — O(W·cap), independent of the vocabulary (1B-row tables).
    ``ROCFM_MERGE=direct|hash`` forces one (tests)."""

    def __init__(self, W: int, cap: int, rows: int, device):
        choice = merge_choice()
        if choice not in ("auto", "direct", "hash", "range", "plan"):
            raise ValueError(f"ROCFM_MERGE must be auto, noplan, direct, hash, range or plan, got {choice!r}")
        direct_bytes = (W + 1) * rows * 4
        # (plan: the multi-step graphs merge by the plan; the per-step path keeps the automatic maps)
        self.hashed = choice == "hash" or (choice in ("auto", "plan") and direct_bytes > MERGE_MAP_BUDGET)
        i32 = dict(dtype=torch.int32, device=device)
        if self.hashed:
            self.slots = 1 << max(4, math.ceil(math.log2(max(2 * W * cap, 2))))
            self.hkeys = torch.zeros(self.slots, dtype=torch.int64, device=device)
            self.hrep = torch.zeros(self.slots, dtype=torch.int64, device=device)
            self.hpos = torch.zeros(self.slots * W, dtype=torch.int64, device=device)
            self.pos = self.rep = torch.zeros(1, **i32)  # unused
        else:
            self.slots = 0
            self.pos = torch.empty(W * rows, **i32)
            self.rep = torch.empty(rows, **i32)

    def bind(self, mp) -> None:
        mp.pos, mp.rep = self.pos.data_ptr(), self.rep.data_ptr()
        mp.hash_slots = self.slots
        if self.hashed:
            mp.hkeys, mp.hrep, mp.hpos = self.hkeys.data_ptr(), self.hrep.data_ptr(), self.hpos.data_ptr()

    def reset(self) -> None:
        """Forget every tag (the step counter went backwards: a checkpoint restore)."""
        if self.hashed:
            for t in (self.hkeys, self.hrep, self.hpos):
                t.zero_()

    def nbytes(self) -> int:
        ts = (self.hkeys, self.hrep, self.hpos) if self.hashed else (self.pos, self.rep)
        return sum(t.numel() * t.element_size() for t in ts)


def pool_exchange_capacity(pool_ids: torch.Tensor, owners: int = 1) -> int:
    """Exact exchange capacity for training on a known batch pool ([NB, B, F] ids): the largest
    number of unique ids in any batch (``owners`` > 1: per owner ``id % owners``, the row-shard
    request lists), MAX-reduced over ranks so every rank builds identical collective shapes."""
    m = 1
    for b in pool_ids:
        u = torch.unique(b)
        c = int(torch.bincount((u % owners).long(), minlength=owners).max()) if owners > 1 else int(u.numel())
        m = max(m, c)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dev = pool_ids.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([m], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        m = int(t.item())
    return m


# ================================================================================================
# eager engine hooks (CPU/gloo tests, PyTorch baseline)
# ================================================================================================
def attach_torch_dp(eng, embedding_update: str = "sparse") -> None:
    """Install gradient-exchange hooks on a TorchDeepFM (rocfm.models.torch_engine)."""
    world = _world()
    if world == 1:
        return

    def allreduce_dense(grads: Dict[str, torch.Tensor]) -> None:
        names = sorted(grads)
        flat = torch.cat([grads[k].reshape(-1) for k in names])
        dist.all_reduce(flat)
        flat /= world
        off = 0
        for k in names:
            n = grads[k].numel()
            grads[k].copy_(flat[off:off + n].view_as(grads[k]))
            off += n

    def exchange_rows(uniq: torch.Tensor, gw: torch.Tensor, gv: torch.Tensor):
        dev = uniq.device
        n = torch.tensor([uniq.numel()], dtype=torch.int64, device=dev)
        ns = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(ns, n)
        cap = int(max(int(x) for x in ns))
        K = gv.shape[1]
        pack = torch.zeros(cap, K + 2, dtype=torch.float64, device=dev)
        pack[: uniq.numel(), 0] = uniq.double()
        pack[: uniq.numel(), 1] = gw.double()
        pack[: uniq.numel(), 2:] = gv.double()
        bufs = [torch.zeros_like(pack) for _ in range(world)]
        dist.all_gather(bufs, pack)
        rows = torch.cat([b[: int(c)] for b, c in zip(bufs, ns)])  # rank-major, deterministic
        ids = rows[:, 0].long()
        u, inv = torch.unique(ids, return_inverse=True)
        acc = torch.zeros(len(u), K + 1, dtype=torch.float64, device=dev)
        acc.index_add_(0, inv, rows[:, 1:])
        acc /= world
        return u, acc[:, 0].float(), acc[:, 1:].float()

    eng.allreduce_dense = allreduce_dense
    if embedding_update != "exact":
        eng.exchange_rows = exchange_rows


def shadow_prefix(w, batches, after_steps=None, with_prefix: bool = False):
    """Train the shadow-validation window of a distributed fused engine ``w`` (its first p2p steps,
    per step with the collective shadow) from the head of a host batch stream.  Returns (the rest
    of the stream, steps trained) — and, ``with_prefix``, the trained batches as device tensors
    ``(ids [n,B,F], vals, labels)`` or None, which ``FusedDeepFM.train_stream(prefix=…)`` puts at
    the head of its HBM ring (so the ring of an epoch holds the whole epoch: the HBM epoch cache).
    Items are single batches, stacked groups or RawGroups, as in FusedDeepFM.train_stream; a group
    that straddles the window's end is split."""
    import itertools

    from ..data.tfrecord import RawGroup
    from ..ops.decode import PARSE_STATUS, decode_on_device

    shadow = getattr(w, "shadow", None)
    if shadow is None or not shadow.active:
        return (batches, 0, None) if with_prefix else (batches, 0)
    it = iter(batches)
    dev = w.eng.device
    got, rest = [], []
    while len(got) < shadow.left:
        b = next(it, None)
        if b is None:
            break
        if isinstance(b, RawGroup):  # undecoded batches: parsed on the device for the shadow steps
            k = min(b.n, shadow.left - len(got))
            ids, vals, labels, err = decode_on_device(b.bytes, b.offs, k, b.B, w.eng.F, dev, w.eng.id_limit,
                                                      getattr(w.eng, "decode_keys", ("label", "ids", "values")))
            if int(err[0]):
                raise RuntimeError(f"decode error in batch {int(err[1])} record {int(err[2])} (device parse): "
                                   f"{PARSE_STATUS.get(int(err[0]))}")
            got += [(ids[i], vals[i], labels[i]) for i in range(k)]
            if k < b.n:
                rest.append(RawGroup(b.bytes[k:].clone(), b.offs[k:].clone(), b.n - k, b.B))
            continue
        ids, vals, labels = b
        if ids.dim() == 2:
            ids, vals, labels = ids.unsqueeze(0), vals.unsqueeze(0), labels.unsqueeze(0)
        k = min(ids.shape[0], shadow.left - len(got))
        for i in range(k):
            got.append((ids[i].to(dev), vals[i].to(dev), labels[i].to(dev)))
        if k < ids.shape[0]:  # the rest of this group is trained by the stream (own host copy)
            rest.append((ids[k:].clone(), vals[k:].clone(), labels[k:].clone()))
    if not got:
        return (itertools.chain(rest, it), 0, None) if with_prefix else (itertools.chain(rest, it), 0)
    e = w.eng
    i0 = e._i
    pre = (torch.stack([g[0] for g in got]), torch.stack([g[1] for g in got]), torch.stack([g[2] for g in got]))
    w.attach_pool(*pre, start=(-i0) % len(got))
    for _ in got:
        w.train_step()
    if after_steps is not None:
        after_steps(i0, len(got))
    if with_prefix:
        return itertools.chain(rest, it), len(got), pre
    return itertools.chain(rest, it), len(got)


# ================================================================================================
# fused engine
# ================================================================================================
class FusedDataParallel:
    """Data-parallel wrapper around one FusedDeepFM per rank (one GPU per process)."""

    def __init__(self, spec: ModelSpec, hp: OptHParams, batch_size: int, device, params=None,
                 embedding_update: str = "sparse", mode: str = "dp", seed: int = 1234, use_graph: bool = True,
                 capacity: Optional[int] = None, check_every: int = 256, compute_dtype: str = "bf16",
                 exchange: Optional[str] = None, table_dtype: str = "f32"):
        from ..models.fused import FusedDeepFM

        self.world = _world()
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        if mode not in ("dp", "dense_dp"):
            raise ValueError(f"FusedDataParallel mode must be dp or dense_dp, got {mode}")
        if mode == "dense_dp" and embedding_update != "exact":
            embedding_update = "exact"
        self.mode = mode
        self.exact = embedding_update == "exact"
        self.eng = FusedDeepFM(spec, hp, batch_size, device, embedding_update=embedding_update, seed=seed,
                               params=params, use_graph=False, fuse_dense_opt=False,
                               dropout_seed=seed + 7919 * self.rank, compute_dtype=compute_dtype,
                               table_dtype=table_dtype)
        e = self.eng
        if e._hazard is not None:  # ROCFM_HAZARD=1: this driver's buffers join the checked set
            e._hazard.attach("dp", self)
        self.use_graph = use_graph
        self.graph_collectives = use_graph and collectives_capturable()
        self.check_every = int(check_every)
        self.device = e.device
        self.p2p = None
        self.force = force_collectives()
        self.exchange = "rccl"  # DP all-gather transport (mode dp: p2p.open_exchanges may pick "p2p")
        self.range = False  # range merge (mode dp, set below)
        self.sdir = False  # bucket directory for the search merge (mode dp, set below)
        # replicas start identical: broadcast rank 0's variables (HVD:418)
        if self.world > 1:
            from .dist import broadcast_tensors

            broadcast_tensors([e.emb, e.dense] + list(e.emb_slots) + list(e.dense_slots))
            e.refresh_bf16()
        P = e.layout.total
        H = e.H
        if mode == "dense_dp":
            # one flat bucket: [dense table grad (V*Kp) | MLP grads (P)]
            self.bucket = torch.zeros(e.V * e.Kp + P, dtype=torch.float32, device=e.device)
            e.dense_grad = self.bucket[: e.V * e.Kp].view(e.V, e.Kp)
            e.touched = None  # every row's gradient comes from the all-reduce
            e.dense_grads_flat = self.bucket[e.V * e.Kp:]
            e._build_params()
            for p in range(2):
                e.emb_dense_params[p].grad_scale = 1.0 / self.world
                e.dense_apply_params[p].grad_scale = 1.0 / self.world
                e.dense_apply_params[p].apply = 1
        else:
            cap = (int(capacity or e.n_lookup) + 3) // 4 * 4  # keeps every row 16-B aligned
            self.cap = cap
            Kp = e.Kp
            # range merge (multi-step path): the sorted export also writes a bucket directory
            self.range = range_merge_enabled(self.world) and Kp <= H.tail_max_kp()
            # search merge (W ≤ SEARCH_MAX_W, multi-step path): the directory narrows the searches
            self.sdir = (not self.range and mode == "dp" and Kp <= H.tail_max_kp()
                         and search_dir_buckets(self.world, e.V) > 0)
            self.nb = (range_merge_buckets(self.world, cap) if self.range
                       else search_dir_buckets(self.world, e.V) if self.sdir else 0)
            self.bdiv = -(-e.V // self.nb) if self.nb else 0
            ndir = (self.nb + 1 + 3) // 4 * 4 if self.nb else 0
            # send buffer (f32 words): [MLP grads P | pad to 4 | count (int32) + pad 3 | dir nb+1 (int32,
            # range merge) | keys cap (int32) | rows cap*Kp]  (every part from the count on 16-B aligned)
            self.off_cnt = (P + 3) // 4 * 4
            self.off_dir = self.off_cnt + 4
            self.off_keys = self.off_dir + ndir
            self.off_rows = self.off_keys + cap
            self.S = (self.off_rows + cap * Kp + 3) // 4 * 4  # float4 payload (p2p push)
            self.send = torch.zeros(self.S, dtype=torch.float32, device=e.device)
            from .p2p import open_exchanges

            exs = open_exchanges([self.S], self.device, exchange)  # transport: p2p push or RCCL
            self.p2p = exs[0] if exs else None
            # fused push (p2p only): the tail's producers store the MLP gradients and the exported
            # rows straight into every rank's receive slot, so the xGMI transfer overlaps the tail;
            # the push launch then carries only the row count + hand-off (ROCFM_DP_PUSH, see
            # p2p.producer_push_enabled)
            self.push_target = None  # fused_push below
            if self.p2p is not None:  # rank slots live in the uncached, peer-mapped receive buffer
                self.exchange = "p2p"
                self.graph_collectives = use_graph  # the push kernel is capturable whatever the backend
                self.recv = None
                self._recv_ptr = self.p2p.recv_ptr
                from .p2p import producer_push_enabled

                if producer_push_enabled(self.p2p):
                    self.push_target = self.p2p.push_target()
                    self.p2p_params = self.p2p.params(self.send[self.off_cnt:].data_ptr(), 4,
                                                      dst_offset_floats=self.off_cnt)
                else:
                    self.p2p_params = self.p2p.params(self.send.data_ptr(), self.S)
            else:  # one rank: the gathered list IS the send buffer (no copy)
                self.recv = (torch.zeros(self.world * self.S, dtype=torch.float32, device=e.device)
                             if self.world > 1 or self.force else self.send)
                self._recv_ptr = self.recv.data_ptr()
            e.dense_grads_flat = self.send[:P]
            self.send_count = self.send[self.off_cnt:self.off_cnt + 4].view(torch.int32)
            # merge maps (merge.hip): position of each key in every rank's list, representative rank
            # (direct addressing, or a W·cap hash table for very large vocabularies)
            self.maps = MergeMaps(self.world, cap, e.V, e.device)
            self.overflow = torch.zeros(1, dtype=torch.int32, device=e.device)
            e._build_params()
            self.export_params, self.merge_params = [], []
            for p in range(2):
                ex = H.EmbUpdateParams()
                src = e.emb_params[p]
                ex.skeys, ex.svals, ex.n, ex.contrib = src.skeys, src.svals, src.n, src.contrib
                ex.n_dev, ex.sorted_contrib, ex.chunk_end = src.n_dev, src.sorted_contrib, src.chunk_end
                ex.K1, ex.Kp, ex.opt, ex.step = e.K1, e.Kp, src.opt, src.step
                ex.mode = 2
                ex.grad_scale = 1.0
                ex.out_keys = self.send[self.off_keys:].data_ptr()
                ex.out_rows = self.send[self.off_rows:].data_ptr()
                ex.out_count = self.send[self.off_cnt:].data_ptr()
                ex.out_cap = cap
                self._set_push(e.rows_params[p], e.wgrad_params[p], ex)
                self.export_params.append(ex)
                mp_ = H.MergeParams()  # merge the gathered lists: Σ over ranks per id → row optimizer
                mp_.keys = self._recv_ptr + 4 * self.off_keys
                mp_.rows = self._recv_ptr + 4 * self.off_rows
                mp_.counts = self._recv_ptr + 4 * self.off_cnt
                mp_.key_stride = mp_.row_stride = mp_.count_stride = self.S
                mp_.W, mp_.cap, mp_.Kp, mp_.K1 = self.world, cap, Kp, e.K1
                mp_.key_div, mp_.Vmap = 1, e.V
                self.maps.bind(mp_)
                mp_.emb, mp_.tbl_bf16 = e.emb.data_ptr(), e.tbl_bf16
                mp_.s0, mp_.s1 = e._slot_ptrs(e.emb_slots)
                mp_.l2, mp_.grad_scale = float(spec.l2_reg), 1.0 / self.world
                mp_.opt, mp_.step = e._opt(p), e.steps[p:].data_ptr()
                mp_.mode = 0
                if self.exact:  # merged rows → the dense gradient table, then the full-table update
                    mp_.mode, mp_.dense_grad, mp_.touched = 1, e.dense_grad.data_ptr(), e.touched.data_ptr()
                    e.emb_dense_params[p].grad_scale = 1.0  # the merge applied 1/W
                mp_.overflow = self.overflow.data_ptr()
                self.merge_params.append(mp_)
                da = e.dense_apply_params[p]
                da.apply, da.grads, da.grad_scale = 1, self._recv_ptr, 1.0 / self.world
                da.nseg, da.seg_stride = self.world, self.S
            H.merge_init(self.merge_params[0], e.stream_ptr)
        for p in range(2):
            e.wgrad_params[p].grads = e.dense_grads_flat.data_ptr()
        self._graphs = {}
        self._warm = 0
        # self-validation (rocfm.parallel.validate): the first steps of a p2p run are shadowed by
        # the collective; replica digests in check()
        from .validate import Shadow, fault_rank

        self.shadow = Shadow(e.device, steps=None if (self.p2p is not None and self.world > 1) else 0)
        self.shadow.corrupt = fault_rank("corrupt_push", self.rank)
        self._set_mirror(self.shadow.active)
        self._shadow_buf = torch.zeros(self.world * self.S, dtype=torch.float32, device=e.device) \
            if self.shadow.active else None
        self._corrupt_replica = fault_rank("corrupt_replica", self.rank)

    @property
    def fused_push(self) -> bool:
        """True when the tail's producers push into the peers' receive slots themselves."""
        return getattr(self, "push_target", None) is not None

    def _set_push(self, rows, wp, ex) -> None:
        """Point one step's producers at the receive slots (fused push; no-op otherwise)."""
        t = getattr(self, "push_target", None)
        if t is None:
            return
        rows.push = t  # workgroup 0 of the row kernel signals "entered"
        wp.push = t
        ex.push = t
        ex.push_off_keys, ex.push_off_rows = self.off_keys, self.off_rows

    # ---- batch feeding (delegated) ------------------------------------------------------------
    def attach_pool(self, ids, vals, labels, start: int = 0):
        self.eng.attach_pool(ids, vals, labels, start)
        self._graphs = {}

    def push_batch(self, ids, vals, labels):
        self.eng.push_batch(ids, vals, labels)

    def load_batch(self, ids, vals, labels=None):
        self.eng.load_batch(ids, vals, labels)

    def set_lr_scale(self, s: float) -> None:
        self.eng.set_lr_scale(s)
        if self.mode == "dp":
            for p in range(2):
                self.export_params[p].opt = self.eng.emb_params[p].opt
                self.merge_params[p].opt = self.eng._opt(p)
        self._graphs = {}

    # ---- step phases ---------------------------------------------------------------------------
    def _phase_a(self, p: int, join_side: bool = True):
        e = self.eng
        side = e._fork_next(p)  # forked first: its own hardware queue in the graph (see FusedDeepFM)
        self.send_count.zero_() if self.mode == "dp" else None
        aux = e._enqueue_rows_then_fork_wgrad(p)
        s = e.stream_ptr
        if self.mode == "dense_dp":
            e.H.emb_rows_update(e.emb_params[p], s)  # mode 1: Σ rows → dense grad table
        else:
            e.H.emb_rows_update(self.export_params[p], s)
        e._join(aux)
        if join_side:
            e._join(side)
        return side

    def _exchange(self):
        if self.p2p is not None:  # fused push: only the row count + the data hand-off are left
            self.p2p.push(self.p2p_params)
            if self.shadow.active:
                self._shadow_exchange()
            return
        if self.world == 1 and not self.force:  # one rank: recv aliases send (dp) / the bucket is the sum
            return
        if self.mode == "dense_dp":
            _all_reduce(self.bucket)
        else:
            _all_gather_flat(self.recv, self.send)

    def _phase_b(self, p: int):
        e = self.eng
        s = e.stream_ptr
        if self.mode == "dense_dp":
            e.H.dense_apply(e.dense_apply_params[p], s)
            e.H.emb_dense_update(e.emb_dense_params[p], s)
            return
        # MLP: Σ over the gathered rank segments (rank order) + optimizer as extra workgroups of
        # the row-scatter launch, then the row merge + optimizer (exact: + the dense table update)
        e.H.merge_scatter_dense(self.merge_params[p], e.dense_apply_params[p], s)
        e.H.merge_apply(self.merge_params[p], s)
        if self.exact:
            e.H.emb_dense_update(e.emb_dense_params[p], s)

    def _run(self, key, fn, collectives: bool = False):
        if not self.use_graph or self._warm < 4 or self.shadow.active:
            fn()
            return
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.device)
            # graphs that contain RCCL collectives: other threads (the PG watchdog) may query
            # events while this thread captures
            with torch.cuda.graph(g, capture_error_mode="thread_local" if collectives else "global"):
                fn()
            self._graphs[key] = g
        g.replay()

    def _step_body(self, p: int) -> None:
        side = self._phase_a(p, join_side=False)  # next batch's fetch+sort overlaps the exchange
        self._exchange()
        self._phase_b(p)
        self.eng._join(side)

    def _after_steps(self, i0: int, i1: int) -> None:
        if self.check_every and i1 // self.check_every != i0 // self.check_every:
            self.check()

    def train_step(self) -> None:
        e = self.eng
        e._m_primed = False
        if not e._primed:
            e.prime()
        p = e._i % 2
        if self.graph_collectives:  # the whole step, collective included, is one graph
            self._run(("step", p), lambda: self._step_body(p), collectives=True)
        else:
            self._run(("a", p), lambda: self._phase_a(p))
            self._exchange()
            self._run(("b", p), lambda: self._phase_b(p))
        self._warm += 1
        e._i += 1
        if self.shadow.step_done():
            self._shadow_finish()
        self._after_steps(e._i - 1, e._i)

    # ---- self-validation (rocfm.parallel.validate) ----------------------------------------------
    def _set_mirror(self, on: bool) -> None:
        """Fused push: while the shadow window is open the producers also write their results to
        the local send buffer (MLP gradients, exported keys / rows / directory), so the shadow's
        reference is what each producer computed, not what landed in a receive slot."""
        m = 1 if (on and self.fused_push) else 0
        for p in range(2):
            self.eng.wgrad_params[p].push_mirror = m
            if self.mode == "dp":
                self.export_params[p].push_mirror = m

    def _shadow_exchange(self) -> None:
        """The p2p all-gather just delivered every rank's slot: all-gather every rank's LOCAL send
        buffer (what its producers computed: the copy push's source, or the fused push's mirror)
        through the collective as well, compare bitwise, and let the merge consume the
        collective's copy.  A producer that pushed wrong bytes to every slot — a wrong offset, a
        wrong directory value — therefore mismatches too, not only a transfer that corrupted one
        receiver's copy."""
        got = self.p2p.recv_tensor(torch.float32, (self.world * self.S,))
        self.shadow.corrupt_(got)
        _all_gather_flat(self._shadow_buf, self.send)
        self.shadow.compare(got, self._shadow_buf)

    def _shadow_finish(self) -> None:
        if self.shadow.finish():
            msg = (f"exchange: p2p result differed from the collective in the first "
                   f"{self.shadow.compared} validated exchanges on some rank; falling back to RCCL")
            import logging

            logging.getLogger("rocfm").warning(msg)
            if self.rank == 0:
                print(f"[rocfm] {msg}", flush=True)
            self._fallback_to_collective()
        self._shadow_buf = None
        self._set_mirror(False)

    def _fallback_to_collective(self) -> None:
        """Agreed switch from the p2p push to the process group's all-gather (every rank)."""
        e, H = self.eng, self.eng.H
        torch.cuda.synchronize(self.device)
        self._graphs = {}
        self._m_dp_S = None
        self.p2p.close()
        self.p2p = None
        self.push_target = None
        self.exchange = "rccl"
        self.graph_collectives = self.use_graph and collectives_capturable()
        self.recv = torch.zeros(self.world * self.S, dtype=torch.float32, device=e.device)
        self._recv_ptr = self.recv.data_ptr()
        for p in range(2):
            for prm in (e.rows_params[p], e.wgrad_params[p], self.export_params[p]):
                prm.push = H.PushTarget()
            mp_ = self.merge_params[p]
            mp_.keys = self._recv_ptr + 4 * self.off_keys
            mp_.rows = self._recv_ptr + 4 * self.off_rows
            mp_.counts = self._recv_ptr + 4 * self.off_cnt
            e.dense_apply_params[p].grads = self._recv_ptr

    def replicated_tensors(self):
        e = self.eng
        return [e.dense, e.emb, e.steps] + list(e.dense_slots) + list(e.emb_slots)

    def verify_replicas(self) -> bool:
        """Collective: every rank's replica (MLP, tables, optimizer slots, step) is bit-identical."""
        if self.world == 1:
            return True
        torch.cuda.synchronize(self.device)
        if self._corrupt_replica:  # fault injection (tests): one rank's replica drifts
            self._corrupt_replica = False
            self.eng.dense.view(-1)[0] += 1e-3
        from .validate import replicas_agree

        return replicas_agree(self.replicated_tensors())

    # ---- multi-step graphs (pool mode, capturable collectives) -----------------------------------
    # The single-GPU pipeline of FusedDeepFM (serial main stream per step, one batched fetch+sort
    # side chain per graph, sorted-order gradient rows) with the step's exchange captured inline:
    #   dp       rows → tail(wgrad grads ‖ export Σrows) → all_gather → dense_apply(Σ ranks) → merge
    #   dense_dp rows → tail(wgrad grads ‖ Σrows → dense table grad) → all_reduce → dense_apply
    #            → emb_dense_update
    def _build_multi_dp(self, Smax: int) -> None:
        e, H = self.eng, self.eng.H
        self._graphs = {}  # captured graphs hold the previous parameter blocks / buffers
        # sorted export (the fused tail's chunks, run heads counted on the side chain) → the merge
        # needs no maps: one search-mode launch (merge.hip) after the exchange
        # (not with the per-tile dedup: its export lists come from the compacted groups, whose chunk
        # heads the plan's unique-id pass does not read)
        self.m_plan = (self.mode == "dp" and e.Kp <= H.tail_max_kp() and not e.dedup
                       and plan_merge_enabled(self.world, self.exchange))
        self.m_sorted = self.mode == "dp" and e.Kp <= H.tail_max_kp() and (self.world <= SEARCH_MAX_W or self.range
                                                                            or self.sdir or self.m_plan)
        e._build_multi(Smax, heads=self.m_sorted)
        e._m_pool = e.pool_ids
        S_, n = e.mS, e.n_lookup
        if self.m_plan:
            self._build_plan(S_)
        self.m_dp = []
        for q in range(2):
            row = []
            for k in range(S_):
                rows, wp, da, ep, ed = e.m_params[q][k]
                wp.grads = e.dense_grads_flat.data_ptr()
                da.apply, da.grad_scale = 1, 1.0 / self.world
                if self.mode == "dense_dp":
                    da.grads = e.dense_grads_flat.data_ptr()
                    ed.grad_scale = 1.0 / self.world
                    row.append((rows, wp, ep, da, ed, None))
                    continue
                da.grads, da.nseg, da.seg_stride = self._recv_ptr, self.world, self.S
                ex = H.EmbUpdateParams()  # export: compacted (id, Σ grad row) into the send buffer
                ex.skeys, ex.svals, ex.n, ex.n_dev = ep.skeys, ep.svals, n, ep.n_dev
                ex.val_base, ex.id_offset, ex.sorted_contrib, ex.chunk_end = ep.val_base, ep.id_offset, 1, ep.chunk_end
                ex.contrib, ex.K1, ex.Kp = e.contrib.data_ptr(), e.K1, e.Kp
                ex.opt, ex.step = ep.opt, ep.step
                ex.mode, ex.grad_scale = 2, 1.0
                ex.out_keys = self.send[self.off_keys:].data_ptr()
                ex.out_rows = self.send[self.off_rows:].data_ptr()
                ex.out_count = self.send[self.off_cnt:].data_ptr()
                ex.out_cap = self.cap
                if self.m_sorted:
                    ex.chunk_heads, ex.nch = e.m_chd[q, k * e.m_nch:].data_ptr(), e.m_nch
                if self.range or (self.sdir and self.m_sorted):  # + the bucket directory of the exported keys
                    ex.dir_nb, ex.dir_div = self.nb, self.bdiv
                    ex.out_dir, ex.push_off_dir = self.send[self.off_dir:].data_ptr(), self.off_dir
                self._set_push(rows, wp, ex)
                mg = H.MergeParams()
                src = self.merge_params[0]
                for f in ("keys", "rows", "counts", "key_stride", "row_stride", "count_stride", "W", "cap", "Kp",
                          "K1", "key_div", "Vmap", "pos", "rep", "emb", "s0", "s1", "l2", "grad_scale", "mode",
                          "overflow", "dense_grad", "touched", "hash_slots", "hkeys", "hrep", "hpos", "tbl_bf16"):
                    setattr(mg, f, getattr(src, f))
                mg.opt, mg.step = ep.opt, ep.step  # this step's global_step / lr_t
                if self.range or (self.sdir and self.m_sorted):
                    mg.dirs, mg.dir_stride = self._recv_ptr + 4 * self.off_dir, self.S
                    mg.nb, mg.bucket_div = self.nb, self.bdiv
                rows.zero_word = self.send[self.off_cnt:].data_ptr()
                if ed is not None:
                    ed.grad_scale = 1.0  # the merge applied 1/W
                row.append((rows, wp, ex, da, ed if self.exact else None, mg))
            self.m_dp.append(row)
        self._m_dp_S = Smax

    def _enqueue_multi_dp(self, q: int, S: int) -> None:
        """Main chain of one S-step DP graph (the side graph is launched by FusedDeepFM._launch_multi)."""
        e, H = self.eng, self.eng.H
        s = torch.cuda.current_stream(self.device).cuda_stream
        v = getattr(self, "_variant", None)  # phase_windows: a truncated step (diagnostic only)
        for k in range(S):
            rows, wp, ep, da, ed, mg = self.m_dp[q][k]
            H.deepfm_rows(rows, s)  # (dp: also zeroes the export counter)
            if v == "rows":
                continue
            e._tail(wp, ep, None, s)
            if v == "compute":
                continue
            if v is None:
                self._exchange()
            if self.mode == "dp" and self.range:
                H.merge_range_apply(mg, da, s)  # bucketed row merge ‖ MLP optimizer, one launch
                if ed is not None:
                    H.emb_dense_update(ed, s)
            elif self.mode == "dp" and self.m_plan:
                H.merge_plan_apply(mg, self.plan_steps[q][k], da, s)  # plan-driven gather-sum ‖ MLP optimizer
                if ed is not None:
                    H.emb_dense_update(ed, s)
            elif self.mode == "dp" and self.m_sorted:
                H.merge_search_apply(mg, da, s)  # row merge ‖ MLP optimizer, one launch
                if ed is not None:
                    H.emb_dense_update(ed, s)
            elif self.mode == "dp":
                H.merge_scatter_dense(mg, da, s)  # row scatter ‖ MLP optimizer, one launch
                H.merge_apply(mg, s)
                if ed is not None:
                    H.emb_dense_update(ed, s)
            else:
                H.dense_apply(da, s)
                H.emb_dense_update(ed, s)

    # ---- plan-ahead merge (merge_plan.hip) -------------------------------------------------------
    def _build_plan(self, S: int) -> None:
        """Buffers of the plan-ahead merge for S-step graphs, and its side-chain hook: after the
        side chain has sorted the next graph's batches, this rank's unique ids of each batch (the
        rows its sorted export will write, in that order) go to every rank; every rank then builds
        the same plan — for each step, the union of the W ranks' ids and each id's position in
        every rank's export.  Outputs by graph parity: the side graph of parity q fills 1-q."""
        e, H = self.eng, self.eng.H
        W, cap, dev = self.world, self.cap, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        Sp = (S + 3) // 4 * 4
        self.plan_S, self.plan_Sp = S, Sp
        self.plan_slot = (Sp + S * cap + 3) // 4 * 4  # [S counts | pad | S lists of cap ids] (4-B words)
        self.plan_send = torch.zeros(self.plan_slot, dtype=torch.float32, device=dev)
        self.plan_ex = None
        if self.exchange == "p2p":  # the ids ride a p2p exchange of their own (collective to open)
            from .p2p import open_exchanges

            if getattr(self, "_plan_ex_open", None) is None or self._plan_ex_open.slot < self.plan_slot:
                if getattr(self, "_plan_ex_open", None) is not None:
                    self._plan_ex_open.close()
                exs = open_exchanges([self.plan_slot], dev, "p2p")
                self._plan_ex_open = exs[0]
            self.plan_ex = self._plan_ex_open
            self.plan_recv_ptr = self.plan_ex.recv_ptr
            self.plan_gstride = self.plan_ex.slot
        else:  # RCCL: a group of its own, so the side chain's all-gather never interleaves with the step's
            if getattr(self, "plan_group", None) is None:
                self.plan_group = dist.new_group(list(range(W))) if dist.is_initialized() else None
            self.plan_recv = torch.zeros(W * self.plan_slot, dtype=torch.float32, device=dev)
            self.plan_recv_ptr = self.plan_recv.data_ptr()
            self.plan_gstride = self.plan_slot
        seg = W * cap
        self.plan_scratch = [torch.zeros(S * seg, **i32) for _ in range(3)]  # sort input, sorted keys, values
        self.plan_tiles = torch.zeros(H.plan_tile_ints(S, W, cap), **i32)
        self.plan_bits = max(1, int(e.V).bit_length())  # the pad key V sorts after every id
        self.plan_temp = torch.zeros(max(16, H.plan_sort_temp_bytes(S, W, cap, self.plan_bits)), dtype=torch.uint8,
                                     device=dev)
        self.plan_rows = torch.zeros(2, S * seg, **i32)
        self.plan_pos = torch.zeros(2, S * seg * W, **i32)
        self.plan_cnt = torch.zeros(2, Sp, **i32)
        self.plan_steps = []
        for q in range(2):
            row = []
            for k in range(S):
                ps = H.PlanStep()
                ps.rows = self.plan_rows[q, k * seg:].data_ptr()
                ps.pos = self.plan_pos[q, k * seg * W:].data_ptr()
                ps.count = self.plan_cnt[q, k:].data_ptr()
                row.append(ps)
            self.plan_steps.append(row)
        e._m_post = self._plan_post

    def _plan_post(self, qo: int, stream) -> None:
        """Side chain (or the prime, on the main stream): the plan of the graph of parity qo."""
        e, H = self.eng, self.eng.H
        s = stream.cuda_stream
        S, Sp, cap, W = self.plan_S, self.plan_Sp, self.cap, self.world
        send = self.plan_send.data_ptr()
        pp = H.PlanParams()
        pp.S, pp.W, pp.cap = S, W, cap
        pp.skeys, pp.chunk_heads = e.m_sk[qo].data_ptr(), e.m_chd[qo].data_ptr()
        pp.n, pp.chunk, pp.nch = e.n_lookup, e.m_chunk, e.m_nch
        pp.id_shift = e.m_idbits if e.m_composite else 0  # the export's ids: key − id_offset
        pp.ukeys, pp.ukey_stride = send + 4 * Sp, cap
        pp.ucount, pp.ucount_stride = send, 1
        pp.overflow = self.overflow.data_ptr()
        H.uniq_keys(pp, s)
        if self.plan_ex is not None:
            self.plan_ex.push(self.plan_ex.params(send, self.plan_slot), s)
        elif dist.is_initialized() and (W > 1 or self.force):
            with torch.cuda.stream(stream):
                dist.all_gather_into_tensor(self.plan_recv, self.plan_send, group=self.plan_group)
        else:
            self.plan_recv[: self.plan_slot].copy_(self.plan_send)
        r0 = self.plan_recv_ptr
        pp.gkeys, pp.gcounts = r0 + 4 * Sp, r0
        pp.gk_stride = pp.gc_stride = self.plan_gstride
        pp.gkey_step, pp.gcount_step = cap, 1
        pp.pad_key = e.V
        pp.pkeys, pp.skeys_sorted, pp.svals_sorted = (t.data_ptr() for t in self.plan_scratch)
        pp.tile_counts = self.plan_tiles.data_ptr()
        pp.plan_rows, pp.plan_pos, pp.plan_count = (self.plan_rows[qo].data_ptr(), self.plan_pos[qo].data_ptr(),
                                                    self.plan_cnt[qo].data_ptr())
        H.plan_build(pp, self.plan_temp.data_ptr(), self.plan_temp.numel(), self.plan_bits, s)

    def _train_steps_multi(self, n: int, Smax: int) -> None:
        e = self.eng
        if getattr(self, "_m_dp_S", None) != Smax or getattr(e, "_m_pool", None) is not e.pool_ids:
            self._build_multi_dp(Smax)
        if not e._m_primed:
            e._prime_multi()
        while n > 0:
            S = min(n, e.mS)
            e._launch_multi(self._graphs, ("mdp",), S, self._enqueue_multi_dp, capture_error_mode="thread_local")
            n -= S
            self._after_steps(e._i - S, e._i)
        torch.cuda.current_stream(self.device).wait_stream(e.sort_stream)
        e._primed = False

    def phase_windows(self, steps: int = 64, steps_per_graph: int = 16) -> Dict[str, Dict[str, float]]:
        """Per-rank device time of the multi-step DP step's phases, min / max over ranks (ms/step).

        Diagnostic, run AFTER a measurement (it trains on stale exchange data and may leave the
        replicas inconsistent): truncated variants of the step graph are replayed ``steps`` times
        each — rows only; rows + tail (wgrad ‖ embedding export); + the merge (row merge ‖ MLP
        optimizer) without the exchange; the full step — and the phase times are their
        differences: rows, tail, merge, exchange (push / all-gather incl. the wait for the
        slowest peer).  Collective: every rank must call it."""
        e = self.eng
        if self.mode != "dp" or not (self.graph_collectives and self.use_graph) or self.shadow.active:
            raise RuntimeError("phase_windows needs the multi-step DP graphs (mode dp, capturable exchange)")
        S = int(steps_per_graph)
        if getattr(self, "_m_dp_S", None) != S or getattr(e, "_m_pool", None) is not e.pool_ids:
            self._build_multi_dp(S)
        if not e._m_primed:
            e._prime_multi()
        t = {}
        try:
            for v in ("rows", "compute", "merge", None):
                self._variant = v
                key = ("mdp", v or "full")
                for _ in range(2):  # both parities captured outside the timed replays
                    e._launch_multi(self._graphs, key, S, self._enqueue_multi_dp, capture_error_mode="thread_local")
                torch.cuda.synchronize(self.device)
                n = max(1, steps // S)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(n):
                    e._launch_multi(self._graphs, key, S, self._enqueue_multi_dp, capture_error_mode="thread_local")
                b.record()
                torch.cuda.synchronize(self.device)
                t[v or "full"] = a.elapsed_time(b) / (n * S)
        finally:
            self._variant = None
            torch.cuda.current_stream(self.device).wait_stream(e.sort_stream)
            e._primed = False
        ph = {"rows": t["rows"], "tail": t["compute"] - t["rows"], "merge": t["merge"] - t["compute"],
              "exchange": t["full"] - t["merge"], "step": t["full"]}
        names = list(ph)
        x = torch.tensor([ph[k] for k in names] + [-ph[k] for k in names], dtype=torch.float64,
                         device=self.device if dist.is_initialized() and dist.get_backend() == "nccl" else "cpu")
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
        n = len(names)
        out = {k: {"max": round(float(x[i]), 4), "min": round(-float(x[n + i]), 4)} for i, k in enumerate(names)}
        out["merge_mode"] = ("plan" if getattr(self, "m_plan", False) else "range" if self.range
                             else "search+dir" if (self.m_sorted and self.sdir) else "search" if self.m_sorted
                             else "maps")
        out["cap"] = int(self.cap)
        out["push"] = "fused" if self.fused_push else ("copy" if self.p2p is not None else "collective")
        return out

    def precapture(self, n: int, steps_per_graph: int = 16) -> None:
        """Capture the graphs ``train_steps(n, steps_per_graph)`` will replay (no launch)."""
        e = self.eng
        if getattr(self, "_m_dp_S", None) == steps_per_graph and e._m_primed and self.graph_collectives \
                and self.use_graph and not e._ring and steps_per_graph > 1:
            e._precapture_multi(self._graphs, ("mdp",), n, self._enqueue_multi_dp, "thread_local")

    def train_steps(self, n: int, steps_per_graph: int = 16) -> None:
        """``n`` steps from the attached pool.  With capturable collectives (RCCL) the steps are
        replayed from multi-step graphs (``steps_per_graph`` steps each, exchange included)."""
        e = self.eng
        while n > 0 and self.shadow.active:  # validated steps first (eager, collective shadow)
            self.train_step()
            n -= 1
        if n <= 0:
            return
        if self.graph_collectives and self.use_graph and not e._ring and steps_per_graph > 1:
            self._train_steps_multi(n, steps_per_graph)
            return
        for _ in range(n):
            self.train_step()

    # ---- streamed training (the Estimator's loader path at world > 1) ----------------------------
    def _stream_build(self, S: int) -> None:
        e = self.eng
        if getattr(self, "_m_dp_S", None) != S or getattr(e, "_m_pool", None) is not e.pool_ids:
            self._build_multi_dp(S)

    def _stream_run(self, n: int) -> None:
        e = self.eng
        e._launch_multi(self._graphs, ("mdp",), n, self._enqueue_multi_dp, capture_error_mode="thread_local")
        self._after_steps(e._i - n, e._i)

    def train_stream(self, batches, steps_per_graph: int = 16, after_steps=None, hold: int = 1,
                     ring_batches: int = 0) -> int:
        """Host batches (single or stacked groups) → the HBM ring → multi-step graphs with the
        exchange captured inline, like FusedDeepFM.train_stream (the single-GPU path): the per-step
        H2D synchronisation of the per-step path is gone.  The shadow-validation window (first p2p
        steps) trains per step first.  Every rank must stream the same number of batches."""
        if not (self.graph_collectives and self.use_graph):
            raise RuntimeError("train_stream needs capturable exchanges (p2p, or RCCL with graphs)")
        batches, done, pre = shadow_prefix(self, batches, after_steps, with_prefix=True)
        n = self.eng.train_stream(batches, steps_per_graph, after_steps, hold, ring_batches,
                                  build=self._stream_build, run=self._stream_run, prefix=pre)
        return done + n

    def close(self) -> None:
        """Release the captured graphs (required before destroy_process_group when they hold
        RCCL collectives)."""
        torch.cuda.synchronize(self.device)
        self._graphs = {}
        if self.p2p is not None:
            self.p2p.close()
            self.p2p = None
        if getattr(self, "_plan_ex_open", None) is not None:
            self._plan_ex_open.close()
            self._plan_ex_open = None
            self.plan_ex = None

    def check(self, replicas: bool = True) -> None:
        """Raise if a rank exported more unique rows than the exchange capacity (rows past the
        capacity would have been dropped from that step's update), if a p2p exchange wait timed
        out (a peer never arrived: its data for that step is missing), or (``replicas``; collective)
        if the replicas are no longer bit-identical across ranks."""
        self.eng.check()
        if self.p2p is not None and self.p2p.errored():
            raise RuntimeError("DP p2p exchange: a peer wait timed out (rank missing or stalled)")
        if self.mode == "dp" and int(self.overflow.item()) & 2:
            raise RuntimeError("DP plan merge: a union row id outside the table (merge_plan_apply skipped its "
                               "gradients; the plan built on the side chain is corrupt)")
        if self.overflowed():
            raise RuntimeError(f"DP exchange overflow: a rank exported more unique rows than capacity {self.cap}; "
                               "rebuild with a larger capacity (default batch_size*field_size never overflows)")
        if replicas and not self.verify_replicas():
            raise RuntimeError("DP replicas diverged: the ranks' variables / optimizer slots are not bit-identical")

    def overflowed(self) -> bool:
        """True if, in any step so far, a rank produced more unique rows than the exchange capacity
        (sticky device flag set by merge_scatter; never with the default capacity)."""
        if self.mode != "dp":
            return False
        return bool(int(self.overflow.item()) & 1)

    def load_state_dict(self, sd, strict: bool = True) -> None:
        self.eng.load_state_dict(sd, strict=strict)
        if self.mode == "dp":
            self.maps.reset()  # the hash merge tags words with the step, which just moved
        self._graphs = {}

    # ---- delegation ----------------------------------------------------------------------------
    def __getattr__(self, name):
        return getattr(self.eng, name)
