"""Row-sharded embedding tables — the reference's Parameter-Server mode on RCCL all-to-all.

The reference's PS mode (PS:461-490 cluster spec, PS:521-531 ``replica_device_setter``) keeps
``fm_w``/``fm_v`` on the parameter servers: each worker pulls the rows its batch touches and
pushes their gradients, which the servers apply asynchronously.  On one MI355X node the servers
are the GPUs themselves: id ``i`` is owned by rank ``i % W`` and stored there at local row
``i // W`` (a 1B-row table is 125M rows × (K+1) f32 + optimizer slots per GPU, well inside 288 GB
of HBM).  Every step, synchronously:

    route   sort the batch's ids owner-major; per owner the unique ids to request       (side stream)
    X1      all_to_all  requested ids                  [W, cap] int32
    serve   owners gather the requested rows from their shard
    X2      all_to_all  rows                           [W, cap, K+1] f32 → the step's "table"
    step    the fused row kernel runs unchanged, with the received rows as its table and
            each lookup's received-row index as its id; the lookup gradients are reduced per
            received row (emb_update.hip mode 1)
    X3      all_to_all  row gradients back to owners   [W, cap, K+1] f32
    update  owners sum each requested row's gradients over source ranks in rank order (merge.hip:
            up to dp.SEARCH_MAX_W ranks one launch — every request list is ascending, so each
            entry finds its row in the other lists by binary search, no maps; larger worlds
            scatter into position maps first, then apply), apply lazy L2 once
            and the row optimizer (or, ``embedding_update=exact``, the dense full-table update of
            the shard — the reference's full L2, with no dense traffic at all); the MLP optimizer
            rides as extra workgroups of the same launch
    X4      all_reduce  MLP gradients (one flat bucket), then the dense optimizer

The exchange buffers have a fixed per-owner capacity so that every collective has static shapes
(no host round trip, graph-capturable phases).  The default capacity (1.25× the even share of the
batch's lookups + 64) is exceeded only by a pathological id distribution; an owner that needs more
sets a sticky device flag that is checked every ``check_every`` steps and raises — results are
never silently truncated without an error.  ``capacity=B*F`` makes overflow impossible.

Synchronous semantics: with gradient averaging over ranks and the learning rate × W (HVD:171,
``lr_scaling``) the result equals the single-process step on the union batch (tests).

``TorchRowShard`` is the same algorithm in eager PyTorch (variable-size all-to-all), used on CPU
(gloo tests) and as the eager baseline; ``FusedRowShard`` is the HIP path (shard.hip kernels +
the fused DeepFM step).
"""
from __future__ import annotations

import dataclasses
import logging
import math
import os
from collections import OrderedDict
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..models.deepfm import TRUNC_NORMAL_STD, ModelSpec, init_params
from ..optim import OptHParams, apply_dense, apply_rows, slot_names

PAD = -1  # int32 view of 0xFFFFFFFF (request padding)
log = logging.getLogger("rocfm")


def _world_rank():
    if dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_size(V: int, W: int) -> int:
    """Rows per shard: ⌈V / W⌉ (the last ranks may hold one padding row that is never touched)."""
    return (V + W - 1) // W


def shard_rows(V: int, W: int, r: int) -> torch.Tensor:
    """Global ids owned by rank r, in local-row order."""
    return torch.arange(r, V, W, dtype=torch.int64)


def slice_rows(t: torch.Tensor, V: int, W: int, r: int) -> torch.Tensor:
    """Rows of a full table [V, ...] owned by rank r, zero-padded to shard_size(V, W) rows."""
    Vs = shard_size(V, W)
    out = torch.zeros((Vs,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    loc = t[r::W]
    out[: loc.shape[0]] = loc
    return out


def _truncated_normal_(t: torch.Tensor, std: float, gen: torch.Generator) -> torch.Tensor:
    x = torch.randn(t.shape, generator=gen, device=t.device, dtype=torch.float32)
    bad = x.abs() > 2.0
    while bool(bad.any()):
        x = torch.where(bad, torch.randn(t.shape, generator=gen, device=t.device, dtype=torch.float32), x)
        bad = x.abs() > 2.0
    return t.copy_(x * std)


def init_shard_params(spec: ModelSpec, seed: int, rank: int, world: int, device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """Initial values of rank ``rank``'s shard without materialising the full table (100M-1B rows).

    Same distributions as ``init_params`` (TF glorot_normal over the FULL table's fans, SURVEY
    App. A); the table rows are drawn on ``device`` from a per-rank stream, the dense part is
    identical on every rank.
    """
    V, K = spec.feature_size, spec.embedding_size
    Vs = shard_size(V, world)
    dense_spec = dataclasses.replace(spec, feature_size=1)
    P = init_params(dense_spec, seed)
    dev = torch.device(device)
    gen = torch.Generator(device=dev).manual_seed(seed * 1000003 + 7 * rank + 1)
    n_loc = len(range(rank, V, world))
    fm_w = torch.zeros(Vs, device=dev)
    fm_v = torch.zeros(Vs, K, device=dev)
    _truncated_normal_(fm_w[:n_loc], math.sqrt(2.0 / (V + V)) / TRUNC_NORMAL_STD, gen)
    _truncated_normal_(fm_v[:n_loc], math.sqrt(2.0 / (V + K)) / TRUNC_NORMAL_STD, gen)
    P["fm_w"], P["fm_v"] = fm_w, fm_v
    return P


def local_params(spec: ModelSpec, params: Optional[Dict[str, torch.Tensor]], seed: int, rank: int, world: int,
                 device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """This rank's parameter set: slice full tables if given, else a fresh sharded init."""
    if params is None:
        return init_shard_params(spec, seed, rank, world, device)
    V = spec.feature_size
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for k, v in params.items():
        out[k] = slice_rows(v, V, world, rank) if k in ("fm_w", "fm_v") else v.clone()
    return out


# ------------------------------------------------------------------------------------------------
# collectives (RCCL fast path; host-staged for gloo with device tensors)
# ------------------------------------------------------------------------------------------------
def all_to_all_equal(out: torch.Tensor, inp: torch.Tensor) -> None:
    """Equal-split all_to_all: inp/out [W * chunk] (first dim split evenly over ranks)."""
    if dist.get_backend() == "nccl" or inp.device.type == "cpu":
        dist.all_to_all_single(out, inp)
        return
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.detach().cpu())
    out.copy_(o)


def all_to_all_var(inp: torch.Tensor, send_counts: List[int], recv_counts: List[int]) -> torch.Tensor:
    out = torch.empty((sum(recv_counts),) + tuple(inp.shape[1:]), dtype=inp.dtype, device=inp.device)
    if dist.get_backend() == "nccl" or inp.device.type == "cpu":
        dist.all_to_all_single(out, inp.contiguous(), recv_counts, send_counts)
        return out
    o = torch.empty(out.shape, dtype=out.dtype)
    dist.all_to_all_single(o, inp.detach().cpu().contiguous(), recv_counts, send_counts)
    return o.to(inp.device)


def all_reduce_(t: torch.Tensor, op=None) -> torch.Tensor:
    op = op or dist.ReduceOp.SUM
    if dist.get_backend() == "nccl" or t.device.type == "cpu":
        dist.all_reduce(t, op=op)
        return t
    c = t.detach().cpu()
    dist.all_reduce(c, op=op)
    t.copy_(c)
    return t


def _gather_table(local: torch.Tensor, V: int, W: int) -> torch.Tensor:
    """Reassemble a full table [V, ...] from every rank's shard [Vs, ...] (all ranks get it)."""
    Vs = local.shape[0]
    dev_ok = dist.get_backend() == "nccl" or local.device.type == "cpu"
    src = local.contiguous() if dev_ok else local.detach().cpu().contiguous()
    buf = torch.empty((W * Vs,) + tuple(local.shape[1:]), dtype=local.dtype, device=src.device)
    dist.all_gather_into_tensor(buf, src) if dev_ok else dist.all_gather(list(buf.chunk(W)), src)
    # buf[r*Vs + l] holds global id l*W + r
    full = buf.view(W, Vs, *local.shape[1:]).transpose(0, 1).reshape(W * Vs, *local.shape[1:])
    return full[:V].to(local.device)


def iter_table_chunks(local: torch.Tensor, V: int, W: int, K: int, chunk_rows: Optional[int] = None):
    """Collective, every rank: ``(row0, fm_w [n], fm_v [n, K])`` CPU f32 chunks of the global
    tables in id order, from each rank's shard ``local`` [Vs, ≥K+1] (row l of rank r = id l·W + r;
    column K = fm_w).  One row range is gathered at a time (≈chunk_rows·(K+1)·4 bytes), so a
    1B-row table is exported without materialising it on any rank."""
    chunk_rows = int(chunk_rows or os.environ.get("ROCFM_EXPORT_CHUNK_ROWS", 1 << 22))
    step = max(W, chunk_rows // W * W)
    for a in range(0, V, step):
        b = min(V, a + step)
        la, lb = a // W, (b + W - 1) // W
        loc = local[la:lb, : K + 1].float().contiguous()
        if W > 1:
            dev_ok = dist.get_backend() == "nccl" or loc.device.type == "cpu"
            src = loc if dev_ok else loc.cpu()
            buf = torch.empty((W * (lb - la), K + 1), dtype=torch.float32, device=src.device)
            dist.all_gather_into_tensor(buf, src) if dev_ok else dist.all_gather(list(buf.chunk(W)), src)
            rows = buf.view(W, lb - la, K + 1).transpose(0, 1).reshape(-1, K + 1)[: b - a]
        else:
            rows = loc[: b - a]
        rows = rows.cpu()
        yield a, rows[:, K].contiguous(), rows[:, :K].contiguous()


# ================================================================================================
# eager engine
# ================================================================================================
class TorchRowShard:
    """Eager-PyTorch DeepFM with row-sharded fm_w/fm_v (one process per device)."""

    row_sharded = True
    collective_predict = True

    def __init__(self, spec: ModelSpec, hp: OptHParams, device="cpu", embedding_update: str = "sparse",
                 params: Optional[Dict[str, torch.Tensor]] = None, seed: int = 1234,
                 dropout_seed: Optional[int] = None):
        from ..models.torch_engine import TorchDeepFM

        self.W, self.rank = _world_rank()
        self.V = spec.feature_size
        self.Vs = shard_size(self.V, self.W)
        self.spec = spec
        P = local_params(spec, params, seed, self.rank, self.W, device)
        self.base = TorchDeepFM(spec, hp, device, embedding_update=embedding_update, params=P, seed=seed,
                                dropout_seed=dropout_seed if dropout_seed is not None else seed + 7919 * self.rank)
        b = self.base
        if self.W > 1:  # dense variables start identical (rank-0 broadcast, HVD:418)
            from .dist import broadcast_tensors

            broadcast_tensors([v for k, v in b.P.items() if k not in ("fm_w", "fm_v")])
        self.hp, self.device, self.embedding_update = hp, b.device, embedding_update
        self.n_loc = len(range(self.rank, self.V, self.W))

    # ---- exchange -------------------------------------------------------------------------------
    def _lookup(self, ids_flat: torch.Tensor):
        W = self.W
        uniq, inv = torch.unique(ids_flat, return_inverse=True)
        owner = uniq % W
        order = torch.argsort(owner, stable=True)
        us = uniq[order]
        sc_t = torch.bincount(owner, minlength=W)
        if W > 1:
            rc_t = torch.empty_like(sc_t)
            all_to_all_equal(rc_t, sc_t)
            sc, rc = sc_t.tolist(), rc_t.tolist()
            recv_ids = all_to_all_var(us, sc, rc)
        else:
            sc = rc = [int(len(us))]
            recv_ids = us
        lr = recv_ids // W
        P = self.base.P
        rows = torch.cat([P["fm_w"][lr].unsqueeze(1), P["fm_v"][lr]], 1)
        got = all_to_all_var(rows, rc, sc) if W > 1 else rows
        rows_u = torch.empty_like(got)
        rows_u[order] = got
        return uniq, inv, rows_u, (order, sc, rc, lr)

    def _push(self, g_u: torch.Tensor, route):
        order, sc, rc, lr = route
        gs = g_u[order]
        gr = all_to_all_var(gs, sc, rc) if self.W > 1 else gs
        lu, linv = torch.unique(lr, return_inverse=True)
        acc = torch.zeros(len(lu), g_u.shape[1], dtype=torch.float64, device=g_u.device)
        acc.index_add_(0, linv, gr.double())
        return lu, (acc / self.W).float()

    def _allreduce_dense(self, grads: Dict[str, torch.Tensor]) -> None:
        if self.W == 1:
            return
        names = sorted(grads)
        flat = torch.cat([grads[k].reshape(-1) for k in names])
        all_reduce_(flat)
        flat /= self.W
        off = 0
        for k in names:
            n = grads[k].numel()
            grads[k].copy_(flat[off:off + n].view_as(grads[k]))
            off += n

    # ---- training -------------------------------------------------------------------------------
    def set_lr_scale(self, s: float) -> None:
        self.base.set_lr_scale(s)

    def train_step(self, ids: torch.Tensor, vals: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        from ..models.deepfm import data_loss, forward

        b, spec = self.base, self.spec
        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        labels = labels.to(self.device).float()
        step = b.t + 1
        hp = b._hp()
        uniq, inv, rows_u, route = self._lookup(ids.reshape(-1))
        inv = inv.reshape(ids.shape)
        rw = rows_u[:, 0].clone().requires_grad_(True)
        rv = rows_u[:, 1:].clone().requires_grad_(True)
        dense_names = [k for k in b.trainable if k not in ("fm_w", "fm_v")]
        params = dict(b.P)
        for k in dense_names:
            params[k] = b.P[k].requires_grad_(True)
            params[k].grad = None
        y = forward(params, ids, vals, spec, train=True, gen=b.gen, rows_w=rw[inv], rows_v=rv[inv])
        loss = data_loss(y, labels, spec.loss_type)
        loss.backward()
        dgrads = {k: params[k].grad for k in dense_names}
        for k in dense_names:
            b.P[k].requires_grad_(False)
        lu, g = self._push(torch.cat([rw.grad.unsqueeze(1), rv.grad], 1), route)
        fw, fv = b.P["fm_w"], b.P["fm_v"]
        if self.embedding_update == "exact":  # full-table L2 on the owner's shard (PS:277-278)
            Gw = torch.zeros_like(fw)
            Gv = torch.zeros_like(fv)
            Gw[lu] = g[:, 0]
            Gv[lu] = g[:, 1:]
            apply_dense(hp, fw, Gw + spec.l2_reg * fw, b.slots["fm_w"], step)
            apply_dense(hp, fv, Gv + spec.l2_reg * fv, b.slots["fm_v"], step)
        else:  # lazy L2 on the rows touched by any rank, once
            gw = g[:, 0] + spec.l2_reg * fw[lu]
            gv = g[:, 1:] + spec.l2_reg * fv[lu]
            apply_rows(hp, fw, lu, gw, b.slots["fm_w"], step)
            apply_rows(hp, fv, lu, gv, b.slots["fm_v"], step)
        self._allreduce_dense(dgrads)
        for k in dense_names:
            apply_dense(hp, b.P[k], dgrads[k], b.slots[k], step)
        b.t += 1
        b._last_loss_t, b._last_has_l2 = loss.detach(), False
        return loss.detach()

    # ---- inference (collective: every rank calls it the same number of times) --------------------
    @torch.no_grad()
    def predict_batch(self, ids, vals, labels=None):
        from ..models.deepfm import forward

        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        uniq, inv, rows_u, _ = self._lookup(ids.reshape(-1))
        inv = inv.reshape(ids.shape)
        if ids.shape[0] == 0:
            z = torch.zeros(0, device=self.device)
            return z, z
        y = forward(self.base.P, ids, vals, self.spec, train=False, rows_w=rows_u[:, 0][inv],
                    rows_v=rows_u[:, 1:][inv])
        p = torch.sigmoid(y)
        if labels is None:
            return p, torch.zeros_like(p)
        labels = labels.to(self.device).float()
        if self.spec.loss_type == "log_loss":
            lr = torch.clamp(y, min=0) - y * labels + torch.log1p(torch.exp(-y.abs()))
        else:
            lr = (p - labels) ** 2
        return p, lr

    # ---- bookkeeping ----------------------------------------------------------------------------
    def l2_value(self) -> float:
        P = self.base.P
        t = torch.tensor([float((P["fm_w"].double() ** 2).sum() + (P["fm_v"].double() ** 2).sum())],
                         dtype=torch.float64, device=self.device)
        if self.W > 1:
            all_reduce_(t)
        return float(self.spec.l2_reg * 0.5 * t.item())

    def batch_loss(self, include_l2: bool = True) -> float:
        v = self.base.batch_loss(include_l2=False)
        return v + (self.l2_value() if include_l2 else 0.0)

    def global_step(self) -> int:
        return self.base.t

    def row_sets(self) -> Dict[str, torch.Tensor]:
        rows = shard_rows(self.V, self.W, self.rank)
        names = ["fm_w", "fm_v"] + [f"{t}/{s}" for t in ("fm_w", "fm_v") for s in slot_names(self.hp.name)]
        return {k: rows for k in names}

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """Local shard (row-sharded variables trimmed to this rank's real rows) + dense state."""
        sd = self.base.state_dict()
        for k in self.row_sets():
            sd[k] = sd[k][: self.n_loc].clone()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        sd = _localize(sd, self.row_sets(), self.V, self.W, self.rank, self.Vs, self.n_loc)
        self.base.load_state_dict(sd, strict=strict)

    def dense_parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        """Every variable except the row-sharded tables (no collective)."""
        out = self.base.parameters_tf()
        out.pop("fm_w")
        out.pop("fm_v")
        return out

    def iter_table_chunks(self, chunk_rows: Optional[int] = None):
        """Collective: the full tables in id order, one gathered row range at a time."""
        local = torch.cat([self.base.P["fm_v"], self.base.P["fm_w"].reshape(-1, 1)], 1)
        yield from iter_table_chunks(local, self.V, self.W, self.spec.embedding_size, chunk_rows)

    def parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        """Full variables (collective: the tables are gathered from every rank)."""
        out = self.base.parameters_tf()
        if self.W > 1:
            out["fm_w"] = _gather_table(self.base.P["fm_w"], self.V, self.W).cpu()
            out["fm_v"] = _gather_table(self.base.P["fm_v"], self.V, self.W).cpu()
        else:
            out["fm_w"], out["fm_v"] = out["fm_w"][: self.V], out["fm_v"][: self.V]
        return out


def _localize(sd, row_names, V, W, rank, Vs, n_loc):
    """Map checkpoint rows to this shard: full tables ([V,…]) are sliced, local ones ([n_loc,…])
    padded to Vs rows."""
    out = dict(sd)
    for k in row_names:
        if k not in sd:
            continue
        t = sd[k]
        if t.shape[0] == n_loc and not (t.shape[0] == V and W > 1):
            pad = torch.zeros((Vs,) + tuple(t.shape[1:]), dtype=t.dtype)
            pad[:n_loc] = t
            out[k] = pad
        elif t.shape[0] == V:
            out[k] = slice_rows(t, V, W, rank)
        else:
            raise ValueError(f"{k}: {t.shape[0]} rows is neither the full table ({V}) nor this shard ({n_loc})")
    return out


# ================================================================================================
# fused HIP engine
# ================================================================================================
class FusedRowShard:
    """Row-sharded DeepFM on the fused HIP step (one GPU per process)."""

    row_sharded = True
    collective_predict = True

    def __init__(self, spec: ModelSpec, hp: OptHParams, batch_size: int, device, params=None,
                 embedding_update: str = "sparse", seed: int = 1234, use_graph: bool = True,
                 capacity: Optional[int] = None, check_every: int = 256, compute_dtype: str = "bf16",
                 exchange: Optional[str] = None, staleness: int = 0, hot_rows: int = 0,
                 table_dtype: str = "f32", replicate_table: bool = False):
        from ..models.fused import FusedDeepFM

        # replicate_table (``parallelism=dp_owner``): owner-sharded DP.  Every rank keeps a FULL table
        # replica for its forward (no X1/X2 before the row kernel); the embedding optimizer is
        # sharded: owner o = id % W sums the row gradients sent to it (X3), applies lazy L2 + the row
        # optimizer with its 1/W share of the slots, and broadcasts the updated rows (X5) into every
        # replica.  Merge work and optimizer state per rank are 1/W of plain DP's.
        self.replicate = bool(replicate_table)
        if self.replicate and (staleness or hot_rows or embedding_update != "sparse" or table_dtype != "f32"):
            raise ValueError("owner-sharded DP (dp_owner) runs the synchronous sparse update on an f32 table "
                             "(no staleness, no hot rows)")

        if staleness not in (0, 1):
            raise ValueError(f"row-shard staleness must be 0 (synchronous) or 1, got {staleness}")
        # staleness 1 (the reference's asynchronous PS, bounded): the rows of step k+1 are served
        # in the same launch as step k's owner update, so a row updated at step k may be read
        # before, during or after its update (Hogwild-style, not bitwise reproducible — as with
        # TF's async PS); the MLP stays synchronous.  Every multi-step graph's first step is
        # served after the previous update (staleness 0 there).
        self.staleness = int(staleness)
        self._pre_served = False
        # ROCFM_P2P_MULTI=0: every p2p exchange as its own launch (A/B switch of _x3_x4 / x1_ahead)
        self.combine_handoffs = os.environ.get("ROCFM_P2P_MULTI", "1") != "0"
        # hot-row replication (SURVEY §2.6 hybrid): the hot_rows most frequent ids (chosen from rank
        # 0's first batches, or set_hot_ids) are replicated on every rank — looked up locally, never
        # routed; their per-rank gradient sums ride the X4 MLP bucket and every rank applies the
        # same (synchronous, rank-order) update to its replica.  The owners' copies are refreshed
        # from the replica whenever the table is read outside training (_flush_hot).
        self.NH = max(0, int(hot_rows))
        self.hot_ids = None  # [n_hot] ascending global ids (int32 storage of uint32), once chosen
        W, r = _world_rank()
        self.W, self.rank = W, r
        self.V = spec.feature_size
        self.Vs = Vs = shard_size(self.V, W)
        self.n_loc = len(range(r, self.V, W))
        self.spec, self.hp = spec, hp
        dev = torch.device(device)
        P = local_params(spec, params, seed, r, W, dev)
        spec_loc = dataclasses.replace(spec, feature_size=Vs)
        self.eng = e = FusedDeepFM(spec_loc, hp, batch_size, dev, embedding_update=embedding_update, seed=seed,
                                   params=P, use_graph=False, fuse_dense_opt=False,
                                   dropout_seed=seed + 7919 * r, compute_dtype=compute_dtype,
                                   table_dtype=table_dtype, dedup=False)  # (rows are routed per owner)
        del P
        e.id_limit = self.V  # the id guard (ROCFM_CHECK_IDS) checks global ids, not local rows
        e._build_fetch()
        if e._hazard is not None:  # ROCFM_HAZARD=1: this driver's buffers join the checked set
            e._hazard.attach("rs", self)
        self.H, self.device, self.embedding_update = e.H, e.device, embedding_update
        self.use_graph, self.check_every = use_graph, int(check_every)
        from .dp import collectives_capturable

        self.graph_collectives = use_graph and collectives_capturable()
        from .dp import force_collectives

        self.force = force_collectives()
        if W > 1:
            from .dist import broadcast_tensors

            broadcast_tensors([e.dense] + list(e.dense_slots))
            e.refresh_bf16()
        H, B, F, Kp = e.H, e.B, e.F, e.Kp
        n = e.n_lookup
        self.n = n
        cap = int(capacity) if capacity else min(n, int(math.ceil(1.25 * n / W)) + 64)
        cap = max(1, min(cap, n))
        self.cap = cap = (cap + 3) // 4 * 4  # whole float4 runs per owner segment (p2p push)
        M = W * cap
        self.M = M
        i32 = dict(dtype=torch.int32, device=dev)
        # ---- routing buffers (parity q = the step that will consume them) ----
        self.route_bits = max(1, math.ceil(math.log2(max((W + (self.NH > 0)) * Vs, 2))))
        self.rkeys = torch.zeros(n, **i32)
        self.rsk = torch.zeros(n, **i32)
        self.rsv = [torch.zeros(n, **i32) for _ in range(2)]
        self.send_ids = [torch.full((M,), PAD, **i32) for _ in range(2)]
        self.local_idx = [torch.zeros(e.Bp, F, **i32) for _ in range(2)]
        self.skl = [torch.zeros(n, **i32) for _ in range(2)]
        self.counts = [torch.zeros(W, **i32) for _ in range(2)]
        self.overflow = torch.zeros(1, **i32)
        self.bad = torch.zeros(1, **i32)
        self.route_scratch = torch.zeros(H.route_scratch_ints(n), **i32)
        from ..models.fused import iota_sort_temp_bytes

        self.route_temp = torch.zeros(max(iota_sort_temp_bytes(H, n, self.route_bits), 16), dtype=torch.uint8,
                                      device=dev)
        # ---- exchange buffers ----
        f32 = dict(dtype=torch.float32, device=dev)
        NH = self.NH
        # rows_in = [W·cap received rows | NH replicated rows] (the row kernel's table)
        self.rows_out = torch.zeros(M + (NH if W == 1 and not self.force else 0), Kp, **f32)
        self.grad_stage = torch.zeros(M, Kp, **f32)
        # X1-X3 all-to-all and X4 MLP all-reduce: one-shot push over IPC-mapped peer buffers on one
        # node (rocfm.parallel.p2p; the receive buffers ARE the peer-mapped slots), else RCCL
        from .p2p import open_exchanges

        self.P = e.layout.total
        # X4 bucket: [MLP grads P | NH·Kp replicated-row gradient sums | NH touched flags]
        self.PX = (self.P + NH * (Kp + 1) + 3) // 4 * 4
        self.mlp_bucket = torch.zeros(self.PX, **f32)
        e.dense_grads_flat = self.mlp_bucket[:self.P]
        # (5th: the request lists of odd steps — staleness 1, or the synchronous p2p path, whose X1 of
        # step k+1 rides step k's X3/X4 hand-off launch)
        slots = [cap, cap * Kp, cap * Kp, self.PX, cap]
        # X5 (dp_owner): each owner's updated rows, [count | pad 3 | keys W·cap | rows W·cap·Kp]
        self.capB = W * cap
        self.S5 = 4 + self.capB * (1 + Kp)
        self.emb_full = self.x5_send = None
        if self.replicate:
            slots.append(self.S5)
            self.x5_send = torch.zeros(self.S5, **f32)
            self.emb_full = (_gather_table(e.emb.float().contiguous(), self.V, W) if W > 1
                             else e.emb[:self.V].float()).contiguous().clone()
        exs = open_exchanges(slots, dev, exchange, extra_floats=[0, NH * Kp] + [0] * (len(slots) - 2))
        self._bind_exchange(exs)
        self._p2p_params = {}
        # owner merge: binary search in the sorted request lists (small worlds), or position maps
        # filled by a scatter launch (direct addressing over the local rows, or a W·cap hash table
        # for very large shards) — see dp.SEARCH_MAX_W
        from .dp import SEARCH_MAX_W, MergeMaps

        self.maps = MergeMaps(W, cap, Vs, dev) if W > SEARCH_MAX_W else None
        self.hot_slots = [torch.zeros(NH, Kp, **f32) for _ in e.emb_slots] if NH else []
        self.hot_ids_dev = torch.full((max(NH, 1),), PAD, **i32)
        self.n_hot = 0
        # prediction routing (own buffers: never races the pipelined training route)
        self.pred_rsv = torch.zeros(n, **i32)
        self.pred_send = torch.full((M,), PAD, **i32)
        self.pred_local = torch.zeros(e.Bp, F, **i32)
        self.pred_skl = torch.zeros(n, **i32)
        self.pred_counts = torch.zeros(W, **i32)
        self._graphs: Dict = {}
        self._warm = 0
        self._build()
        if self.maps is not None:
            H.merge_init(self.owner_params[0], e.stream_ptr)
        # self-validation (rocfm.parallel.validate): the first steps of a p2p run shadow every
        # exchange through the collective; replica digests (MLP + replicated rows) in check()
        from .validate import Shadow, fault_rank

        self.shadow = Shadow(dev, steps=None if (self.exchange == "p2p" and W > 1) else 0)
        self.shadow.corrupt = fault_rank("corrupt_push", r)
        self._corrupt_replica = fault_rank("corrupt_replica", r)
        self._set_mirror(self.shadow.active)

    def _set_mirror(self, on: bool) -> None:
        """Producer pushes: also keep each result locally while the shadow window is open — X3 row
        gradients in grad_stage, X4 MLP gradients in the MLP bucket (the shadow's local copies)."""
        for p in range(2):
            self.eng.emb_params[p].push_mirror = 1 if (on and self.grad_push is not None) else 0
            self.eng.wgrad_params[p].push_mirror = 1 if (on and self.mlp_push is not None) else 0

    def _bind_exchange(self, exs) -> None:
        """Receive-side buffers of the X1-X4 exchanges: the peer-mapped p2p slots (``exs``), the
        send buffers themselves (one rank), or plain tensors for the collectives."""
        from .p2p import producer_push_enabled

        W, M, NH, Kp, dev = self.W, self.M, self.NH, self.eng.Kp, self.device
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.exchange = "p2p" if exs else "rccl"
        self.mlp_push = self.grad_push = None  # X4 / X3 producer-side push targets (below)
        self.p2p_x = {}
        self.recv_pair = None  # staleness 1: request lists of consecutive steps (parity)
        self._p2p_params = {}
        if exs:
            self.x_ids, self.x_rows, self.x_grad, self.x_mlp = exs[:4]
            self.x_all = list(exs)
            self.recv_ids = self.x_ids.recv_tensor(torch.int32, (M,))
            self.recv_ids.fill_(PAD)
            self.rows_in = self.x_rows.recv_tensor(torch.float32, (M + NH, Kp))
            self.grad_back = self.x_grad.recv_tensor(torch.float32, (M, Kp))
            for t, ex in ((self.recv_ids, self.x_ids), (self.rows_in, self.x_rows), (self.grad_back, self.x_grad)):
                self.p2p_x[t.data_ptr()] = ex
            r2 = exs[4].recv_tensor(torch.int32, (M,))
            r2.fill_(PAD)
            self.p2p_x[r2.data_ptr()] = exs[4]
            self.recv_pair = [self.recv_ids, r2]
            self.graph_collectives = self.use_graph  # push kernels are capturable whatever the backend
            # X4 pushed by its producer (csrc/kernels/push.h): the wgrad workgroups store the MLP
            # gradients straight into every rank's X4 slot from inside the step tail, and the X4
            # launch only hands the data off.  Same switch as the DP push
            # (p2p.producer_push_enabled); replicated hot rows keep the copy (their sums ride the
            # same bucket from the embedding role).
            if NH == 0 and producer_push_enabled(self.x_mlp):
                self.mlp_push = self.x_mlp.push_target()
                # X3 likewise: the embedding role stores each requested row's gradient sum straight
                # into its owner's slot (row o·cap + j → owner o, row j)
                self.grad_push = self.x_grad.push_target()
        elif W == 1 and not self.force:
            # one rank: every exchange is the identity, so the receive side IS the send side (rows
            # and row gradients share one buffer each; the request list each step reads is that
            # step's own send list, bound per step below) — no copies in the step
            self.x_all = []
            self.recv_ids = None
            self.rows_in = self.rows_out
            self.grad_back = self.grad_stage
        else:
            self.x_all = []
            self.recv_ids = torch.full((M,), PAD, **i32)
            self.rows_in = torch.zeros(M + NH, Kp, **f32)
            self.grad_back = torch.zeros(M, Kp, **f32)
            if self.staleness:
                self.recv_pair = [self.recv_ids, torch.full((M,), PAD, **i32)]
            from .dp import collectives_capturable

            self.graph_collectives = self.use_graph and collectives_capturable()
        self.rows_x = self.rows_in[:M]  # the X2 all-to-all part of rows_in
        self.hot_rep = self.rows_in[M:]  # the replica
        # X5 (dp_owner): the owners' updated-row lists — peer-mapped slots (the owner merge pushes
        # keys + rows itself; the X5 launch carries the counts), the send buffer itself (one rank),
        # or a gathered tensor for the collective
        self.x_bc = self.bc_push = self.bc_recv = None
        if self.replicate:
            if exs:
                self.x_bc = exs[5]
                self.x_all = list(exs)
                self.bc_recv_ptr, self.bc_slot = self.x_bc.recv_ptr, self.x_bc.slot
                self.bc_push = self.x_bc.push_target()
            elif W == 1 and not self.force:
                self.bc_recv, self.bc_slot = self.x5_send, self.S5
                self.bc_recv_ptr = self.x5_send.data_ptr()
            else:
                self.bc_recv, self.bc_slot = torch.zeros(W * self.S5, **f32), self.S5
                self.bc_recv_ptr = self.bc_recv.data_ptr()

    # ---- kernel parameter blocks ------------------------------------------------------------------
    def _route_params(self, ids, rsv, send, local, skl, counts, n):
        H = self.H
        kp = H.ShardKeysParams()
        kp.ids, kp.n, kp.W, kp.Vs, kp.keys = ids.data_ptr(), n, self.W, self.Vs, self.rkeys.data_ptr()
        kp.hot_ids, kp.n_hot = self.hot_ids_dev.data_ptr(), self.n_hot
        rp = H.ShardRouteParams()
        rp.skeys, rp.svals, rp.n = self.rsk.data_ptr(), rsv.data_ptr(), n
        rp.W, rp.Vs, rp.cap = self.W, self.Vs, self.cap
        rp.send_ids, rp.local_idx, rp.skeys_local = send.data_ptr(), local.data_ptr(), skl.data_ptr()
        rp.counts, rp.overflow = counts.data_ptr(), self.overflow.data_ptr()
        rp.scratch = self.route_scratch.data_ptr()
        return kp, rp

    def _build(self):
        e, H = self.eng, self.H
        self.route = [self._route_params(e.slot_ids[q], self.rsv[q], self.send_ids[q], self.local_idx[q], self.skl[q],
                                         self.counts[q], self.n) for q in range(2)]
        self.serve = [self._serve_params(self._recv_ids_for(self.send_ids[p], p)) for p in range(2)]
        self.pred_serve = self._serve_params(self._recv_ids_for(self.pred_send))
        self.owner_params = []
        for p in range(2):
            rp = e.rows_params[p]
            rp.ids, rp.emb = self.local_idx[p].data_ptr(), self.rows_in.data_ptr()
            rp.tbl_bf16 = 0  # the row kernel's table is the f32 received-rows buffer
            self._bind_replica(rp, e.slot_ids[p])
            lp = e.emb_params[p]  # local: Σ lookup grads per received row → grad_stage
            lp.skeys, lp.svals, lp.n = self.skl[p].data_ptr(), self.rsv[p].data_ptr(), self.n
            lp.mode, lp.dense_grad, lp.max_key, lp.grad_scale = 1, self.grad_stage.data_ptr(), 0, 1.0
            lp.touched = 0  # writes the exchange stage, not the table's gradient rows
            self._bind_hot_out(lp)
            op = H.MergeParams()  # owner: Σ over source ranks per local row → optimizer
            op.keys, op.key_stride = self._recv_ids_for(self.send_ids[p], p).data_ptr(), self.cap
            op.rows, op.row_stride = self.grad_back.data_ptr(), self.cap * e.Kp
            op.counts = 0
            op.W, op.cap, op.Kp, op.K1 = self.W, self.cap, e.Kp, e.K1
            op.key_div, op.Vmap = self.W, self.Vs
            if self.maps is not None:
                self.maps.bind(op)
                op.use_maps = 1
            op.emb, op.tbl_bf16 = e.emb.data_ptr(), e.tbl_bf16
            op.s0, op.s1 = e._slot_ptrs(e.emb_slots)
            op.l2, op.grad_scale = float(self.spec.l2_reg), 1.0 / self.W
            op.opt, op.step = e._opt(p), e.steps[p:].data_ptr()
            self._bind_bcast(op)
            if self.embedding_update == "exact":
                op.mode, op.dense_grad = 1, e.dense_grad.data_ptr()
                op.touched = e.touched.data_ptr()  # the owner's dense update reads these rows
                e.emb_dense_params[p].grad_scale = 1.0
            else:
                op.mode = 0
            self.owner_params.append(op)
            da = e.dense_apply_params[p]
            da.apply, da.grad_scale = 1, 1.0 / self.W
            self._set_mlp_grads(da)
            e.wgrad_params[p].grads = e.dense_grads_flat.data_ptr()
            self._set_push(rp, e.wgrad_params[p], lp)
        pp = e.pred_params
        pp.ids, pp.emb = self.pred_local.data_ptr(), self.rows_in.data_ptr()
        pp.tbl_bf16 = 0
        self.pred_route = self._route_params(e.pred_ids, self.pred_rsv, self.pred_send, self.pred_local,
                                             self.pred_skl, self.pred_counts, self.n)
        self.pred_route[0].n_hot = 0  # predictions read the owners' (flushed) rows
        self.hot_params = [self._hot_params(lp_, self.owner_params[p].opt, self.owner_params[p].step)
                           for p, lp_ in enumerate(e.emb_params[:2])]

    # ---- owner-sharded DP (replicate_table) --------------------------------------------------------
    def _bind_replica(self, rp, ids) -> None:
        """dp_owner: the row kernel gathers the batch's global ids from the full replica, and its
        workgroup 0 also raises "entered" for X5 (the previous step's row_scatter, the last reader
        of this rank's X5 slots, is done); it zeroes this step's X5 row counter."""
        if not self.replicate:
            return
        rp.ids, rp.emb, rp.tbl_bf16 = ids.data_ptr(), self.emb_full.data_ptr(), 0
        rp.push3 = self.bc_push if self.bc_push is not None else self.H.PushTarget()
        rp.zero_word = self.x5_send.data_ptr()

    def _bind_bcast(self, op) -> None:
        """dp_owner: the owner merge appends every updated row (global id, f32 row) to X5."""
        if not self.replicate:
            return
        op.bc_count = self.x5_send.data_ptr()
        op.bc_keys = self.x5_send[4:].data_ptr()
        op.bc_rows = self.x5_send[4 + self.capB:].data_ptr()
        op.bc_cap, op.bc_mul, op.bc_add = self.capB, self.W, self.rank
        op.bc_push = self.bc_push if self.bc_push is not None else self.H.PushTarget()

    def _x5(self) -> None:
        """X5 all-gather of the owners' updated rows, then every replica takes them (row_scatter)."""
        if self.x_bc is not None:  # p2p: keys + rows already pushed by the merge; counts + hand-off here
            prm = self._p2p_params.get("x5")
            if prm is None:
                prm = self._p2p_params["x5"] = self.x_bc.params(self.x5_send.data_ptr(), 4)
            self.x_bc.push(prm)
            if self.shadow.active:  # an all-gather: this rank's own slot holds its list (the merge
                # pushes the rows straight into the slots and keeps no local copy, so this check
                # covers the transfer and the receivers' agreement, not the owner's row values)
                from .dp import _all_gather_flat

                sl = self.bc_slot
                got = self.x_bc.recv_tensor(torch.float32, (self.W * sl,))
                own = got[self.rank * sl:(self.rank + 1) * sl].clone()  # (before a fault hits the copy)
                self.shadow.corrupt_(got)
                want = torch.empty_like(got)
                _all_gather_flat(want, own)
                self.shadow.compare(got, want)
        elif self.W > 1 or self.force:
            from .dp import _all_gather_flat

            _all_gather_flat(self.bc_recv, self.x5_send)
        sp = self.H.RowScatterParams()
        sp.recv, sp.slot_stride, sp.W, sp.cap, sp.Kp = self.bc_recv_ptr, self.bc_slot, self.W, self.capB, self.eng.Kp
        sp.table, sp.rows = self.emb_full.data_ptr(), self.V
        self.H.row_scatter(sp, self.eng.stream_ptr)

    def _sync_full(self) -> None:
        """Rebuild the full replica from the owners' shards (after a checkpoint restore)."""
        e = self.eng
        full = _gather_table(e.emb.float().contiguous(), self.V, self.W) if self.W > 1 else e.emb[:self.V].float()
        self.emb_full.copy_(full)

    # ---- hot-row replication ----------------------------------------------------------------------
    def _bind_hot_out(self, ep) -> None:
        """The local reduction sends replicated rows' sums to the X4 bucket instead of grad_stage."""
        if self.n_hot:
            ep.hot_out, ep.hot_base, ep.n_hot = self.mlp_bucket[self.P:].data_ptr(), self.M, self.n_hot
        else:
            ep.hot_out, ep.n_hot = 0, 0

    def _hot_params(self, ep, opt, step_ptr):
        """Replica update block (merge_search_apply role) or None without replicated rows."""
        if not self.n_hot:
            return None
        e, H = self.eng, self.H
        h = H.HotApplyParams()
        h.rows = self.hot_rep.data_ptr()
        sl = self.hot_slots
        h.s0 = sl[0].data_ptr() if len(sl) > 0 else 0
        h.s1 = sl[1].data_ptr() if len(sl) > 1 else 0
        hot_part = self.mlp_bucket[self.P:]
        if self.exchange == "p2p":  # W rank segments, summed in rank order by the kernel
            h.grads, h.nseg, h.seg_stride = self.x_mlp.recv_ptr + 4 * self.P, self.W, self.x_mlp.slot
        else:  # all-reduced in place (or one rank)
            h.grads, h.nseg, h.seg_stride = hot_part.data_ptr(), 1, 0
        h.zero = hot_part.data_ptr()
        h.H, h.Kp, h.K1 = self.n_hot, e.Kp, e.K1
        h.l2, h.grad_scale = float(self.spec.l2_reg), 1.0 / self.W
        h.opt, h.step = opt, step_ptr
        h.dense = 1 if self.embedding_update == "exact" else 0
        return h

    def set_hot_ids(self, ids) -> None:
        """Replicate these global ids (≤ hot_rows; rank 0's list is used on every rank).  Collective.
        The replica (and its optimizer slots) is loaded from the owners."""
        if not self.NH:
            raise ValueError("set_hot_ids needs hot_rows > 0 at construction")
        self._flush_hot()
        t = torch.full((self.NH + 1,), -1, dtype=torch.int64)
        u = torch.unique(torch.as_tensor(ids, dtype=torch.int64).flatten().cpu())
        u = u[(u >= 0) & (u < self.V)][: self.NH]
        t[0] = len(u)
        t[1:1 + len(u)] = u
        if self.W > 1:
            from .dist import broadcast_tensors

            tt = t.to(self.device) if dist.get_backend() == "nccl" else t
            broadcast_tensors([tt])
            t = tt.cpu()
        k = int(t[0])
        self.hot_ids = t[1:1 + k].clone()
        self.n_hot = k
        self.hot_ids_dev.fill_(PAD)
        self.hot_ids_dev[:k].copy_(self.hot_ids.to(torch.int32))
        self._load_hot()
        self._build()  # parameter blocks carry n_hot
        self._graphs = {}
        self._ms_S = None  # multi-step blocks are rebuilt with the hot ids
        self._pre_served = False

    def _choose_hot(self, ids: torch.Tensor) -> None:
        """Pick the hot_rows most frequent ids of these batches (rank 0's choice wins)."""
        u, c = torch.unique(ids.flatten().to(torch.int64), return_counts=True)
        # count descending, ties to the lower id (stable sort over the ascending unique ids):
        # the same hot set on every run
        order = torch.argsort(c.cpu(), descending=True, stable=True)[: self.NH]
        self.set_hot_ids(u.cpu()[order])

    def _owned_hot(self):
        """(replica slots, local rows) of the replicated ids this rank owns."""
        hid = self.hot_ids
        mine = (hid % self.W) == self.rank
        slot = torch.nonzero(mine).flatten()
        return slot.to(self.device), (hid[mine] // self.W).to(self.device)

    @torch.no_grad()
    def _load_hot(self) -> None:
        """Replica ← owners' rows (and slots): every rank adds the rows it owns, all-reduced."""
        if not self.n_hot:
            return
        e = self.eng
        slot, rows = self._owned_hot()
        bufs = [self.hot_rep] + self.hot_slots
        srcs = [e.emb] + list(e.emb_slots)
        flat = torch.zeros(len(bufs), self.n_hot, e.Kp, dtype=torch.float32, device=self.device)
        for i, src in enumerate(srcs):
            flat[i].index_copy_(0, slot, src.index_select(0, rows).float())
        if self.W > 1:
            if dist.get_backend() == "nccl":
                all_reduce_(flat)
            else:
                c = flat.cpu()
                all_reduce_(c)
                flat.copy_(c)
        for i, b in enumerate(bufs):
            b[: self.n_hot].copy_(flat[i])

    @torch.no_grad()
    def _flush_hot(self) -> None:
        """Owners' rows (and slots) ← the replica, for the replicated ids this rank owns."""
        if not self.n_hot:
            return
        e = self.eng
        torch.cuda.current_stream(self.device).wait_stream(e.sort_stream)
        slot, rows = self._owned_hot()
        for dst, src in zip([e.emb] + list(e.emb_slots), [self.hot_rep] + self.hot_slots):
            dst.index_copy_(0, rows, src.index_select(0, slot).to(dst.dtype))

    def _recv(self, parity: int = 0) -> Optional[torch.Tensor]:
        """X1 receive buffer of a step of this parity (None: world 1, the send list is read)."""
        if self.recv_ids is None:
            return None
        return self.recv_pair[parity] if self.recv_pair is not None else self.recv_ids

    def _recv_ids_for(self, send: torch.Tensor, parity: int = 0) -> torch.Tensor:
        """The request list an owner reads after exchanging ``send`` (world 1: ``send`` itself)."""
        r = self._recv(parity)
        return send if r is None else r

    def _serve_params(self, ids: torch.Tensor):
        e = self.eng
        sv = self.H.ShardServeParams()
        sv.ids, sv.m, sv.W, sv.rank, sv.Vs = ids.data_ptr(), self.M, self.W, self.rank, self.Vs
        sv.table, sv.Kp, sv.rows_out, sv.lkeys = e.emb.data_ptr(), e.Kp, self.rows_out.data_ptr(), 0
        sv.bad = self.bad.data_ptr()
        sv.tbl_bf16 = e.tbl_bf16
        return sv

    # ---- batch feeding (delegated) ------------------------------------------------------------
    def attach_pool(self, ids, vals, labels, start: int = 0):
        if self.NH and self.hot_ids is None:
            self._choose_hot(ids[: min(len(ids), 8)])
        self.eng.attach_pool(ids, vals, labels, start)
        self._graphs = {}
        self._pre_served = False

    def push_batch(self, ids, vals, labels):
        self.eng.push_batch(ids, vals, labels)

    def load_batch(self, ids, vals, labels=None):
        if self.NH and self.hot_ids is None:
            self._choose_hot(ids)
        self.eng.load_batch(ids, vals, labels)
        self._pre_served = False

    def set_lr_scale(self, s: float) -> None:
        e = self.eng
        e.set_lr_scale(s)
        for p in range(2):
            self.owner_params[p].opt = e._opt(p)
        self._graphs = {}

    # ---- step pieces ---------------------------------------------------------------------------
    def _route_launch(self, rt, n, stream) -> None:
        kp, rp = rt
        H, s = self.H, stream.cuda_stream
        if n > 0:
            H.shard_keys(kp, s)
            from ..models.fused import iota_sort

            iota_sort(H, self.route_temp, self.rkeys.data_ptr(), self.rsk.data_ptr(), rp.svals, n, self.route_bits, s)
        H.shard_route(rp, s)

    def prime(self) -> None:
        e = self.eng
        e.prime()  # fetch the current batch into its slot
        self._route_launch(self.route[e._i % 2], self.n, torch.cuda.current_stream(self.device))
        e._primed = True

    def _fork_next(self, p: int, fork=None):
        e = self.eng
        main = torch.cuda.current_stream(self.device)
        side = e.sort_stream
        if fork is None:
            side.wait_stream(main)
        else:
            side.wait_event(fork)
        with torch.cuda.stream(side):
            e.H.fetch_batch(e.fetch_params[p], side.cuda_stream)
            self._route_launch(self.route[1 - p], self.n, side)
        return side

    def _phase_serve(self, p: int) -> None:
        self.H.shard_serve(self.serve[p], self.eng.stream_ptr)

    def _phase_compute(self, p: int, with_side: bool = True) -> None:
        e, H = self.eng, self.H
        main = torch.cuda.current_stream(self.device)
        side = self._fork_next(p) if with_side else None  # forked first: own hardware queue in the graph
        aux = e._enqueue_rows_then_fork_wgrad(p)
        H.emb_rows_update(e.emb_params[p], main.cuda_stream)
        e._join(aux)
        if side is not None:
            e._join(side)

    def _phase_update(self, p: int) -> None:
        e, H = self.eng, self.H
        s = e.stream_ptr
        if self.maps is not None:
            H.merge_scatter(self.owner_params[p], s)
        H.merge_search_apply(self.owner_params[p], e.dense_apply_params[p], s, None,
                             self.hot_params[p])  # owner merge ‖ MLP opt ‖ replicated rows
        if self.embedding_update == "exact":
            H.emb_dense_update(e.emb_dense_params[p], s)

    def _run(self, key, fn, collectives: bool = False):
        if not self.use_graph or self._warm < 4 or self.shadow.active:
            fn()
            return
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.device)
            with torch.cuda.graph(g, capture_error_mode="thread_local" if collectives else "global"):
                fn()
            self._graphs[key] = g
        g.replay()

    def _p2p_prm(self, out, inp):
        """(exchange, push parameters) of the p2p all-to-all of ``inp`` into ``out``."""
        ex = self.p2p_x[out.data_ptr()]
        key = (out.data_ptr(), inp.data_ptr())
        prm = self._p2p_params.get(key)
        if prm is None:
            chunk = out.numel() // self.W
            if self.grad_push is not None and ex is self.x_grad:  # X3 already in the slots
                prm = self._p2p_params[key] = ex.params(inp.data_ptr(), 0)
            else:
                prm = self._p2p_params[key] = ex.params(inp.data_ptr(), chunk, src_stride_floats=chunk)
        return ex, prm

    def _mlp_prm(self):
        prm = self._p2p_params.get("mlp")
        if prm is None:  # fused push: the payload is already in the slots, only the hand-off
            n = 0 if self.mlp_push is not None else self.PX
            prm = self._p2p_params["mlp"] = self.x_mlp.params(self.mlp_bucket.data_ptr(), n)
        return self.x_mlp, prm

    def _x3_x4(self, x1_next=None, x1_now=None) -> None:
        """X3 row gradients + X4 MLP gradients (+ ``x1_next`` = (out, inp): the next step's X1
        requests).  On the p2p path ONE hand-off launch carries all of them (p2p_push_multi: the
        exchanges' peer waits overlap instead of running as consecutive launches); the shadow
        window and the collectives run them one by one."""
        if self.exchange == "p2p" and not self.shadow.active and self.combine_handoffs:
            from .p2p import P2PExchange

            pairs = [self._p2p_prm(self.grad_back, self.grad_stage), self._mlp_prm()]
            for x1 in (x1_now, x1_next):
                if x1 is not None:
                    pairs.append(self._p2p_prm(*x1))
            P2PExchange.push_multi([a for a, _ in pairs], [b for _, b in pairs])
            return
        if x1_now is not None:
            self._exchange(*x1_now)                                             # X1 of this step (dp_owner)
        self._exchange(self.grad_back, self.grad_stage)                         # X3 row grads
        self._allreduce_mlp()                                                   # X4 MLP grads
        if x1_next is not None:
            self._exchange(*x1_next)                                            # X1 of the next step

    @property
    def x1_ahead(self) -> bool:
        """Synchronous p2p multi-step graphs: the X1 requests of step k+1 are handed off with
        step k's X3/X4 (their routing is done by the side chain before the graph starts)."""
        return not self.staleness and not self.replicate and self.exchange == "p2p" and self.combine_handoffs

    def _exchange(self, out, inp):
        """Equal-split all-to-all of ``inp`` into ``out`` (X1-X3).  World 1 (no forced collectives):
        the receive side aliases the send side, nothing to move."""
        if out is None or out is inp or out.data_ptr() == inp.data_ptr():
            return
        ex = self.p2p_x.get(out.data_ptr())
        if ex is not None:
            ex, prm = self._p2p_prm(out, inp)
            ex.push(prm)
            if self.shadow.active:  # the same all-to-all through the collective, compared bitwise
                self.shadow.corrupt_(out)
                want = torch.empty_like(out)
                all_to_all_equal(want, inp)
                self.shadow.compare(out, want)
        elif self.W > 1 or self.force:
            all_to_all_equal(out, inp)
        else:
            out.copy_(inp)

    def _set_mlp_grads(self, da) -> None:
        """Point a dense-apply block at the X4 result: the W gathered rank segments (p2p, summed in
        rank order by the kernel) or the RCCL all-reduced flat gradient."""
        e = self.eng
        if self.exchange == "p2p":
            da.grads, da.nseg, da.seg_stride = self.x_mlp.recv_ptr, self.W, self.x_mlp.slot
        else:
            da.grads, da.nseg = e.dense_grads_flat.data_ptr(), 1

    @property
    def fused_push(self) -> bool:
        """True when the step tail's wgrad workgroups push X4 into the peers' slots themselves."""
        return self.mlp_push is not None

    def _set_push(self, rows, wp, ep) -> None:
        """X4 / X3 producer push: the row kernel raises "entered" for both (their consumer, the
        previous update launch, is done), the wgrad role stores X4 and the embedding role X3."""
        none = self.H.PushTarget()  # W = 0: no push (also clears targets after a fallback)
        mlp = self.mlp_push if self.mlp_push is not None else none
        rows.push, wp.push = mlp, mlp
        if self.grad_push is not None:
            rows.push2 = self.grad_push
            ep.push, ep.push_seg = self.grad_push, self.cap
        else:
            rows.push2, ep.push, ep.push_seg = none, none, 0

    def _allreduce_mlp(self) -> None:
        """X4: the MLP gradients of every rank (p2p all-gather; the sum happens in dense_apply)."""
        e = self.eng
        if self.exchange == "p2p":
            _, prm = self._mlp_prm()
            self.x_mlp.push(prm)
            if self.shadow.active:  # X4 is an all-gather of every rank's local MLP bucket (the copy
                from .dp import _all_gather_flat  # push's source, or the fused push's mirror)

                got = self.x_mlp.recv_tensor(torch.float32, (self.W * self.x_mlp.slot,))
                sl = self.x_mlp.slot
                loc = torch.zeros(sl, dtype=torch.float32, device=self.device)
                loc[:self.PX].copy_(self.mlp_bucket)
                self.shadow.corrupt_(got)
                want = torch.empty_like(got)
                _all_gather_flat(want, loc)
                self.shadow.compare(got, want)
        elif self.W > 1 or self.force:
            all_reduce_(self.mlp_bucket)  # MLP grads + replicated-row sums, one collective

    def _step_body(self, p: int) -> None:
        e = self.eng
        if self.staleness:
            self._step_body_stale(p, serve_first=not self._pre_served)
            return
        side = self._fork_next(p)  # next batch's fetch + route overlaps the whole step
        if self.replicate:  # dp_owner: the forward reads the full replica; X1 only keys the merge
            self._phase_compute(p, with_side=False)
            self._x3_x4(None, (self._recv(p), self.send_ids[p]))                # X1 + X3 + X4
            self._phase_update(p)
            self._x5()                                                          # X5 updated rows
            e._join(side)
            return
        self._exchange(self._recv(p), self.send_ids[p])                         # X1 requests
        self._phase_serve(p)
        self._exchange(self.rows_x, self.rows_out[:self.M])                             # X2 rows
        self._phase_compute(p, with_side=False)
        self._x3_x4()                                                           # X3 + X4
        self._phase_update(p)
        e._join(side)

    def _step_body_stale(self, p: int, serve_first: bool) -> None:
        """Staleness 1: this step's rows were served by the previous step's update launch (unless
        ``serve_first``); the next batch is routed on the side chain during the compute and its
        rows are served by this step's update launch."""
        e, H = self.eng, self.H
        if serve_first:
            self._exchange(self._recv(p), self.send_ids[p])                     # X1 requests
            self._phase_serve(p)
            self._exchange(self.rows_x, self.rows_out[:self.M])                         # X2 rows
        self._phase_compute(p, with_side=True)  # joins the side chain: batch 1-p is routed
        self._x3_x4((self._recv(1 - p), self.send_ids[1 - p]))                  # X3 + X4 + X1 of the next step
        if self.maps is not None:
            H.merge_scatter(self.owner_params[p], e.stream_ptr)
        H.merge_search_apply(self.owner_params[p], e.dense_apply_params[p], e.stream_ptr, self.serve[1 - p],
                             self.hot_params[p])
        if self.embedding_update == "exact":
            H.emb_dense_update(e.emb_dense_params[p], e.stream_ptr)
        self._exchange(self.rows_x, self.rows_out[:self.M])                             # X2 of the next step

    def train_step(self) -> None:
        e = self.eng
        e._m_primed = False
        if not e._primed:
            self.prime()
        p = e._i % 2
        if self.staleness:
            first = not self._pre_served
            if self.graph_collectives:
                self._run(("stale", p, first), lambda: self._step_body_stale(p, first), collectives=True)
            else:
                self._step_body_stale(p, first)
            self._pre_served = True
        elif self.graph_collectives:  # one graph per step, collectives included
            self._run(("step", p), lambda: self._step_body(p), collectives=True)
        elif self.replicate:
            self._run(("compute", p), lambda: self._phase_compute(p))
            self._x3_x4(None, (self._recv(p), self.send_ids[p]))
            self._run(("update", p), lambda: self._phase_update(p))
            self._x5()
        else:
            self._exchange(self._recv(p), self.send_ids[p])
            self._run(("serve", p), lambda: self._phase_serve(p))
            self._exchange(self.rows_x, self.rows_out[:self.M])
            self._run(("compute", p), lambda: self._phase_compute(p))
            self._exchange(self.grad_back, self.grad_stage)
            self._allreduce_mlp()
            self._run(("update", p), lambda: self._phase_update(p))
        self._warm += 1
        e._i += 1
        if self.shadow.step_done():
            self._shadow_finish()
        self._after_steps(e._i - 1, e._i)

    # ---- self-validation (rocfm.parallel.validate) ----------------------------------------------
    def _shadow_finish(self) -> None:
        self._set_mirror(False)
        if self.shadow.finish():
            msg = (f"row-shard exchange: p2p results differed from the collective in the first "
                   f"{self.shadow.compared} validated exchanges on some rank; falling back to RCCL")
            if self.replicate:  # the collective X5 gathers every owner's whole list each step
                msg += (f"; dp_owner's X5 row broadcast then all-gathers {self.W * self.S5 * 4 / 2**20:.1f} MiB "
                        f"per rank per step (W x the {self.S5 * 4 / 2**20:.1f} MiB list capacity, however few "
                        f"rows changed)")
            log.warning(msg)
            if self.rank == 0:
                print(f"[rocfm] {msg}", flush=True)
            self._fallback_to_collective()

    def _fallback_to_collective(self) -> None:
        """Agreed switch of X1-X4 from the p2p pushes to the process group's collectives (every
        rank).  The receive buffers' contents (replica, already-served rows / requests) move over."""
        torch.cuda.synchronize(self.device)
        self._graphs = {}
        self._ms_S = None
        old = [self.rows_in, self.grad_back] + (list(self.recv_pair) if self.recv_pair else [self.recv_ids])
        keep = [t.clone() for t in old]
        xs = self.x_all
        self._bind_exchange(None)
        new = [self.rows_in, self.grad_back] + (list(self.recv_pair) if self.recv_pair else [self.recv_ids])
        for dst, src in zip(new, keep):
            dst.copy_(src)
        torch.cuda.synchronize(self.device)
        for ex in xs:
            ex.close()
        self._build()

    def replicated_tensors(self):
        e = self.eng
        full = [self.emb_full] if self.replicate else []
        return [e.dense, e.steps, self.hot_rep] + list(e.dense_slots) + list(self.hot_slots) + full

    def verify_replicas(self) -> bool:
        """Collective: the replicated state (MLP, its slots, the step, replicated hot rows) is
        bit-identical on every rank."""
        if self.W == 1:
            return True
        torch.cuda.synchronize(self.device)
        if self._corrupt_replica:  # fault injection (tests)
            self._corrupt_replica = False
            self.eng.dense.view(-1)[0] += 1e-3
        from .validate import replicas_agree

        return replicas_agree(self.replicated_tensors())

    def _after_steps(self, i0: int, i1: int) -> None:
        if self.check_every and i1 // self.check_every != i0 // self.check_every:
            self.check()

    def precapture(self, n: int, steps_per_graph: int = 16) -> None:
        """Capture the graphs ``train_steps(n, steps_per_graph)`` will replay (no launch)."""
        e = self.eng
        if getattr(self, "_ms_S", None) == steps_per_graph and e._m_primed and self.graph_collectives \
                and self.use_graph and not e._ring and steps_per_graph > 1:
            e._precapture_multi(self._graphs, ("mrs",), n, self._enqueue_multi_rs, "thread_local")

    def train_steps(self, n: int, steps_per_graph: int = 16) -> None:
        e = self.eng
        while n > 0 and self.shadow.active:  # validated steps first (eager, collective shadow)
            self.train_step()
            n -= 1
        if n <= 0:
            return
        if self.graph_collectives and self.use_graph and not e._ring and steps_per_graph > 1:
            self._train_steps_multi(n, steps_per_graph)
            return
        if self.staleness:
            for _ in range(n):
                self.train_step()
            return
        S = max(2, steps_per_graph // 2 * 2)
        while n > 0:
            if (self.graph_collectives and self.use_graph and self._warm >= 4 and e._primed and n >= S
                    and e._i % 2 == 0 and not e._ring):
                key = ("multi", S)
                g = self._graphs.get(key)
                if g is None:
                    g = torch.cuda.CUDAGraph()
                    torch.cuda.synchronize(self.device)
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):
                        for k in range(S):
                            self._step_body(k % 2)
                    self._graphs[key] = g
                g.replay()
                e._i += S
                self._warm += S
                n -= S
                self._after_steps(e._i - S, e._i)
            else:
                self.train_step()
                n -= 1

    def close(self) -> None:
        """Release the captured graphs (required before destroy_process_group when they hold
        RCCL collectives) and the peer-mapped exchange buffers."""
        torch.cuda.synchronize(self.device)
        self._graphs = {}
        if self.exchange == "p2p":
            self.recv_ids = self.rows_in = self.grad_back = self.recv_pair = None  # views of the buffers freed below
            self.p2p_x = {}
            for ex in self.x_all:
                ex.close()
            self.exchange = "closed"

    # ---- multi-step graphs (pool mode, capturable collectives) -----------------------------------
    # FusedDeepFM's multi-step pipeline with row-shard routing: the side chain of a graph fetches
    # the next graph's S batches with owner-major sort keys, sorts them at once and routes every
    # batch (S route launches); each step then runs X1 → serve → X2 → rows → tail → X3 → X4 →
    # owner merge ‖ MLP optimizer → merge apply, collectives captured inline.
    def _build_multi_rs(self, Smax: int) -> None:
        e, H = self.eng, self.H
        self._graphs = {}  # captured graphs hold the previous parameter blocks / buffers
        W, cap, n, F = self.W, self.cap, self.n, e.F
        e._build_multi(Smax, shard=(W, self.Vs) + ((self.hot_ids_dev[: self.n_hot],) if self.n_hot else ()))
        e._m_pool = e.pool_ids
        S_ = e.mS
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.ms_send = torch.full((2, S_, W * cap), PAD, **i32)
        self.ms_local = torch.zeros(2, S_, e.Bp, F, **i32)
        self.ms_skl = torch.zeros(2, S_, n, **i32)
        self.ms_counts = torch.zeros(2, S_, W, **i32)
        self.ms_scratch = torch.zeros(H.route_scratch_ints(n), **i32)
        self.ms_route = []
        self.ms_steps = []
        for q in range(2):
            routes, steps = [], []
            for k in range(S_):
                rp = H.ShardRouteParams()
                rp.skeys, rp.svals, rp.n = e.m_sk[q, k * n:].data_ptr(), e.m_sv[q, k * n:].data_ptr(), n
                rp.W, rp.Vs, rp.cap = W, self.Vs, cap
                rp.key_base, rp.val_base = (k << e.m_idbits) if e.m_composite else 0, k * n
                rp.send_ids, rp.local_idx = self.ms_send[q, k].data_ptr(), self.ms_local[q, k].data_ptr()
                rp.skeys_local, rp.counts = self.ms_skl[q, k].data_ptr(), self.ms_counts[q, k].data_ptr()
                rp.overflow, rp.scratch = self.overflow.data_ptr(), self.ms_scratch.data_ptr()
                routes.append(rp)
                rows, wp, da, ep, ed = e.m_params[q][k]
                rows.ids, rows.emb = self.ms_local[q, k].data_ptr(), self.rows_in.data_ptr()
                rows.tbl_bf16 = 0
                self._bind_replica(rows, e.m_ids[q, k])
                wp.grads = e.dense_grads_flat.data_ptr()
                self._set_push(rows, wp, ep)
                ep.skeys, ep.n = self.ms_skl[q, k].data_ptr(), n
                ep.mode, ep.dense_grad, ep.id_offset, ep.max_key = 1, self.grad_stage.data_ptr(), 0, 0
                ep.touched = 0
                ep.grad_scale = 1.0
                self._bind_hot_out(ep)
                da.apply, da.grad_scale = 1, 1.0 / W
                self._set_mlp_grads(da)
                mg = H.MergeParams()
                src = self.owner_params[0]
                for f in ("keys", "rows", "counts", "key_stride", "row_stride", "count_stride", "W", "cap", "Kp",
                          "K1", "key_div", "Vmap", "emb", "s0", "s1", "l2", "grad_scale", "mode",
                          "dense_grad", "touched", "tbl_bf16", "pos", "rep", "hash_slots", "hkeys", "hrep",
                          "hpos", "use_maps", "bc_count", "bc_keys", "bc_rows", "bc_cap", "bc_mul", "bc_add",
                          "bc_push"):
                    setattr(mg, f, getattr(src, f))
                mg.opt, mg.step = ep.opt, ep.step  # this step's global_step / lr_t
                par = k % 2 if self.recv_pair is not None else 0
                mg.keys = self._recv_ids_for(self.ms_send[q, k], par).data_ptr()
                if ed is not None:
                    ed.grad_scale = 1.0
                steps.append((rows, wp, ep, da, ed, mg, self._serve_params(self._recv_ids_for(self.ms_send[q, k], par)),
                              self._hot_params(ep, mg.opt, mg.step)))
            self.ms_route.append(routes)
            self.ms_steps.append(steps)

        def route_all(q, stream):
            for rp in self.ms_route[q]:
                H.shard_route(rp, stream.cuda_stream)

        e._m_post = route_all
        self._ms_S = Smax

    def _enqueue_multi_rs(self, q: int, S: int) -> None:
        """Main chain of one S-step row-shard graph (the side graph is launched by
        FusedDeepFM._launch_multi)."""
        e, H = self.eng, self.H
        s = torch.cuda.current_stream(self.device).cuda_stream
        st = self.staleness
        ahead = self.x1_ahead  # X1 of step k+1 rides step k's X3/X4 hand-off
        for k in range(S):
            rows, wp, ep, da, ed, mg, sv, hot = self.ms_steps[q][k]
            par = k % 2 if self.recv_pair is not None else 0
            rep_ = self.replicate  # dp_owner: no serve / X2; X1 rides this step's X3/X4 hand-off
            if not rep_ and (k == 0 or not (st or ahead)):  # (later steps: requested by the previous step)
                self._exchange(self._recv(par), self.ms_send[q, k])             # X1 requests
            if not rep_ and (k == 0 or not st):  # (staleness 1: later steps were served by the previous update)
                H.shard_serve(sv, s)
                self._exchange(self.rows_x, self.rows_out[:self.M])                     # X2 rows
            H.deepfm_rows(rows, s)
            e._tail(wp, ep, None, s)                                            # wgrad ‖ Σ rows per request
            nxt = (self._recv(1 - par), self.ms_send[q, k + 1]) if (st or ahead) and k + 1 < S else None
            now = (self._recv(par), self.ms_send[q, k]) if rep_ else None
            self._x3_x4(nxt, now)                                               # X3 + X4 (+ X1)
            if self.maps is not None:
                H.merge_scatter(mg, s)                                          # (larger worlds)
            if st and k + 1 < S:  # owner merge ‖ MLP opt ‖ serve of step k+1
                H.merge_search_apply(mg, da, s, self.ms_steps[q][k + 1][6], hot)
                if ed is not None:
                    H.emb_dense_update(ed, s)
                self._exchange(self.rows_x, self.rows_out[:self.M])                     # X2 of step k+1
                continue
            H.merge_search_apply(mg, da, s, None, hot)                          # owner merge ‖ MLP opt ‖ hot
            if ed is not None:
                H.emb_dense_update(ed, s)
            if rep_:
                self._x5()                                                      # X5 updated rows → replicas

    def _train_steps_multi(self, n: int, Smax: int) -> None:
        e = self.eng
        if getattr(self, "_ms_S", None) != Smax or getattr(e, "_m_pool", None) is not e.pool_ids:
            self._build_multi_rs(Smax)
        if not e._m_primed:
            e._prime_multi()
        while n > 0:
            S = min(n, e.mS)
            e._launch_multi(self._graphs, ("mrs",), S, self._enqueue_multi_rs, capture_error_mode="thread_local")
            n -= S
            self._after_steps(e._i - S, e._i)
        torch.cuda.current_stream(self.device).wait_stream(e.sort_stream)
        e._primed = False
        self._pre_served = False

    # ---- streamed training (the Estimator's loader path at world > 1) ----------------------------
    def _stream_build(self, S: int) -> None:
        e = self.eng
        if getattr(self, "_ms_S", None) != S or getattr(e, "_m_pool", None) is not e.pool_ids:
            self._build_multi_rs(S)

    def _stream_run(self, n: int) -> None:
        e = self.eng
        e._launch_multi(self._graphs, ("mrs",), n, self._enqueue_multi_rs, capture_error_mode="thread_local")
        self._after_steps(e._i - n, e._i)

    def train_stream(self, batches, steps_per_graph: int = 16, after_steps=None, hold: int = 1,
                     ring_batches: int = 0) -> int:
        """Host batches → the HBM ring → multi-step graphs with X1-X4 inline (FusedDeepFM.train_stream
        with this engine's graphs).  The shadow-validation window trains per step first."""
        if not (self.graph_collectives and self.use_graph):
            raise RuntimeError("train_stream needs capturable exchanges (p2p, or RCCL with graphs)")
        from .dp import shadow_prefix

        batches, done, pre = shadow_prefix(self, batches, after_steps, with_prefix=True)
        if self.NH and self.hot_ids is None:  # replicated ids from the stream's first group
            first = next(iter(batches), None)
            if first is None:
                return done
            from ..data.tfrecord import RawGroup

            if isinstance(first, RawGroup):  # undecoded: parse a copy of its first batches
                from ..ops.decode import decode_on_device

                k = min(first.n, 8)
                ids = decode_on_device(first.bytes, first.offs, k, first.B, self.eng.F, self.device,
                                       self.eng.id_limit)[0]
            else:
                ids = first[0] if first[0].dim() == 3 else first[0].unsqueeze(0)
            self._choose_hot(ids[: min(len(ids), 8)].to(self.device))
            import itertools

            batches = itertools.chain([first], batches)
        n = self.eng.train_stream(batches, steps_per_graph, after_steps, hold, ring_batches,
                                  build=self._stream_build, run=self._stream_run, prefix=pre)
        self._pre_served = False
        return done + n

    def train_on(self, batches):
        it = iter(batches)
        cur = next(it, None)
        if cur is None:
            return
        self.load_batch(*cur)
        nxt = next(it, None)
        while True:
            if nxt is not None:
                self.push_batch(*nxt)
            self.train_step()
            yield
            if nxt is None:
                break
            nxt = next(it, None)

    def check(self, replicas: bool = True) -> None:
        """Raise if any owner's request list overflowed the exchange capacity (or a request was
        routed to the wrong owner) since construction, or (``replicas``; collective) if the
        replicated state differs across ranks."""
        self.eng.check()
        ov, bad = int(self.overflow.item()), int(self.bad.item())
        if ov:
            c = torch.stack(self.counts).max().item()
            raise RuntimeError(f"row-shard exchange overflow: an owner needed {c} rows > capacity {self.cap}; "
                               f"rebuild with capacity >= {c} (or capacity=batch_size*field_size)")
        if bad:
            raise RuntimeError("row-shard routing error: a rank received ids it does not own")
        if self.exchange == "p2p" and any(x.errored() for x in self.x_all):
            raise RuntimeError("row-shard p2p exchange: a peer wait timed out (rank missing or stalled)")
        if replicas and not self.verify_replicas():
            raise RuntimeError("row-shard replicas diverged: MLP / replicated rows differ across ranks")

    # ---- inference (collective) ------------------------------------------------------------------
    @torch.no_grad()
    def predict_batch(self, ids: torch.Tensor, vals: torch.Tensor, labels: Optional[torch.Tensor] = None):
        e = self.eng
        self._flush_hot()  # predictions read the replicated rows from their owners
        self._pre_served = False  # the prediction reuses the serve / row buffers
        nrows = int(ids.shape[0])
        nch = max(1, (nrows + e.B - 1) // e.B)
        if self.W > 1:
            t = torch.tensor([nch], dtype=torch.int64, device=self.device if dist.get_backend() == "nccl" else "cpu")
            all_reduce_(t, dist.ReduceOp.MAX)
            nch = int(t.item())
        probs, losses = [], []
        for c in range(nch):
            a, b = min(c * e.B, nrows), min((c + 1) * e.B, nrows)
            m = b - a
            if m:
                e.pred_ids[:m].copy_(ids[a:b])
                e.pred_vals[:m].copy_(vals[a:b])
                if labels is not None:
                    e.pred_labels[:m].copy_(labels[a:b])
                else:
                    e.pred_labels.zero_()
            kp, rp = self.pred_route
            kp.n = rp.n = m * e.F
            self._route_launch(self.pred_route, m * e.F, torch.cuda.current_stream(self.device))
            self._exchange(self.recv_ids, self.pred_send)
            self.H.shard_serve(self.pred_serve, e.stream_ptr)
            self._exchange(self.rows_x, self.rows_out[:self.M])
            if m:
                pp = e.pred_params
                pp.B = m
                self.H.deepfm_rows(pp, e.stream_ptr)
                probs.append(e.pred_prob[:m].clone())
                losses.append(e.pred_loss[:m].clone())
        if not probs:
            z = torch.zeros(0, device=self.device)
            return z, z
        return torch.cat(probs), torch.cat(losses)

    # ---- bookkeeping ----------------------------------------------------------------------------
    def l2_value(self) -> float:
        e = self.eng
        self._flush_hot()
        nb = 1024
        part = torch.zeros(nb, dtype=torch.float32, device=self.device)
        self.H.emb_sumsq(e.emb.data_ptr(), e.V * e.Kp // 4, e.Kp, e.K1, part.data_ptr(), nb, e.stream_ptr, e.tbl_bf16)
        t = part.double().sum().reshape(1)
        if self.W > 1:
            all_reduce_(t)
        return float(self.spec.l2_reg * 0.5 * t.item())

    def batch_loss(self, include_l2: bool = True) -> float:
        v = self.eng.batch_loss(include_l2=False)
        return v + (self.l2_value() if include_l2 else 0.0)

    def global_step(self) -> int:
        return self.eng._i

    def row_sets(self) -> Dict[str, torch.Tensor]:
        rows = shard_rows(self.V, self.W, self.rank)
        names = ["fm_w", "fm_v"] + [f"{t}/{s}" for t in ("fm_w", "fm_v") for s in slot_names(self.hp.name)]
        return {k: rows for k in names}

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        self._flush_hot()
        sd = self.eng.state_dict()
        for k in self.row_sets():
            sd[k] = sd[k][: self.n_loc].clone()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        sd = _localize(sd, self.row_sets(), self.V, self.W, self.rank, self.Vs, self.n_loc)
        self.eng.load_state_dict(sd, strict=strict)
        self._load_hot()
        if self.replicate:
            self._sync_full()
        if self.maps is not None:
            self.maps.reset()  # the hash merge tags words with the step, which just moved
        self._pre_served = False
        self._graphs = {}
        self._warm = 0

    def dense_parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        """Every variable except the row-sharded tables (no collective)."""
        e = self.eng
        tf = e._tf_views(e.emb, e.dense)
        tf.update(e._bn_views())
        return OrderedDict((k, v.detach().float().cpu().clone()) for k, v in tf.items() if k not in ("fm_w", "fm_v"))

    def iter_table_chunks(self, chunk_rows: Optional[int] = None):
        """Collective: the full tables in id order, one gathered row range at a time (streamed
        servable export: ``checkpoint.StreamedServable``)."""
        self._flush_hot()
        torch.cuda.synchronize(self.device)
        yield from iter_table_chunks(self.eng.emb, self.V, self.W, self.eng.K, chunk_rows)

    def parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        e = self.eng
        self._flush_hot()
        out = e.parameters_tf()
        if self.W > 1:
            out["fm_w"] = _gather_table(e.emb[:, e.K].float().contiguous(), self.V, self.W).cpu()
            out["fm_v"] = _gather_table(e.emb[:, : e.K].float().contiguous(), self.V, self.W).cpu()
        else:
            out["fm_w"], out["fm_v"] = out["fm_w"][: self.V], out["fm_v"][: self.V]
        return out

    def __getattr__(self, name):
        return getattr(self.__dict__["eng"], name)
