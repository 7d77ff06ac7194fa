"""Fused MI355X training engine for DeepFM (the HIP path).

One training step on one GPU is three kernels on the critical path plus a side stream that
prepares the NEXT step's batch, captured once per step parity into a HIP graph and replayed:

    side stream : fetch_batch     — copy batch i+1 from the device pool into its input slot (batch.hip)
                  sort_pairs      — radix sort of its (id, lookup) pairs (sort.hip)
    main stream : deepfm_rows     — gather + FM + MLP fwd + head + MLP bwd + FM bwd (deepfm_rows.hip)
                  mlp_wgrad       — dW/db on MFMA + fused optimizer + bf16 weight refresh (mlp_wgrad.hip)
                  emb_rows_update — sorted segment-sum of lookup grads + row optimizer (emb_update.hip)

which replaces the reference's per-step TF graph (PS:172-313 ≡ HVD:164-303 forward/backward +
ApplyAdam ×11 variables).  ``embedding_update='exact'`` keeps the reference semantics of the
full-table L2 (dense gradient, every row's optimizer slots move every step) by
writing the summed lookup gradients into a dense table and running one dense update kernel.

State layout (device):
  emb   [V, Kp] f32 — fm_v in columns 0..K-1, fm_w in column K, zero padding (Kp = 4·⌈(K+1)/4⌉)
  dense [P] f32     — MLP weights/biases (dims padded to 32), deep_out, fm_bias (DenseLayout)
  WT/Wb             — bf16 copies of each hidden layer's W (forward / backward MFMA operands)
  slots             — optimizer state with the same layouts (Adam m,v; Adagrad acc; …)
  steps [2] int64   — global_step by step parity, read by the kernels (Adam bias correction,
                      dropout keys); the side-stream fetch of step i publishes step i+1
"""
from __future__ import annotations

import dataclasses
import math
import os
import time
from collections import OrderedDict
from typing import Dict, List, Optional

import torch

from ..data.tfrecord import RawGroup
from ..optim import OPT_ID, OptHParams, init_slots, slot_names
from ..ops import require_hip
from ..utils import hazard
from .deepfm import ModelSpec, init_params, mlp_names


def sort_lib() -> str:
    """The (key, index) sort behind every embedding-gradient aggregation: ``rocfm`` (default) — the
    segmented stable radix sort of csrc/kernels/seg_sort.hip; ``rocprim`` (ROCFM_SORT_LIB=rocprim)
    — rocPRIM's device radix sort over the composite keys (A/B; profiles/r4_seg_sort.md)."""
    return "rocprim" if os.environ.get("ROCFM_SORT_LIB", "") == "rocprim" else "rocfm"


def iota_sort_temp_bytes(H, n: int, bits: int, nseg: int = 1, seg_bits: int = 0) -> int:
    """Temporary bytes of ``iota_sort`` over ``nseg`` segments of ``n`` keys."""
    if sort_lib() == "rocprim":
        return H.sort_pairs_temp_bytes(nseg * n, bits + seg_bits)
    return H.seg_sort_temp_bytes(nseg, n, bits)


def iota_sort(H, temp, kin: int, kout: int, vout: int, n: int, bits: int, stream: int, nseg: int = 1,
              seg_bits: int = 0) -> None:
    """Stable sort of ``nseg`` segments of ``n`` keys each by key bits [0, bits), values = global
    index.  Segment k's keys must carry k in bits [bits, bits + seg_bits) when nseg > 1 (the
    composite keys of the multi-step side chain): rocPRIM sorts them as ONE array on those bits."""
    if sort_lib() == "rocprim":
        H.sort_pairs_iota(temp.data_ptr(), temp.numel(), kin, kout, vout, nseg * n, bits + seg_bits, stream)
    else:
        H.seg_sort_iota(temp.data_ptr(), temp.numel(), kin, kout, vout, nseg, n, bits, stream)


def _r32(x: int) -> int:
    return (x + 31) // 32 * 32


class DenseLayout:
    """Flat f32 layout of every non-embedding parameter."""

    def __init__(self, spec: ModelSpec):
        self.spec = spec
        real = [spec.deep_in] + list(spec.layers)
        self.real = real
        self.dims = [_r32(d) for d in real]
        self.nl = len(spec.layers)
        off = 0
        self.offW, self.offb = [], []
        for l in range(self.nl):
            self.offW.append(off)
            off += self.dims[l] * self.dims[l + 1]
            self.offb.append(off)
            off += self.dims[l + 1]
        self.off_wout = off
        off += self.dims[self.nl]
        self.off_bout = off
        off += 1
        self.off_fmb = off
        off += 1
        # batch_norm: trainable γ / β per hidden layer (padded columns: γ 1, β 0 — they stay 0)
        self.off_gamma, self.off_beta = [], []
        if spec.batch_norm:
            for l in range(self.nl):
                self.off_gamma.append(off)
                off += self.dims[l + 1]
                self.off_beta.append(off)
                off += self.dims[l + 1]
        self.total = (off + 3) // 4 * 4

    def views(self, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        """TF-named views (unpadded) into a flat buffer (params or any slot)."""
        v: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        v["fm_bias"] = flat[self.off_fmb:self.off_fmb + 1]
        for l, (wn, bn) in enumerate(mlp_names(self.spec)[:-1]):
            W = flat[self.offW[l]:self.offW[l] + self.dims[l] * self.dims[l + 1]].view(self.dims[l], self.dims[l + 1])
            v[wn] = W[: self.real[l], : self.real[l + 1]]
            v[bn] = flat[self.offb[l]:self.offb[l] + self.real[l + 1]]
            if self.spec.batch_norm:
                v[f"Deep-part/bn_{l}/beta"] = flat[self.off_beta[l]:self.off_beta[l] + self.real[l + 1]]
                v[f"Deep-part/bn_{l}/gamma"] = flat[self.off_gamma[l]:self.off_gamma[l] + self.real[l + 1]]
        wn, bn = mlp_names(self.spec)[-1]
        v[wn] = flat[self.off_wout:self.off_wout + self.real[self.nl]].view(-1, 1)
        v[bn] = flat[self.off_bout:self.off_bout + 1]
        return v

    def pack(self, P: Dict[str, torch.Tensor], flat: torch.Tensor) -> None:
        flat.zero_()
        for name, view in self.views(flat).items():
            view.copy_(P[name].reshape(view.shape))


class FusedDeepFM:
    """Device-resident DeepFM state + the fused HIP training/inference steps for one GPU.

    Step pipeline (parity p = step % 2; every buffer a step reads is double-buffered):

        side : fetch batch i+1 → input slot 1−p ; radix-sort its ids → keys[1−p]
        main : deepfm_rows(slot p) → mlp_wgrad → emb_rows_update(keys[p]) ; join side

    so the batch copy and the sort are off the critical path.  Batches come from a device pool
    ([NB,B,F]): an HBM-resident dataset (``attach_pool``) or a 2-slot staging ring fed with
    ``push_batch`` one batch ahead (the Estimator's loader path).
    """

    def __init__(self, spec: ModelSpec, hp: OptHParams, batch_size: int, device="cuda",
                 embedding_update: str = "sparse", seed: int = 1234,
                 params: Optional[Dict[str, torch.Tensor]] = None, grad_scale: float = 1.0,
                 use_graph: bool = True, fuse_dense_opt: bool = True, dropout_seed: Optional[int] = None,
                 force_generic_kernels: bool = False, compute_dtype: str = "bf16", table_dtype: str = "f32",
                 dedup: Optional[bool] = None):
        if len(spec.layers) > 6:
            raise ValueError("the fused engine supports at most 6 hidden layers")
        self.H = require_hip()
        # ROCFM_HAZARD=1: launches recorded, each new side/main graph pair checked for shared buffers
        self._hazard = None
        if hazard.enabled():
            self._hazard = hazard.Recorder()
            self._hazard.attach("eng", self)
            self.H = hazard.HipProxy(self.H, self._hazard)
        self.spec, self.hp = spec, hp
        self.device = torch.device(device)
        self.B = int(batch_size)
        self.Bp = (self.B + 127) // 128 * 128
        self.F, self.K = spec.field_size, spec.embedding_size
        self.K1 = self.K + 1
        self.Kp = (self.K1 + 3) // 4 * 4
        if self.Kp > 64:
            raise ValueError("embedding_size must be <= 63 for the fused engine")
        self.V = spec.feature_size
        self.layout = DenseLayout(spec)
        self.embedding_update = embedding_update
        self.grad_scale = float(grad_scale)
        self.use_graph = use_graph
        self.fuse_dense_opt = fuse_dense_opt
        self.seed = int(seed if dropout_seed is None else dropout_seed)
        self.loss_code = 0 if spec.loss_type == "log_loss" else 1
        self.lr_scale = 1.0
        self.force_generic = bool(force_generic_kernels)
        # examples per row-kernel workgroup (compile-time-shape kernels): 16, 8 or 4 — more, smaller
        # workgroups on the 256-CU chip (ROCFM_ROW_TILE; 0 = the kernel's default, 8)
        self.row_tile = int(os.environ.get("ROCFM_ROW_TILE", "0"))
        if self.row_tile not in (0, 4, 8, 16):
            raise ValueError(f"ROCFM_ROW_TILE must be 0, 4, 8 or 16, got {self.row_tile}")
        if compute_dtype not in ("bf16", "fp8"):
            raise ValueError(f"compute_dtype must be bf16 or fp8, got {compute_dtype!r}")
        self.compute_dtype = compute_dtype
        # table_dtype bf16: fm_v / fm_w rows stored as bf16 (half the HBM and
        # gather bytes; 1B rows = 24 GB instead of 48 GB), updated in f32 with stochastic rounding;
        # optimizer slots and the exact-mode gradient table stay f32
        if table_dtype not in ("f32", "bf16"):
            raise ValueError(f"table_dtype must be f32 or bf16, got {table_dtype!r}")
        self.table_dtype = table_dtype
        self.tbl_bf16 = 1 if table_dtype == "bf16" else 0
        dev = self.device
        L = self.layout

        # ---- parameters + optimizer state ----------------------------------------------------
        self.emb = torch.zeros(self.V, self.Kp, dtype=torch.bfloat16 if self.tbl_bf16 else torch.float32, device=dev)
        if params is not None:
            P = params
            self.emb[:, : self.K].copy_(P["fm_v"])
            self.emb[:, self.K].copy_(P["fm_w"])
        else:  # tables drawn on the device in row chunks (no host copy of a 100M-1B-row table)
            P = init_params(dataclasses.replace(spec, feature_size=1), seed)
            self._init_table_device(seed)
        self.dense = torch.zeros(L.total, dtype=torch.float32, device=dev)
        L.pack({k: v.to(dev) for k, v in P.items() if k not in ("fm_w", "fm_v")}, self.dense)
        # f32 slots whatever the table dtype (an expanded scalar only carries shape / device)
        self.emb_slots = [x.contiguous() for x in init_slots(
            hp, torch.zeros((), dtype=torch.float32, device=dev).expand(self.V, self.Kp))]
        self.dense_slots = init_slots(hp, self.dense)
        # batch_norm: moving moments [layer][mean|var][column] (pads: mean 0, var 1) + the row
        # kernel's grid-reduction scratch (per-barrier partials, γ/β gradient sums, counters)
        self.bn = bool(spec.batch_norm)
        self.bn_dmax = max(L.dims[1:])
        if self.bn:
            self.bn_stats = torch.zeros(L.nl, 2, self.bn_dmax, dtype=torch.float32, device=dev)
            self.bn_stats[:, 1] = 1.0
            for l in range(L.nl):
                n = L.real[l + 1]
                self.bn_stats[l, 0, :n].copy_(P[f"Deep-part/bn_{l}/moving_mean"].reshape(-1))
                self.bn_stats[l, 1, :n].copy_(P[f"Deep-part/bn_{l}/moving_variance"].reshape(-1))
            nwg = (self.B + 127) // 128 * 128 // 16
            self.bn_part = torch.zeros(2 * L.nl, nwg, self.bn_dmax, 2, dtype=torch.float32, device=dev)
            self.bn_grad = torch.zeros(L.nl, 2, self.bn_dmax, dtype=torch.float32, device=dev)
            self.bn_sync = torch.zeros(4, dtype=torch.int32, device=dev)
            self.bn_error = torch.zeros(4, dtype=torch.int32, device=dev)
        # row-tile split (deepfm_rows.hip CtShape G; profiles/r5_layer0_split.md): two workgroups per
        # 8-row tile, each streaming half of a wide input layer's weights, with an in-launch exchange
        # of layer 0's outputs.  ROCFM_ROW_SPLIT = auto (wide input layers: dims[0] ≥ 1024 and a
        # 256-wide first hidden layer — the kernel has it for the reference's flag defaults), 1, 2.
        sp = os.environ.get("ROCFM_ROW_SPLIT", "auto")
        if sp not in ("auto", "1", "2"):
            raise ValueError(f"ROCFM_ROW_SPLIT must be auto, 1 or 2, got {sp!r}")
        self.row_split = 2 if (sp == "2" or (sp == "auto" and L.dims[0] >= 1024 and L.dims[1] >= 256)) else 1
        if self.row_split > 1:
            self.xbuf = torch.zeros(self.Bp // 8 * L.dims[1] * 16, dtype=torch.int16, device=dev)
            self.xctr = torch.zeros(self.Bp // 8, dtype=torch.int32, device=dev)
            self.xerr = torch.zeros(4, dtype=torch.int32, device=dev)
        self.WT = [torch.zeros(L.dims[l + 1], L.dims[l], dtype=torch.bfloat16, device=dev) for l in range(L.nl)]
        self.Wb = [torch.zeros(L.dims[l], L.dims[l + 1], dtype=torch.bfloat16, device=dev) for l in range(L.nl)]
        # MFMA-fragment-swizzled copies (common.h frag_swz): what the compile-time-shape row kernel loads
        self.WTs = [torch.zeros_like(w) for w in self.WT]
        self.Wbs = [torch.zeros_like(w) for w in self.Wb]
        # compute_dtype=fp8: pre-quantised e4m3 copies of the input layer's swizzled weights, one
        # scale per tensor from the previous weights' max |w| (deepfm_rows.h Fp8W0)
        self.w8 = None
        if self.compute_dtype == "fp8":
            self.w8 = (torch.zeros(self.WTs[0].numel(), dtype=torch.uint8, device=dev),
                       torch.zeros(self.Wbs[0].numel(), dtype=torch.uint8, device=dev),
                       torch.zeros(2, dtype=torch.float32, device=dev),   # amax by step parity
                       torch.zeros(1, dtype=torch.float32, device=dev))   # de-scale of the copies
        self.steps = torch.zeros(2, dtype=torch.int64, device=dev)   # global_step, by parity
        self.cursor = torch.zeros(2, dtype=torch.int64, device=dev)  # pool batch index, by parity
        self.lrt = torch.zeros(2, dtype=torch.float32, device=dev)     # per-step lr_t, by parity

        # ---- static step buffers (double-buffered by parity where the pipeline needs it) -------
        B, Bp, F = self.B, self.Bp, self.F
        self.slot_ids = [torch.zeros(Bp, F, dtype=torch.int32, device=dev) for _ in range(2)]
        self.slot_vals = [torch.zeros(Bp, F, dtype=torch.float32, device=dev) for _ in range(2)]
        self.slot_labels = [torch.zeros(Bp, dtype=torch.float32, device=dev) for _ in range(2)]
        self.prob = torch.zeros(Bp, dtype=torch.float32, device=dev)
        self.loss_rows = torch.zeros(Bp, dtype=torch.float32, device=dev)
        self.g = torch.zeros(Bp, dtype=torch.float32, device=dev)
        self.contrib = torch.zeros(B * F, self.Kp, dtype=torch.float32, device=dev)
        self.actT = [torch.zeros(L.dims[a], Bp, dtype=torch.bfloat16, device=dev) for a in range(L.nl + 1)]
        self.dzT = [torch.zeros(L.dims[a], Bp, dtype=torch.bfloat16, device=dev) if a > 0 else None
                    for a in range(L.nl + 1)]
        self.n_lookup = B * F
        # per-tile dedup (batch.h DedupParams; ROCFM_DEDUP=1, off by default): the row kernel sums
        # the gradient rows of each id within its row tile and the embedding update walks one entry
        # per (id, tile) — the numeric fields' fixed ids come as ≤ B/RT entries instead of B.
        # Measured at the bench config (profiles/r3_dedup.md): the tail 13.3 → 12.3 µs, the row
        # kernel +0.75 µs and the side chain's three extra launches per graph — no net gain
        if dedup is None:
            dedup = os.environ.get("ROCFM_DEDUP", "0") == "1"
        self.dedup = bool(dedup) and not self.bn
        self.end_bit = max(1, math.ceil(math.log2(max(self.V, 2))))
        self.skeys = [torch.zeros(self.n_lookup, dtype=torch.int32, device=dev) for _ in range(2)]
        self.svals = [torch.zeros(self.n_lookup, dtype=torch.int32, device=dev) for _ in range(2)]
        tb = iota_sort_temp_bytes(self.H, self.n_lookup, self.end_bit)
        self.sort_temp = torch.zeros(max(tb, 16), dtype=torch.uint8, device=dev)
        if self.dedup:  # per parity: group index / next member by lookup, compacted keys, count, run ends
            n, nch = self.n_lookup, (self.n_lookup + self.H.tail_chunk() - 1) // self.H.tail_chunk()
            self.d_pos = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
            self.d_nxt = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
            self.d_ckeys = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
            self.d_count = torch.zeros(2, dtype=torch.int32, device=dev)
            self.d_cend = [torch.zeros(nch, dtype=torch.int32, device=dev) for _ in range(2)]
            self.d_bcount = [torch.zeros(self.H.dedup_scratch_ints(n, 1), dtype=torch.int32, device=dev)
                             for _ in range(2)]
        self.dense_grad = (torch.zeros_like(self.emb, dtype=torch.float32) if embedding_update == "exact" else None)
        # exact mode: rows whose dense_grad holds this step's gradient carry touched[row] = step + 1,
        # so the dense update reads / clears gradient rows only there (None: read every row —
        # dense_dp, whose gradient table arrives all-reduced)
        self.touched = (torch.zeros(self.V, dtype=torch.int32, device=dev) if embedding_update == "exact"
                        else None)
        self.dense_grads_flat = torch.zeros(L.total, dtype=torch.float32, device=dev)
        # side (fetch + sort), aux (mlp_wgrad beside the embedding update) and copy (train_stream's
        # H2D + device parse) streams: process-wide, so every engine gets the same hardware queues
        # whatever ran before it (utils/streams.py)
        from ..utils.streams import engine_streams

        self.sort_stream, self.aux_stream, self._copy_stream = engine_streams(dev)
        # ROCFM_LEAN_LAUNCH (bit mask, multi-step graph launches; profiles/r6_window_fixed_cost.md):
        # bit 0 preallocated launch events + no wait on a side graph already complete, bit 1 lazy
        # trailing join of the side chain
        self._lean_launch = int(os.environ.get("ROCFM_LEAN_LAUNCH", "3"))
        self._lean_evs = [[torch.cuda.Event(), torch.cuda.Event()] for _ in range(8)]
        self._side_join_pending = False
        # ROCFM_SIDE_AFTER_MAIN=1 (diagnostic): serialise each side graph behind its main graph, to
        # measure what the overlapped side chain costs the main chain
        self._side_after_main = os.environ.get("ROCFM_SIDE_AFTER_MAIN", "0") == "1"
        # inference buffers (separate from the training slots)
        self.pred_ids = torch.zeros(Bp, F, dtype=torch.int32, device=dev)
        self.pred_vals = torch.zeros(Bp, F, dtype=torch.float32, device=dev)
        self.pred_labels = torch.zeros(Bp, dtype=torch.float32, device=dev)
        self.pred_prob = torch.zeros(Bp, dtype=torch.float32, device=dev)
        self.pred_loss = torch.zeros(Bp, dtype=torch.float32, device=dev)
        # ROCFM_CHECK_IDS=1: device-side id guard in the batch fetch (out-of-range ids flag a sticky
        # error and are replaced by row 0, so no kernel indexes outside the table); check() raises.
        # id_limit is the GLOBAL vocabulary (the row-shard engine's local table is smaller).
        from ..utils.numerics import ids_check_enabled

        self.id_guard = ids_check_enabled()
        self.id_limit = self.V
        self.bad_ids = torch.zeros(1, dtype=torch.int32, device=dev)
        # the device Example parser's sticky error word [code, batch, record, -] (decode.hip); the
        # side chain's batch preparation reads it, and once it is set every prepared step is halted
        # (optim.h kHaltStepBit: no optimizer update), so a malformed record never trains
        self.halt_word = torch.zeros(4, dtype=torch.int32, device=dev)
        # default batch source: a 2-slot ring fed by push_batch()
        self._ring = True
        self._set_pool(torch.zeros(2, B, F, dtype=torch.int32, device=dev),
                       torch.zeros(2, B, F, dtype=torch.float32, device=dev),
                       torch.zeros(2, B, dtype=torch.float32, device=dev))
        self._pushed = 0

        self._i = 0  # completed steps (host mirror of global_step)
        self._primed = False
        self._m_primed = False
        self.mS = None
        self._graphs = [None, None]
        self._warm = 0
        self._build_params()
        self.refresh_bf16()

    def _init_table_device(self, seed: int, chunk_rows: int = 1 << 24) -> None:
        """fm_v / fm_w with the reference initialisers (TF glorot_normal over the full table's fans,
        truncated at ±2σ) drawn on the GPU chunk by chunk."""
        from ..models.deepfm import TRUNC_NORMAL_STD

        V, K = self.V, self.K
        gen = torch.Generator(device=self.device).manual_seed(int(seed) * 1000003 + 1)
        sv = math.sqrt(2.0 / (V + K)) / TRUNC_NORMAL_STD
        sw = math.sqrt(2.0 / (V + V)) / TRUNC_NORMAL_STD
        for r0 in range(0, V, chunk_rows):
            blk = self.emb[r0:min(V, r0 + chunk_rows)]
            x = torch.randn(blk.shape[0], K + 1, generator=gen, device=self.device)
            bad = x.abs() > 2.0
            while bool(bad.any()):
                x = torch.where(bad, torch.randn(x.shape, generator=gen, device=self.device), x)
                bad = x.abs() > 2.0
            blk[:, :K].copy_(x[:, :K] * sv)
            blk[:, K].copy_(x[:, K] * sw)
            del x, bad

    # ------------------------------------------------------------------------------------------
    def _opt(self, p: int = 0, lrt_ptr: Optional[int] = None):
        o = self.H.OptParams()
        o.lrt = self.lrt[p:].data_ptr() if lrt_ptr is None else lrt_ptr
        hp = self.hp
        o.type = OPT_ID[hp.name]
        o.lr = hp.lr * self.lr_scale
        o.beta1, o.beta2, o.eps = hp.beta1, hp.beta2, hp.eps
        o.momentum = hp.momentum
        o.ftrl_lr_power, o.ftrl_l1, o.ftrl_l2 = hp.ftrl_lr_power, hp.ftrl_l1, hp.ftrl_l2
        return o

    @staticmethod
    def _slot_ptrs(slots):
        s0 = slots[0].data_ptr() if len(slots) > 0 else 0
        s1 = slots[1].data_ptr() if len(slots) > 1 else 0
        return s0, s1

    def _rows_params(self, ids, vals, labels, prob, loss_rows, step_ptr, train):
        H, L = self.H, self.layout
        rp = H.RowsParams()
        rp.ids, rp.vals, rp.labels = ids.data_ptr(), vals.data_ptr(), labels.data_ptr()
        rp.emb = self.emb.data_ptr()
        rp.tbl_bf16 = self.tbl_bf16
        rp.fm_bias = self.dense[L.off_fmb:].data_ptr()
        rp.w_out = self.dense[L.off_wout:].data_ptr()
        rp.b_out = self.dense[L.off_bout:].data_ptr()
        rp.step = step_ptr
        rp.prob, rp.loss_rows, rp.g_out = prob.data_ptr(), loss_rows.data_ptr(), self.g.data_ptr()
        rp.contrib = self.contrib.data_ptr()
        rp.nl, rp.F, rp.K, rp.Kp, rp.B, rp.Bp = L.nl, self.F, self.K, self.Kp, self.B, self.Bp
        rp.inv_scale = 1.0 / self.B
        rp.train = 1 if train else 0
        rp.loss_type = self.loss_code
        rp.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        rp.force_generic = 1 if self.force_generic else 0
        rp.fp8 = 1 if self.compute_dtype == "fp8" else 0
        rp.row_tile = self.row_tile
        rp.wt = int(os.environ.get("ROCFM_WT", "0"))  # write-through row-kernel outputs (deepfm_rows.h wt)
        if self.row_split > 1:  # (the launcher keeps one workgroup per tile where the split does not apply)
            rp.split, rp.xbuf, rp.xctr, rp.xerr = 2, self.xbuf.data_ptr(), self.xctr.data_ptr(), self.xerr.data_ptr()
        self._set_w8(rp, 0)
        rp.dedup = 1 if (train and self.dedup) else 0
        rp.set_dims(L.dims)
        for l in range(L.nl):
            rp.set_layer(l, self.WT[l].data_ptr(), self.Wb[l].data_ptr(), self.dense[L.offb[l]:].data_ptr(),
                         float(self.spec.keep_probs[l]))
            rp.set_swz(l, self.WTs[l].data_ptr(), self.Wbs[l].data_ptr())
        for a in range(L.nl + 1):
            rp.set_act(a, self.actT[a].data_ptr(), self.dzT[a].data_ptr() if self.dzT[a] is not None else 0)
        if self.bn:
            rp.bn, rp.bn_decay, rp.bn_eps, rp.bn_dmax = 1, float(self.spec.batch_norm_decay), 1e-3, self.bn_dmax
            rp.bn_part, rp.bn_grad = self.bn_part.data_ptr(), self.bn_grad.data_ptr()
            rp.bn_sync, rp.bn_error = self.bn_sync.data_ptr(), self.bn_error.data_ptr()
            for l in range(L.nl):
                rp.set_bn(l, self.dense[L.off_gamma[l]:].data_ptr(), self.dense[L.off_beta[l]:].data_ptr(),
                          self.bn_stats[l, 0].data_ptr(), self.bn_stats[l, 1].data_ptr())
        if rp.dedup and rp.lds_bytes() > 160 * 1024 - 256:  # no room for the tile's gradient rows
            self.dedup = False
            rp.dedup = 0
        if rp.lds_bytes() > 160 * 1024 - 256:  # 256 B: the kernel's static LDS (diagnostic stamps)
            raise ValueError(f"field_size*embedding_size too large for the fused row kernel ({rp.lds_bytes()} B LDS)")
        return rp

    def _step_param_set(self, ids, vals, labels, step_ptr: int, lrt_ptr: int, skeys_ptr: int, svals_ptr: int,
                        val_base: int = 0, id_offset: int = 0):
        """Kernel parameter blocks of one step: (rows, wgrad, dense_apply, emb_update, emb_dense)."""
        H, L = self.H, self.layout
        rows = self._rows_params(ids, vals, labels, self.prob, self.loss_rows, step_ptr, True)
        wp = H.WgradParams()
        wp.g = self.g.data_ptr()
        wp.params = self.dense.data_ptr()
        wp.grads = self.dense_grads_flat.data_ptr()
        wp.s0, wp.s1 = self._slot_ptrs(self.dense_slots)
        wp.step = step_ptr
        wp.nl, wp.Bp = L.nl, self.Bp
        wp.off_wout, wp.off_bout, wp.off_fmb = L.off_wout, L.off_bout, L.off_fmb
        wp.fuse_opt = 1 if self.fuse_dense_opt else 0
        wp.opt = self._opt(lrt_ptr=lrt_ptr)
        wp.grad_scale = 1.0
        wp.set_dims(L.dims)
        for a in range(L.nl + 1):
            wp.set_act(a, self.actT[a].data_ptr(), self.dzT[a].data_ptr() if self.dzT[a] is not None else 0)
        for l in range(L.nl):
            wp.set_layer(l, L.offW[l], L.offb[l], self.WT[l].data_ptr(), self.Wb[l].data_ptr())
            wp.set_swz(l, self.WTs[l].data_ptr(), self.Wbs[l].data_ptr())
        if self.fuse_dense_opt:
            self._set_w8(wp, 1)
        if self.bn:
            wp.bn, wp.bn_grad, wp.bn_dmax = 1, self.bn_grad.data_ptr(), self.bn_dmax
            for l in range(L.nl):
                wp.set_bn(l, L.off_gamma[l], L.off_beta[l])
        dp = H.DenseApplyParams()
        dp.params = self.dense.data_ptr()
        dp.grads = self.dense_grads_flat.data_ptr()
        dp.s0, dp.s1 = self._slot_ptrs(self.dense_slots)
        dp.step = step_ptr
        dp.n, dp.nl = L.total, L.nl
        dp.opt = self._opt(lrt_ptr=lrt_ptr)
        dp.set_dims(L.dims)
        for l in range(L.nl):
            dp.set_layer(l, L.offW[l], self.WT[l].data_ptr(), self.Wb[l].data_ptr())
            dp.set_swz(l, self.WTs[l].data_ptr(), self.Wbs[l].data_ptr())
        self._set_w8(dp, 1)
        ep = H.EmbUpdateParams()
        ep.skeys, ep.svals = skeys_ptr, svals_ptr
        ep.n = self.n_lookup
        ep.val_base, ep.id_offset = val_base, id_offset
        ep.contrib = self.contrib.data_ptr()
        ep.K1, ep.Kp = self.K1, self.Kp
        ep.emb = self.emb.data_ptr()
        ep.tbl_bf16 = self.tbl_bf16
        ep.s0, ep.s1 = self._slot_ptrs(self.emb_slots)
        ep.l2 = float(self.spec.l2_reg)
        ep.grad_scale = 1.0
        ep.opt = self._opt(lrt_ptr=lrt_ptr)
        ep.step = step_ptr
        ep.mode = 1 if self.embedding_update == "exact" else 0
        if self.dense_grad is not None:
            ep.dense_grad = self.dense_grad.data_ptr()
        if self.touched is not None:
            ep.touched = self.touched.data_ptr()
        ed = None
        if self.embedding_update == "exact":
            ed = H.EmbDenseParams()
            ed.emb = self.emb.data_ptr()
            ed.tbl_bf16 = self.tbl_bf16
            ed.s0, ed.s1 = self._slot_ptrs(self.emb_slots)
            ed.dense_grad = self.dense_grad.data_ptr()
            ed.touched = self.touched.data_ptr() if self.touched is not None else 0
            ed.step = step_ptr
            ed.n4 = self.V * self.Kp // 4
            ed.Kp, ed.K1 = self.Kp, self.K1
            ed.l2 = float(self.spec.l2_reg)
            ed.opt = self._opt(lrt_ptr=lrt_ptr)
        return rows, wp, dp, ep, ed

    def _build_params(self):
        self.rows_params, self.wgrad_params, self.dense_apply_params = [], [], []
        self.emb_params, self.emb_dense_params = [], []
        for p in range(2):
            rows, wp, dp, ep, ed = self._step_param_set(
                self.slot_ids[p], self.slot_vals[p], self.slot_labels[p], self.steps[p:].data_ptr(),
                self.lrt[p:].data_ptr(), self.skeys[p].data_ptr(), self.svals[p].data_ptr())
            self.rows_params.append(rows)
            self.wgrad_params.append(wp)
            self.dense_apply_params.append(dp)
            self.emb_params.append(ep)
            if ed is not None:
                self.emb_dense_params.append(ed)
            if self.dedup:  # the per-step sort's dedup outputs of this parity (_sort)
                rows.contrib_pos, rows.contrib_nxt = self.d_pos[p].data_ptr(), self.d_nxt[p].data_ptr()
                ep.skeys, ep.n_dev, ep.sorted_contrib = self.d_ckeys[p].data_ptr(), self.d_count[p:].data_ptr(), 1
                if self.Kp <= self.H.tail_max_kp():
                    ep.chunk_end = self.d_cend[p].data_ptr()
        if self.dedup:
            self._rt = self.H.deepfm_rows_tile(self.rows_params[0])  # the row tiles the dedup must cut
        self.pred_params = self._rows_params(self.pred_ids, self.pred_vals, self.pred_labels, self.pred_prob,
                                             self.pred_loss, self.steps.data_ptr(), False)
        self._build_fetch()

    def _build_fetch(self):
        H = self.H
        self.fetch_params = []
        for p in range(2):  # step with parity p fetches batch cur[p]+1 into slot 1-p
            f = H.FetchParams()
            f.ids_pool, f.vals_pool, f.labels_pool = (self.pool_ids.data_ptr(), self.pool_vals.data_ptr(),
                                                      self.pool_labels.data_ptr())
            f.pool_batches = self.pool_ids.shape[0]
            f.B, f.F = self.B, self.F
            f.cur_src, f.cur_dst, f.advance = self.cursor[p:].data_ptr(), self.cursor[1 - p:].data_ptr(), 1
            f.step_src, f.step_dst, f.step_advance = self.steps[p:].data_ptr(), self.steps[1 - p:].data_ptr(), 1
            f.ids, f.vals, f.labels = (self.slot_ids[1 - p].data_ptr(), self.slot_vals[1 - p].data_ptr(),
                                       self.slot_labels[1 - p].data_ptr())
            f.lrt_dst = self.lrt[1 - p:].data_ptr()
            f.lr, f.beta1, f.beta2 = self.hp.lr * self.lr_scale, self.hp.beta1, self.hp.beta2
            f.opt_type = OPT_ID[self.hp.name]
            self._guard(f)
            self.fetch_params.append(f)

    def _guard(self, f) -> None:
        if self.id_guard:
            f.bad_ids, f.max_id = self.bad_ids.data_ptr(), int(self.id_limit)

    def _set_pool(self, ids, vals, labels):
        if ids.dim() != 3 or ids.shape[1:] != (self.B, self.F) or vals.shape != ids.shape or \
                labels.shape != ids.shape[:2]:
            raise ValueError(f"pool must be ids/vals [NB,{self.B},{self.F}], labels [NB,{self.B}]")
        self.pool_ids = ids.to(self.device, torch.int32).contiguous()
        self.pool_vals = vals.to(self.device, torch.float32).contiguous()
        self.pool_labels = labels.to(self.device, torch.float32).contiguous()

    def attach_pool(self, ids: torch.Tensor, vals: torch.Tensor, labels: torch.Tensor, start: int = 0) -> None:
        """Train from a device-resident pool of batches ([NB,B,F] ids/vals, [NB,B] labels), cycling."""
        self._join_side_chain()
        self._set_pool(ids, vals, labels)
        self._ring = False
        self._build_fetch()
        self._graphs = [None, None]
        self._multi_graph = None
        self._primed = False
        self._m_primed = False
        self._start_batch = start

    def push_batch(self, ids: torch.Tensor, vals: torch.Tensor, labels: torch.Tensor) -> None:
        """Ring mode: enqueue the next batch (must stay exactly one batch ahead of train_step)."""
        self._join_side_chain()
        if not self._ring:
            raise RuntimeError("push_batch() is for the loader ring; this engine trains from an attached pool")
        n = ids.shape[0]
        if n != self.B:
            raise ValueError(f"batch has {n} rows, engine built for {self.B} (drop_remainder semantics)")
        slot = self._pushed % 2
        self.pool_ids[slot].copy_(ids, non_blocking=True)
        self.pool_vals[slot].copy_(vals, non_blocking=True)
        self.pool_labels[slot].copy_(labels, non_blocking=True)
        self._pushed += 1

    def load_batch(self, ids, vals, labels=None) -> None:
        """Compatibility helper: make (ids, vals, labels) the batch of the NEXT train_step().

        Non-pipelined (re-primes the input slot); use push_batch/attach_pool for full speed.
        """
        self._join_side_chain()
        if labels is None:
            labels = torch.zeros(ids.shape[0], device=ids.device)
        if not self._ring:
            raise RuntimeError("load_batch() needs ring mode")
        self._pushed = self._i
        self.push_batch(ids, vals, labels)
        self._primed = False

    def train_on(self, batches):
        """Train one step per (ids, vals, labels) batch from an iterable, feeding the ring one ahead.

        Yields after each enqueued step (so callers can log / checkpoint between steps).
        """
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

    def set_lr_scale(self, s: float) -> None:
        """Multiply the learning rate (Horovod's lr × world size, HVD:171)."""
        self._join_side_chain()
        self.lr_scale = float(s)
        for lst in (self.wgrad_params, self.dense_apply_params, self.emb_params, self.emb_dense_params):
            for p, q in enumerate(lst):
                q.opt = self._opt(p)
        for f in self.fetch_params:
            f.lr = self.hp.lr * self.lr_scale
        self._graphs = [None, None]
        self._primed = False
        # the multi-step parameter blocks carry the lr: the next train_steps rebuilds them (through
        # the wrapper that built them — DP / row-shard add their own blocks on top)
        self._m_pool = None
        self._m_primed = False

    # ------------------------------------------------------------------------------------------
    @property
    def stream_ptr(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def _set_w8(self, prm, track: int) -> None:
        if self.w8 is not None:
            f, b, amax, inv = self.w8
            prm.set_w8(f.data_ptr(), b.data_ptr(), amax.data_ptr(), inv.data_ptr(), int(track))

    def refresh_bf16(self) -> None:
        """Rewrite the bf16 / swizzled (and fp8) weight copies from the f32 master weights."""
        self._join_side_chain()
        dp = self.dense_apply_params[0]
        dp.apply = 0
        if self.w8 is not None:  # host refresh: the exact max in both slots, no accumulation
            L = self.layout
            w0 = self.dense[L.offW[0]: L.offW[0] + L.dims[0] * L.dims[1]]
            self.w8[2].copy_(w0.abs().max().reshape(1).expand(2))
            self._set_w8(dp, 0)
        self.H.dense_apply(dp, self.stream_ptr)
        if self.w8 is not None:
            self._set_w8(dp, 1)

    def _sort(self, q: int, stream) -> None:
        iota_sort(self.H, self.sort_temp, self.slot_ids[q].data_ptr(), self.skeys[q].data_ptr(),
                  self.svals[q].data_ptr(), self.n_lookup, self.end_bit, stream.cuda_stream)
        if self.dedup:
            d = self.H.DedupParams()
            d.skeys, d.svals, d.n, d.S, d.F, d.rt = (self.skeys[q].data_ptr(), self.svals[q].data_ptr(),
                                                     self.n_lookup, 1, self.F, self._rt)
            d.val_base_step = 0
            d.pos, d.nxt, d.ckeys = self.d_pos[q].data_ptr(), self.d_nxt[q].data_ptr(), self.d_ckeys[q].data_ptr()
            d.count, d.bcount = self.d_count[q:].data_ptr(), self.d_bcount[q].data_ptr()
            d.chunk, d.chunk_end = self.H.tail_chunk(), self.d_cend[q].data_ptr()
            self.H.dedup(d, stream.cuda_stream)

    def prime(self) -> None:
        """Fetch + sort the current step's batch into its slot (before the first step / after a reset)."""
        self._join_side_chain()
        p = self._i % 2
        base = 0 if self._ring else getattr(self, "_start_batch", 0)
        self.cursor[p] = base + self._i
        self.steps[p] = self._i
        lr = self.hp.lr * self.lr_scale
        self.lrt[p] = (self.H.adam_lr_t(lr, self.hp.beta1, self.hp.beta2, self._i) if self.hp.name == "Adam" else lr)
        f = self.H.FetchParams()
        src = self.fetch_params[p]
        f.ids_pool, f.vals_pool, f.labels_pool, f.pool_batches = (src.ids_pool, src.vals_pool, src.labels_pool,
                                                                  src.pool_batches)
        f.B, f.F = self.B, self.F
        f.cur_src, f.cur_dst, f.advance = self.cursor[p:].data_ptr(), 0, 0
        f.step_src, f.step_dst, f.step_advance = self.steps[p:].data_ptr(), 0, 0
        f.ids, f.vals, f.labels = (self.slot_ids[p].data_ptr(), self.slot_vals[p].data_ptr(),
                                   self.slot_labels[p].data_ptr())
        self._guard(f)
        self.H.fetch_batch(f, self.stream_ptr)
        self._sort(p, torch.cuda.current_stream(self.device))
        self._primed = True

    # ---- the step ------------------------------------------------------------------------------
    def _fork_point(self):
        """Event marking the current position of the main stream (fork point for side streams).
        Forking from a recorded point lets the main stream's kernels be enqueued (and, in a
        graph, submitted) before the side stream's, without making the side wait for them."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _fork_next(self, p: int, fork=None):
        """Side stream: fetch + sort batch i+1 (into parity 1-p buffers)."""
        main = torch.cuda.current_stream(self.device)
        side = self.sort_stream
        if fork is None:
            side.wait_stream(main)
        else:
            side.wait_event(fork)
        with torch.cuda.stream(side):
            self.H.fetch_batch(self.fetch_params[p], side.cuda_stream)
            self._sort(1 - p, side)
        return side

    def _join(self, side) -> None:
        torch.cuda.current_stream(self.device).wait_stream(side)

    def _enqueue_forward_backward(self, p: int) -> None:
        s = self.stream_ptr
        self.H.deepfm_rows(self.rows_params[p], s)
        self.H.mlp_wgrad(self.wgrad_params[p], s)

    def _enqueue_rows_then_fork_wgrad(self, p: int):
        """rows kernel on the main stream, then mlp_wgrad on the aux stream (it only reads the
        activations; the embedding update on the main stream is independent of it)."""
        main = torch.cuda.current_stream(self.device)
        self.H.deepfm_rows(self.rows_params[p], main.cuda_stream)
        aux = self.aux_stream
        aux.wait_stream(main)
        with torch.cuda.stream(aux):
            self.H.mlp_wgrad(self.wgrad_params[p], aux.cuda_stream)
        return aux

    def _enqueue_emb_update(self, p: int) -> None:
        s = self.stream_ptr
        self.H.emb_rows_update(self.emb_params[p], s)
        if self.embedding_update == "exact":
            self.H.emb_dense_update(self.emb_dense_params[p], s)

    def _enqueue_step(self, p: int) -> None:
        # the side chain is forked first: in the captured graph it then gets its own hardware
        # queue and starts at once (forked later it was serialised behind the embedding update)
        side = self._fork_next(p)
        s = self.stream_ptr
        self.H.deepfm_rows(self.rows_params[p], s)
        self._tail(self.wgrad_params[p], self.emb_params[p],
                   self.emb_dense_params[p] if self.embedding_update == "exact" else None, s)
        self._join(side)

    def _enqueue_pipelined(self, S: int) -> None:
        """S consecutive steps for one multi-step graph, with the side chain decoupled from the
        step boundary: step k's side chain (fetch + sort of batch k+1) forks at the start of
        step k; step k+1's rows kernel waits only for that fetch and its embedding update only
        for that sort, so the sort overlaps the rest of step k AND the rows kernel of step k+1."""
        main = torch.cuda.current_stream(self.device)
        side = self.sort_stream
        prev = None
        for k in range(S):
            p = k % 2
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.H.fetch_batch(self.fetch_params[p], side.cuda_stream)
                ev_fetch = torch.cuda.Event()
                ev_fetch.record(side)
                self._sort(1 - p, side)
                ev_sort = torch.cuda.Event()
                ev_sort.record(side)
            if prev is not None:
                main.wait_event(prev[0])
            aux = self._enqueue_rows_then_fork_wgrad(p)
            if prev is not None:
                main.wait_event(prev[1])
            self._enqueue_emb_update(p)
            self._join(aux)
            prev = (ev_fetch, ev_sort)
        main.wait_stream(side)

    # ---- multi-step graphs (pool mode) ------------------------------------------------------------
    # One graph replays S steps whose main stream is strictly serial (rows → wgrad → emb_update per
    # step: cross-stream waits inside a graph cost more than the concurrency they buy — measured
    # 47 vs 55 µs/step); ONE side chain per graph prepares the NEXT graph's S batches (one copy
    # kernel) and sorts all S·B·F lookups at once (S segments of one batch each), joined at the
    # graph's end.
    def _multi_S(self, Smax: int, shard: Optional[tuple] = None):
        """(id bits, steps per graph).  Graphs of S steps sort all S·B·F lookups at once as S
        segments (seg_sort.hip: each batch on its own id bits).  While S << id_bits fits 32 bits
        (vocabularies up to 2^26 rows at S = 64) the keys carry their batch, ``k << id_bits | id``
        (``m_composite``: what rocPRIM's one-array sort needs, kept as the A/B); wider vocabularies
        (100M-1B rows) sort plain per-batch id keys (``m_plain``) — no 64-bit keys unless the
        rocPRIM A/B is asked for (ROCFM_SORT_LIB=rocprim: 64-bit composite keys)."""
        key_range = self.V if shard is None else (shard[0] + (len(shard) > 2)) * shard[1]  # + hot owner
        idbits = max(1, math.ceil(math.log2(max(key_range, 2))))
        return idbits, max(1, int(Smax))

    def _build_multi(self, Smax: int, shard: Optional[tuple] = None, heads: bool = False, plan: bool = False) -> None:
        """``shard=(W, Vs)``: the batches' sort keys are row-shard owner-major keys (emb_shard).
        ``heads``: the side chain also counts run heads per tail chunk (``m_chd``; the sorted DP
        export places each chunk's rows from them).  ``plan``: the single-GPU sparse update runs the
        planned step tail (``emb_plan.hip``: the side chain cuts every batch's sorted lookups into
        equal-cost items, one per embedding workgroup; ``ROCFM_EMB_PLAN=0`` keeps the fixed chunks)."""
        H, dev = self.H, self.device
        Bp, F, n = self.Bp, self.F, self.n_lookup
        self._m_shard = shard  # (W, Vs) or (W, Vs, hot ids tensor)
        self.m_req = int(Smax)
        idbits, Smax = self._multi_S(Smax, shard)
        sbits = math.ceil(math.log2(Smax)) if Smax > 1 else 0
        self.m_composite = (Smax << idbits) <= (1 << 32) and os.environ.get("ROCFM_SORT", "") != "wide"
        self.m_plain = not self.m_composite and sort_lib() == "rocfm"  # per-batch 32-bit id keys
        self.mS, self.m_idbits = Smax, idbits
        self.m_bits = idbits + sbits
        i32 = dict(dtype=torch.int32, device=dev)
        self.m_ids = torch.zeros(2, Smax, Bp, F, **i32)
        self.m_vals = torch.zeros(2, Smax, Bp, F, dtype=torch.float32, device=dev)
        self.m_labels = torch.zeros(2, Smax, Bp, dtype=torch.float32, device=dev)
        self.m_keys = torch.zeros(Smax * n, **i32)
        self.m_sk = torch.zeros(2, Smax * n, **i32)
        self.m_sv = torch.zeros(2, Smax * n, **i32)
        if self.m_composite or self.m_plain:
            tb = iota_sort_temp_bytes(H, n, idbits, Smax, sbits if self.m_composite else 0)
            self.m_keys64 = None
        else:  # rocPRIM A/B: 64-bit keys in / out (the sorted ids land in m_sk via sort_aux)
            tb = H.sort_pairs64_temp_bytes(Smax * n, self.m_bits)
            self.m_keys64 = torch.zeros(2, Smax * n, dtype=torch.int64, device=dev)
        self.m_temp = torch.zeros(max(tb, 16), dtype=torch.uint8, device=dev)
        # each lookup's position in its batch's sorted order (the row kernel writes its gradient row
        # there) and the per-chunk run ends of the fused step tail (sort_aux, side chain)
        self.m_pos = torch.zeros(2, Smax * n, **i32)
        self.m_chunk = self.H.tail_chunk()
        self.m_nch = (n + self.m_chunk - 1) // self.m_chunk
        self.m_cend = torch.zeros(2, Smax * self.m_nch, **i32)
        self.m_chd = torch.zeros(2, Smax * self.m_nch, **i32) if heads else None
        # per-tile dedup (rows of ONE batch per row tile): group links, compacted keys and counts
        self.m_dedup = self.dedup and shard is None
        if self.m_dedup:
            self.m_nxt = torch.zeros(2, Smax * n, **i32)
            self.m_ck = torch.zeros(2, Smax * n, **i32)
            self.m_cnt = torch.zeros(2, Smax, **i32)
            self.m_bcount = torch.zeros(self.H.dedup_scratch_ints(n, Smax), **i32)
        self.m_steps = torch.zeros(2, Smax, dtype=torch.int64, device=dev)
        self.m_lrt = torch.zeros(2, Smax, dtype=torch.float32, device=dev)
        self.m_cur = torch.zeros(2, dtype=torch.int64, device=dev)
        self.m_step = torch.zeros(2, dtype=torch.int64, device=dev)
        self.m_params = [[self._step_param_set(self.m_ids[q, k], self.m_vals[q, k], self.m_labels[q, k],
                                               self.m_steps[q, k:].data_ptr(), self.m_lrt[q, k:].data_ptr(),
                                               self.m_sk[q, k * n:].data_ptr(), self.m_sv[q, k * n:].data_ptr(),
                                               val_base=k * n, id_offset=(k << idbits) if self.m_composite else 0)
                          for k in range(Smax)] for q in range(2)]
        for q in range(2):
            for k in range(Smax):
                rows, _, _, ep, _ = self.m_params[q][k]
                rows.contrib_pos = self.m_pos[q, k * n:].data_ptr()
                ep.sorted_contrib = 1
                if self.m_dedup:
                    rows.contrib_nxt = self.m_nxt[q, k * n:].data_ptr()
                    ep.skeys, ep.n_dev = self.m_ck[q, k * n:].data_ptr(), self.m_cnt[q, k:].data_ptr()
                else:
                    rows.dedup = 0
                if self.Kp <= self.H.tail_max_kp():  # the fused tail's 512-entry chunks
                    ep.chunk_end = self.m_cend[q, k * self.m_nch:].data_ptr()
        self._build_emb_plan(plan and shard is None)
        self._m_graphs = {}
        self._m_primed = False
        self._m_warm = 0
        self._mq = 0

    def _build_emb_plan(self, want: bool) -> None:
        """Buffers of the planned step tail (emb_plan.hip / emb_plan_body.h) and the plan fields of
        every multi-step parameter block: per parity the S batches' items and split-run slots, built
        on the side chain; the split runs' window pieces, head folds and arrival counters, shared by
        the steps (they run one after another on the main stream)."""
        H = self.H
        self.m_eplan = bool(want and not self.m_dedup and self.embedding_update == "sparse"
                            and self.Kp <= H.tail_max_kp() and os.environ.get("ROCFM_EMB_PLAN", "1") != "0")
        if not self.m_eplan:
            return
        dev, n, Smax = self.device, self.n_lookup, self.mS
        i32 = dict(dtype=torch.int32, device=dev)
        nw = int(H.tail_plan_workgroups(self.m_params[0][0][1], n))
        self.m_plan_nw = nw
        self.m_plan_beta = int(os.environ.get("ROCFM_EMB_BETA", "4"))
        # runs longer than this are cut at window boundaries (split runs cost a hand-off; a 512-entry
        # run in one item costs less than that at B = 1024: profiles/r6_planned_tail.md)
        self.m_plan_lsplit = int(os.environ.get("ROCFM_EMB_LSPLIT", "512"))
        self.m_pitems = torch.zeros(2, Smax * nw * 4, **i32)
        self.m_pslots = torch.zeros(2, Smax * nw * 4, **i32)
        self.m_pruns = torch.zeros(Smax * (n + 1), **i32)
        # per item its run heads' keys (the tail prefetches their table rows at entry); ROCFM_EMB_HSLAB=0: off
        self.m_hslab_on = os.environ.get("ROCFM_EMB_HSLAB", "1") != "0"
        slab = int(H.plan_bounds()[2])
        self.m_phslab = torch.zeros(2, Smax * nw * slab if self.m_hslab_on else 1, **i32)
        self.m_pwin = torch.zeros((n // 64 + 2) * self.Kp, dtype=torch.float32, device=dev)
        self.m_phead = torch.zeros(nw * self.Kp, dtype=torch.float32, device=dev)
        self.m_pctr = torch.zeros(nw + 4, **i32)  # [nw]: sticky "item outside the plan's bounds" flag
        for q in range(2):
            for k in range(Smax):
                ep = self.m_params[q][k][3]
                if ep.mode != 0:
                    continue
                ep.plan_items = self.m_pitems[q, k * nw * 4:].data_ptr()
                ep.plan_slots = self.m_pslots[q, k * nw * 4:].data_ptr()
                ep.plan_hslab = self.m_phslab[q, k * nw * slab:].data_ptr() if self.m_hslab_on else 0
                ep.plan_nw = nw
                ep.plan_win, ep.plan_head = self.m_pwin.data_ptr(), self.m_phead.data_ptr()
                ep.plan_ctr = self.m_pctr.data_ptr()

    def _emb_plan(self, q: int, stream) -> None:
        """Side chain: the work plans of the S batches just sorted into the parity-q buffers."""
        H = self.H
        pp = H.EmbPlanParams()
        pp.skeys = self.m_sk[q].data_ptr()
        pp.n, pp.S, pp.nw = self.n_lookup, self.mS, self.m_plan_nw
        pp.beta, pp.lsplit = self.m_plan_beta, self.m_plan_lsplit
        pp.runs, pp.items, pp.slots = self.m_pruns.data_ptr(), self.m_pitems[q].data_ptr(), self.m_pslots[q].data_ptr()
        pp.hslab = self.m_phslab[q].data_ptr() if self.m_hslab_on else 0
        H.emb_plan(pp, stream.cuda_stream)

    def _fetch_multi_params(self, q: int, advance: int):
        """Preparation run beside a graph of parity q and ``advance`` steps: batches start at
        m_cur[q] + advance, written to the parity 1-q slots."""
        f = self.H.FetchMultiParams()
        f.ids_pool, f.vals_pool, f.labels_pool = (self.pool_ids.data_ptr(), self.pool_vals.data_ptr(),
                                                  self.pool_labels.data_ptr())
        f.pool_batches = self.pool_ids.shape[0]
        f.B, f.F, f.Bp, f.S, f.advance = self.B, self.F, self.Bp, self.mS, advance
        f.cur_src, f.cur_dst = self.m_cur[q:].data_ptr(), self.m_cur[1 - q:].data_ptr()
        f.step_src, f.step_dst = self.m_step[q:].data_ptr(), self.m_step[1 - q:].data_ptr()
        f.ids, f.vals, f.labels = (self.m_ids[1 - q].data_ptr(), self.m_vals[1 - q].data_ptr(),
                                   self.m_labels[1 - q].data_ptr())
        f.keys, f.id_bits = self.m_keys.data_ptr(), self.m_idbits
        if self.m_plain:
            f.plain_keys = 1
        elif not self.m_composite:
            f.keys, f.keys64 = 0, self.m_keys64[0].data_ptr()
        if getattr(self, "_m_shard", None) is not None:
            f.shard_W, f.shard_Vs = self._m_shard[:2]
            if len(self._m_shard) > 2:  # replicated (hot) ids: the virtual owner W
                f.shard_hot, f.shard_nhot = self._m_shard[2].data_ptr(), self._m_shard[2].numel()
        f.steps, f.lrt = self.m_steps[1 - q].data_ptr(), self.m_lrt[1 - q].data_ptr()
        f.lr, f.beta1, f.beta2 = self.hp.lr * self.lr_scale, self.hp.beta1, self.hp.beta2
        f.opt_type = OPT_ID[self.hp.name]
        f.halt = self.halt_word.data_ptr()
        self._guard(f)
        return f

    def _prepare_multi(self, q: int, advance: int, stream) -> None:
        H = self.H
        H.fetch_multi(self._fetch_multi_params(q, advance), stream.cuda_stream)
        if self.m_composite or self.m_plain:  # all S batches in one (segmented) sort
            iota_sort(H, self.m_temp, self.m_keys.data_ptr(), self.m_sk[1 - q].data_ptr(), self.m_sv[1 - q].data_ptr(),
                      self.n_lookup, self.m_idbits, stream.cuda_stream, nseg=self.mS,
                      seg_bits=(self.m_bits - self.m_idbits) if self.m_composite else 0)
        else:  # rocPRIM A/B: one sort of 64-bit composite keys
            H.sort_pairs64_iota(self.m_temp.data_ptr(), self.m_temp.numel(), self.m_keys64[0].data_ptr(),
                                self.m_keys64[1].data_ptr(), self.m_sv[1 - q].data_ptr(), self.mS * self.n_lookup,
                                self.m_bits, stream.cuda_stream)
        a = H.SortAuxParams()
        a.skeys, a.svals = self.m_sk[1 - q].data_ptr(), self.m_sv[1 - q].data_ptr()
        a.n, a.S, a.chunk = self.n_lookup, self.mS, self.m_chunk
        a.pos, a.chunk_end = self.m_pos[1 - q].data_ptr(), self.m_cend[1 - q].data_ptr()
        if self.m_chd is not None:
            a.chunk_heads = self.m_chd[1 - q].data_ptr()
        if self.m_keys64 is not None:  # sorted 64-bit keys → plain per-batch ids in m_sk
            a.skeys64, a.skeys_out, a.id_bits = self.m_keys64[1].data_ptr(), self.m_sk[1 - q].data_ptr(), self.m_idbits
        if self.m_dedup:  # positions / run ends / run heads come from the dedup over the compacted list
            a.chunk_end = a.chunk_heads = 0
        if not (self.m_dedup and self.m_keys64 is None):  # (64-bit keys: sort_aux writes the plain ids)
            H.sort_aux(a, stream.cuda_stream)
        if self.m_dedup:
            d = H.DedupParams()
            d.skeys, d.svals, d.n, d.S, d.F, d.rt = (self.m_sk[1 - q].data_ptr(), self.m_sv[1 - q].data_ptr(),
                                                     self.n_lookup, self.mS, self.F, self._rt)
            d.val_base_step = self.n_lookup
            d.pos, d.nxt, d.ckeys = (self.m_pos[1 - q].data_ptr(), self.m_nxt[1 - q].data_ptr(),
                                     self.m_ck[1 - q].data_ptr())
            d.count, d.bcount = self.m_cnt[1 - q].data_ptr(), self.m_bcount.data_ptr()
            d.chunk, d.chunk_end = self.m_chunk, self.m_cend[1 - q].data_ptr()
            if self.m_chd is not None:
                d.chunk_heads = self.m_chd[1 - q].data_ptr()
            H.dedup(d, stream.cuda_stream)
        if getattr(self, "m_eplan", False):
            self._emb_plan(1 - q, stream)
        if getattr(self, "_m_post", None) is not None:  # e.g. row-shard routing of the sorted batches
            self._m_post(1 - q, stream)

    def _prime_multi(self) -> None:
        self._join_side_chain()
        base = 0 if self._ring else getattr(self, "_start_batch", 0)
        self.m_cur[1] = base + self._i
        self.m_step[1] = self._i
        self._prepare_multi(1, 0, torch.cuda.current_stream(self.device))  # → parity-0 buffers
        self._pl_op("main", f"prime steps {self._i}+", self._pl_ring(self._i, self.mS, False)
                    + [("m_batches", 0, 1, True)])
        self._m_side_ev = None  # the prime ran on the main stream
        self._mq = 0
        self._m_primed = True

    def _multi_body(self, q: int, S: int) -> None:
        """The main chain of one S-step graph: rows → tail per step, strictly serial."""
        H, s = self.H, torch.cuda.current_stream(self.device).cuda_stream
        for k in range(S):
            rows, wp, _, ep, ed = self.m_params[q][k]
            H.deepfm_rows(rows, s)
            self._tail(wp, ep, ed, s)

    def _launch_multi(self, graphs: dict, key: tuple, S: int, body, capture_error_mode: str = "global",
                      capture_only: bool = False) -> None:
        """Launch one S-step multi-step graph of parity q = ``self._mq`` as TWO graphs on two streams:

        * the side graph (fetch + sort of the NEXT graph's S batches into the parity 1-q buffers)
          on the sort stream, after the previous main graph (the last reader of those buffers);
        * the main graph ``body(q, S)`` on the current stream, after the previous side graph (the
          producer of this graph's parity-q buffers).

        Side graph N therefore runs concurrently with main graph N on its own hardware queue.  (A
        single graph with the side chain as a forked branch was measured to run the branch AFTER
        the main chain on ROCm 7 — ≈200 µs of sort per 16 steps exposed at every graph boundary.)
        The first launch is eager (code objects load outside capture).  ``capture_only``: capture
        the pair if missing and return without launching (used to keep captures out of timed
        regions)."""
        q = self._mq
        main = torch.cuda.current_stream(self.device)
        side = self.sort_stream
        eager = self._m_warm < 1
        gs = gm = None
        if not eager:
            gs, gm = graphs.get(key + (q, S, "side")), graphs.get(key + (q, S, "main"))
            if gm is None:
                torch.cuda.synchronize(self.device)
                gs, gm = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                rec = self._hazard
                if rec is not None:
                    rec.begin("side")
                with torch.cuda.graph(gs, capture_error_mode=capture_error_mode):
                    self._prepare_multi(q, S, torch.cuda.current_stream(self.device))
                if rec is not None:
                    rec.begin("main")
                with torch.cuda.graph(gm, capture_error_mode=capture_error_mode):
                    body(q, S)
                if rec is not None:
                    rec.end()
                    rec.check(f"{key + (q, S)}")  # before the pair ever runs
                graphs[key + (q, S, "side")], graphs[key + (q, S, "main")] = gs, gm
        if capture_only:
            return
        # (ROCFM_HAZARD stream plan: the side graph reads the ring slots of the next graph's steps
        # and writes the parity 1-q batch buffers; the main graph reads parity q)
        side_rng = ((self._pl_ring(self._i + S, self.mS, False) if getattr(self, "_ring_mode_stream", False) else [])
                    + [("m_batches", 1 - q, 2 - q, True)])
        main_rng = [("m_batches", q, q + 1, False)]
        if eager:
            rec = self._hazard
            if rec is not None:
                rec.begin("side")
            side.wait_stream(main)
            if getattr(self, "_plan", None) is not None:
                self._plan.wait_stream("side", "main")
            with torch.cuda.stream(side):
                self._prepare_multi(q, S, side)
            self._pl_op("side", f"side graph @{self._i} (eager)", side_rng)
            ev = self._pl_mark(torch.cuda.Event(), "side")
            ev.record(side)
            if self._m_side_ev is not None:
                main.wait_event(self._m_side_ev)
                self._pl_wait("main", self._m_side_ev)
            if rec is not None:
                rec.begin("main")
            body(q, S)
            self._pl_op("main", f"main graph @{self._i} (eager)", main_rng)
            if rec is not None:
                rec.end()
                rec.check(f"eager {key + (q, S)}")
        else:
            # main graph submitted first: its kernels start while the host is still submitting the
            # side graph (a timed window otherwise begins with the side graph's whole submission);
            # the side graph still waits only for the main work queued BEFORE this main graph
            lean = self._lean_launch
            if lean & 1:
                # (ROCFM_LEAN_LAUNCH bit 0) preallocated events instead of two
                # hipEventCreate calls ahead of the replay, and no barrier packet for a side graph the
                # host already sees complete (the window's first graph after a synchronize)
                # (a ring of 8 launches: train_stream keeps the side events of the last 4 graphs)
                evs = self._lean_evs[self._m_warm % len(self._lean_evs)]
                before = self._pl_mark(evs[0], "main")
            else:
                before = self._pl_mark(torch.cuda.Event(), "main")
            before.record(main)
            if self._m_side_ev is not None:
                if not (lean & 1) or not self._m_side_ev.query():
                    main.wait_event(self._m_side_ev)
                self._pl_wait("main", self._m_side_ev)
            st = getattr(self, "stall_timing", None)  # diagnostics (bench): GPU-side gaps of the main stream
            if st is not None:
                t_start, t_end, t_side = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                t_start.record(main)  # completes when graph N may start: main work before it + side N-1
            gm.replay()
            if st is not None:
                t_end.record(main)
            self._pl_op("main", f"main graph @{self._i}", main_rng)
            if self._side_after_main:  # diagnostic: the side graph after the main graph (no overlap)
                after = torch.cuda.Event()
                after.record(main)
                side.wait_event(after)
            else:
                side.wait_event(before)
            self._pl_wait("side", before)
            with torch.cuda.stream(side):
                gs.replay()
            self._pl_op("side", f"side graph @{self._i}", side_rng)
            if st is not None:
                t_side.record(side)
                st.append((t_start, t_end, t_side))
            ev = self._pl_mark(evs[1] if lean & 1 else torch.cuda.Event(), "side")
            ev.record(side)
        self._m_side_ev = ev
        self._m_warm += 1
        self._mq ^= 1
        self._i += S

    def _precapture_multi(self, graphs: dict, key: tuple, n, body, capture_error_mode: str = "global") -> None:
        """Capture every (parity, S) graph pair that ``n`` more steps will launch, so that no
        capture lands inside a timed region (e.g. the S < Smax remainder graph).  ``n`` may be a
        list of consecutive ``train_steps`` call lengths (each split into graphs on its own)."""
        if self._m_warm < 1:
            return
        q0 = self._mq
        try:
            for m in ([n] if isinstance(n, int) else n):
                while m > 0:
                    S = min(m, self.mS)
                    self._launch_multi(graphs, key, S, body, capture_error_mode, capture_only=True)
                    self._mq ^= 1
                    m -= S
        finally:
            self._mq = q0

    # ---- ROCFM_HAZARD: the streamed loop's three-stream plan (utils/hazard.py StreamPlan) --------
    def _pl_tok(self, ev):
        return getattr(ev, "_hz_tok", 0)

    def _pl_mark(self, ev, stream: str):
        """Note that ``ev`` was just recorded on ``stream`` (plan token on the event)."""
        pl = getattr(self, "_plan", None)
        if pl is not None and ev is not None:
            ev._hz_tok = pl.record(stream)
        return ev

    def _pl_wait(self, stream: str, ev) -> None:
        pl = getattr(self, "_plan", None)
        if pl is not None and ev is not None:
            pl.wait(stream, self._pl_tok(ev))

    def _pl_ring(self, first_step: int, count: int, write: bool, slot0: Optional[int] = None):
        """Ring-slot ranges of ``count`` batches from global step ``first_step`` (or from slot
        ``slot0``), split at the ring's end."""
        R = int(self.pool_ids.shape[0])
        s0 = (getattr(self, "_start_batch", 0) + first_step) % R if slot0 is None else slot0 % R
        out, left = [], count
        while left > 0:
            m = min(left, R - s0)
            out.append(("ring", s0, s0 + m, write))
            left -= m
            s0 = 0
        return out

    def _pl_op(self, stream: str, label: str, ranges=()) -> None:
        pl = getattr(self, "_plan", None)
        if pl is not None:
            pl.op(stream, label, ranges)

    def _tail(self, wp, ep, ed, s: int) -> None:
        """MLP weight gradients + embedding update: one launch (step_tail.hip) when the rows fit."""
        H = self.H
        if self.Kp <= H.tail_max_kp():
            H.step_tail(wp, ep, s)
        else:
            H.mlp_wgrad(wp, s)
            H.emb_rows_update(ep, s)
        if ed is not None:
            H.emb_dense_update(ed, s)

    def _train_steps_multi(self, n: int, Smax: int) -> None:
        if getattr(self, "m_req", None) != Smax or getattr(self, "_m_pool", None) is not self.pool_ids:
            self._build_multi(Smax, plan=True)
            self._m_pool = self.pool_ids
        if not self._m_primed:
            self._prime_multi()
        while n > 0:
            S = min(n, self.mS)
            self._run_multi_graph(S)
            n -= S
        if self._lean_launch & 2:
            # (ROCFM_LEAN_LAUNCH bit 1) no trailing barrier packet: the side graph only writes the
            # next graph's batch buffers, which the next main graph already waits for (_m_side_ev);
            # every other reader joins first (_join_side_chain)
            self._side_join_pending = True
        else:
            torch.cuda.current_stream(self.device).wait_stream(self.sort_stream)
        self._primed = False  # the per-step path re-primes from the global step if used next

    def _join_side_chain(self) -> None:
        """Order the current stream after the multi-step side chain (lazy trailing join)."""
        if getattr(self, "_side_join_pending", False):
            torch.cuda.current_stream(self.device).wait_stream(self.sort_stream)
            self._side_join_pending = False

    def _run_multi_graph(self, S: int) -> None:
        """One multi-step graph of S steps (eager the first time: code objects load outside capture)."""
        self._launch_multi(self._m_graphs, ("m",), S, self._multi_body)

    def precapture(self, n: int, steps_per_graph: int = 16) -> None:
        """Capture the graphs ``train_steps(n, steps_per_graph)`` will replay (no launch)."""
        if self.use_graph and not self._ring and self.fuse_dense_opt and steps_per_graph > 1 \
                and getattr(self, "m_req", None) == steps_per_graph and self._m_primed:
            self._precapture_multi(self._m_graphs, ("m",), n, self._multi_body)

    def train_stream(self, *args, **kwargs) -> int:
        """``_train_stream``; under ``ROCFM_HAZARD=1`` with every torch write into the batch ring
        observed on its stream as well (``hazard.ObservedWrites``: a copy the loop does not declare
        is still checked)."""
        self._join_side_chain()
        if self._hazard is None:
            return self._train_stream(*args, **kwargs)

        def stream_name():
            return getattr(self, "_plan_names", {}).get(torch.cuda.current_stream(self.device).cuda_stream, "?")

        ring = lambda: {"ring": list(getattr(self, "_stream_ring", None) or ())}  # noqa: E731
        with hazard.ObservedWrites(lambda: getattr(self, "_plan", None), ring, stream_of=stream_name) as obs:
            try:
                return self._train_stream(*args, **kwargs)
            finally:
                self.hazard_observed = obs.seen  # torch writes into the ring seen on their streams

    def _train_stream(self, batches, steps_per_graph: int = 16, after_steps=None, hold: int = 1,
                      ring_batches: int = 0, build=None, run=None, prefix=None) -> int:
        """Train on a stream of host batches (the Estimator's loader) through multi-step graphs.

        Batches are copied host → HBM on a copy stream into a device ring of 4·S batch slots, two
        graphs ahead of the graph that consumes them (a graph's side chain reads the NEXT graph's
        batches).  A graph waits only for the copies of the batches its side chain reads, and a
        copy only for the graph that last read its slots (three graphs back), so the host, which
        stages copies and launches one graph per S steps, runs up to two graphs ahead of the GPU.
        Items are single batches ``(ids [B,F], vals [B,F], labels [B])``, groups of n ≤ S
        consecutive batches stacked ``[n,B,F]`` (``TFRecordDataset.groups``: one copy per group),
        or undecoded ``RawGroup``s (``TFRecordDataset.raw_groups``): their Example payload bytes
        are copied as they are and parsed on the copy stream by the decode kernel straight into
        the ring slots (``csrc/kernels/decode.hip``) — the host only moves bytes.  A malformed
        record sets the parser's sticky error word: every step the side chain prepares from then on
        is halted on the device (no optimizer update — the bad batch, and any batch after it, never
        trains), and RuntimeError is raised within two groups, by ``check()`` and so before any
        checkpoint (``state_dict``).
        The source may recycle an item's host memory once it has been advanced ``hold`` more
        times; the copy of every such item is waited for first.  Returns the number of steps
        trained; ``after_steps(first_step, n_steps)`` runs after each graph launch.
        ``ring_batches`` ≥ the number of batches streamed sizes the HBM ring to hold them all, so
        that afterwards ``stream_ring()[i]`` is the i-th batch of this call (the decoded-epoch HBM
        cache of the Estimator: later epochs train from it via attach_pool).
        ``build(S)`` / ``run(n)`` (the distributed wrappers, rocfm.parallel): (re)build the
        multi-step structures for the attached ring, and launch one n-step graph with the step's
        exchange inline; default: this engine's single-GPU graphs.
        ``prefix`` = device batches ``(ids [n,B,F], vals, labels)`` ALREADY trained just before this
        call (the distributed wrappers' shadow-validation steps): they take ring slots 0..n-1 so
        that the ring holds the stream's batches in order from its first one (``ring_batches``
        counts them too).
        """
        S = self._multi_S(int(steps_per_graph))[1]
        npre = 0 if prefix is None else int(prefix[0].shape[0])
        R = max(4 * S + npre, (int(ring_batches) + S - 1) // S * S)
        hold = max(1, int(hold))
        dev = self.device
        # ROCFM_HAZARD=1: every copy / side / main operation of this loop and its event waits go
        # into a happens-before plan, checked after each graph launch (utils/hazard.py StreamPlan)
        self._plan = hazard.StreamPlan() if self._hazard is not None else None
        names = {}  # stream handle → plan stream name
        if self._plan is not None:
            names = {self._copy_stream.cuda_stream: "copy", self.sort_stream.cuda_stream: "side",
                     torch.cuda.current_stream(dev).cuda_stream: "main"}
        self._plan_names = names
        ring = getattr(self, "_stream_ring", None)
        if ring is None or ring[0].shape[0] != R:
            ring = (torch.zeros(R, self.B, self.F, dtype=torch.int32, device=dev),
                    torch.zeros(R, self.B, self.F, dtype=torch.float32, device=dev),
                    torch.zeros(R, self.B, dtype=torch.float32, device=dev))
            self._stream_ring = ring
            # the zero fill runs on the CURRENT stream, behind whatever is queued there (a 1B-row
            # engine's table initialisation: seconds) — the copy stream below waits for it
            self._pl_op("main", "ring allocation (zero fill)", [("ring", 0, R, True)])
        i0 = self._i
        # pool batch index of global step i = (start + i) % R  with start ≡ −(i0 − npre) (mod R) →
        # slot i − i0 + npre: the prefix (steps i0 − npre .. i0 − 1) in slots 0 .. npre − 1
        self.attach_pool(*ring, start=(R - (i0 - npre) % R) % R)
        if npre:
            for k in range(3):
                ring[k][:npre].copy_(prefix[k])
            self._pl_op("main", "prefix", self._pl_ring(0, npre, True, slot0=0))
        self._ring_mode_stream = True
        copy = self._copy_stream
        it = iter(batches)
        # every copy-stream write (H2D copies, the device parser into the ring) is ordered after all
        # the work queued so far on the current stream: the ring's zero fill above, the engine's own
        # initialisation, the prefix copies.  Without it the zero fill of a new ring could land
        # AFTER the parser had written the first batches (seen at 1B rows, where the table's
        # initialisation keeps the current stream busy for seconds: the whole stream trained on
        # zeroed batches; tests/test_sort_gpu.py::test_wide_vocabulary_streams_through_seg_sort)
        if os.environ.get("ROCFM_HAZARD_INJECT", "") != "ring_init":  # (hazard test: leave it out)
            copy.wait_stream(torch.cuda.current_stream(dev))
            if self._plan is not None:
                self._plan.wait_stream("copy", "main")

        def mark(stream):
            e = torch.cuda.Event()
            e.record(stream)
            return self._pl_mark(e, names.get(stream.cuda_stream, "?"))

        pending = []  # (event, host batch) kept alive until its copy has completed
        carry = [None]  # the part of a group that did not fit the previous graph (same host memory)
        staged = npre  # ring slots filled so far (the prefix first)

        def stage(k):  # copy up to k more batches; returns how many were available
            nonlocal staged
            got = 0
            while got < k:
                if carry[0] is not None:
                    b, carry[0] = carry[0], None
                else:
                    while len(pending) > hold - 1:  # the item `hold` back is recycled by this next()
                        t_h = time.perf_counter()
                        pending.pop(0)[0].synchronize()
                        self.host_copy_wait_s = getattr(self, "host_copy_wait_s", 0.0) + time.perf_counter() - t_h
                    b = next(it, None)
                    if b is None:
                        break
                if isinstance(b, RawGroup):
                    if b.B != self.B:
                        raise ValueError(f"batch has {b.B} rows, engine built for {self.B}")
                    n = b.n
                    if got + n > k:  # split: the rest goes to the next graph's staging
                        m = k - got
                        carry[0] = RawGroup(b.bytes[m:], b.offs[m:], n - m, b.B)
                        b, n = RawGroup(b.bytes[:m], b.offs[:m], m, b.B), m
                    timing = getattr(self, "copy_timing", None)  # diagnostics (bench): H2D + parse time
                    if timing is not None:
                        t0 = torch.cuda.Event(enable_timing=True)
                        t0.record(copy)
                    with torch.cuda.stream(copy):
                        self._stage_raw(b, staged % R, R, staged)
                    if timing is not None:
                        t1 = torch.cuda.Event(enable_timing=True)
                        t1.record(copy)
                        timing.append((t0, t1, int(b.used_bytes()), n, self._copy_mid))
                    self._pl_op("copy", f"raw stage of batches {staged}..{staged + n - 1}",
                                self._pl_ring(0, n, True, slot0=staged % R) + [("raw_stage", 0, 1, True)])
                    pending.append((mark(copy), b))
                    staged += n
                    got += n
                    self._check_decode(block=False)
                    continue
                ids, vals, labels = b
                if ids.dim() == 2:
                    ids, vals, labels = ids.unsqueeze(0), vals.unsqueeze(0), labels.unsqueeze(0)
                n = ids.shape[0]
                if ids.shape[1] != self.B:
                    raise ValueError(f"batch has {ids.shape[1]} rows, engine built for {self.B}")
                if got + n > k:  # split: the rest goes to the next graph's staging
                    m = k - got
                    carry[0] = (ids[m:], vals[m:], labels[m:])
                    ids, vals, labels, n = ids[:m], vals[:m], labels[:m], m
                with torch.cuda.stream(copy):
                    o = 0
                    while o < n:  # contiguous ring slots (split at the ring's end)
                        slot = (staged + o) % R
                        m = min(n - o, R - slot)
                        ring[0][slot:slot + m].copy_(ids[o:o + m], non_blocking=True)
                        ring[1][slot:slot + m].copy_(vals[o:o + m], non_blocking=True)
                        ring[2][slot:slot + m].copy_(labels[o:o + m], non_blocking=True)
                        o += m
                self._pl_op("copy", f"copy of batches {staged}..{staged + n - 1}",
                            self._pl_ring(0, n, True, slot0=staged % R))
                pending.append((mark(copy), b))
                staged += n
                got += n
            return got

        main = torch.cuda.current_stream(dev)
        avail = stage(2 * S)
        if avail == 0:
            return 0
        staged_new = lambda: staged - npre  # noqa: E731 — batches of this call's stream
        cevs = [mark(copy)]  # cevs[j]: copies read by graph j's side chain (graph j+1's batches)
        main.wait_event(cevs[0])
        self._pl_wait("main", cevs[0])
        if build is not None:
            build(S)
        elif getattr(self, "m_req", None) != S or getattr(self, "_m_pool", None) is not self.pool_ids:
            self._build_multi(S, plan=True)
            self._m_pool = self.pool_ids
        self._prime_multi()  # prepares steps i0 .. i0+S-1 from the ring
        prime_ev = mark(main)
        sevs = []  # sevs[j]: end of graph j's side chain (side graph, sort stream)
        inject = self._plan is not None and os.environ.get("ROCFM_HAZARD_INJECT", "") == "ring"
        done, j = 0, 0
        while done < staged_new():
            n = min(S, staged_new() - done)
            # stage graph j+2's batches; their ring slots held graph j-2's batches, last read by
            # graph j-3's side chain (or by the prime)
            wait_ev = sevs[j - 3] if j >= 3 else prime_ev
            if inject and j >= 3:  # (hazard test only) the refill waits one side graph too early
                wait_ev = sevs[j - 4] if j >= 4 else prime_ev
            copy.wait_event(wait_ev)
            self._pl_wait("copy", wait_ev)
            more = stage(S)
            cevs.append(mark(copy))
            self.sort_stream.wait_event(cevs[j])
            self._pl_wait("side", cevs[j])
            if run is not None:
                run(n)
            else:
                self._run_multi_graph(n)
            sevs.append(self._m_side_ev)
            if self._plan is not None:
                self._plan.check(f"train_stream graph {j}")
            if after_steps is not None:
                after_steps(i0 + done, n)
            done += n
            j += 1
            if n < S and more == 0:
                break
        main.wait_stream(self.sort_stream)
        for e0, _ in pending:
            e0.synchronize()
        self._plan = None
        self._check_decode(block=True)
        self._primed = False
        return done

    # ---- device-side Example parsing (raw groups) ----------------------------------------------
    def _stage_raw(self, g, slot0: int, R: int, batch0: int) -> None:
        """On the current (copy) stream: H2D-copy a RawGroup's payload bytes + offsets and parse
        them into ring slots slot0 .. slot0+n-1 (mod R)."""
        H, n, cap = self.H, g.n, int(g.bytes.shape[1])
        st = getattr(self, "_raw_dev", None)
        if st is None or st[0].numel() < n * cap + 64 or st[1].shape[0] < n or st[1].shape[1] != self.B + 1:
            d_bytes = torch.empty(n * cap + 64, dtype=torch.uint8, device=self.device)  # +64: window reads
            d_offs = torch.empty(n, self.B + 1, dtype=torch.int32, device=self.device)
            d_err = self.halt_word  # (the error word the step preparation halts on)
            h_err = torch.zeros(4, dtype=torch.int32, pin_memory=True)
            st = self._raw_dev = [d_bytes, d_offs, d_err, h_err, None]
        d_bytes, d_offs, d_err, h_err, _ = st
        used = g.used_bytes()
        d_bytes[:used].copy_(g.bytes.reshape(-1)[:used], non_blocking=True)
        d_offs[:n].copy_(g.offs, non_blocking=True)
        if getattr(self, "copy_timing", None) is not None:  # diagnostics: H2D | parse split
            self._copy_mid = torch.cuda.Event(enable_timing=True)
            self._copy_mid.record(torch.cuda.current_stream(self.device))
        p = H.DecodeParams()
        p.bytes, p.offs, p.cap, p.nb, p.B, p.F = d_bytes.data_ptr(), d_offs.data_ptr(), cap, n, self.B, self.F
        ring = self._stream_ring
        p.ids, p.vals, p.labels = ring[0].data_ptr(), ring[1].data_ptr(), ring[2].data_ptr()
        p.slot0, p.R, p.max_id, p.batch0, p.err = int(slot0), int(R), int(self.id_limit), int(batch0), d_err.data_ptr()
        keys = getattr(self, "decode_keys", ("label", "ids", "values"))
        p.set_keys(*keys)
        H.decode_examples(p, torch.cuda.current_stream(self.device).cuda_stream)
        h_err.copy_(d_err, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        st[4] = ev

    def _check_decode(self, block: bool) -> None:
        """Raise on the decode kernel's sticky error word (tfrecord.h ParseStatus codes)."""
        st = getattr(self, "_raw_dev", None)
        if st is None or st[4] is None:
            return
        if block:
            st[4].synchronize()
        elif not st[4].query():
            return
        code, batch, rec = (int(x) for x in st[3][:3])
        if code:
            names = {1: "malformed Example protobuf", 2: "missing feature",
                     3: "wrong feature length (FixedLenFeature expects field_size values)",
                     4: "id out of range [0, feature_size)", 5: "bad record offsets"}
            st[2].zero_()
            st[3].zero_()
            raise RuntimeError(f"decode error in batch {batch} record {rec} (device parse): "
                               f"{names.get(code, code)}")

    def stream_ring(self):
        """The HBM ring of the last train_stream call (ids, vals, labels)."""
        return self._stream_ring

    def train_steps(self, n: int, steps_per_graph: int = 8) -> None:
        """``n`` optimisation steps from the attached pool; full step-pairs are replayed from one
        multi-step HIP graph (``steps_per_graph`` steps per launch) to amortise launch overhead."""
        if self.use_graph and not self._ring and self.fuse_dense_opt and steps_per_graph > 1:
            hp = self._main_stream()
            if hp is None:
                self._train_steps_multi(n, steps_per_graph)
                return
            cur = torch.cuda.current_stream(self.device)
            hp.wait_stream(cur)
            with torch.cuda.stream(hp):
                self._train_steps_multi(n, steps_per_graph)
            cur.wait_stream(hp)
            return
        S = max(2, steps_per_graph // 2 * 2)
        while n > 0:
            if (self.use_graph and self._primed and self._warm >= 2 and n >= S and self._i % 2 == 0
                    and not self._ring):
                g = getattr(self, "_multi_graph", None)
                if g is None or self._pipe_S != S:
                    g = torch.cuda.CUDAGraph()
                    torch.cuda.synchronize(self.device)
                    with torch.cuda.graph(g):
                        self._enqueue_pipelined(S)
                    self._multi_graph, self._pipe_S = g, S
                g.replay()
                self._i += S
                n -= S
            else:
                self.train_step()
                n -= 1

    def _main_stream(self):
        """ROCFM_MAIN_PRIORITY=1: the multi-step main graphs run on a high-priority stream (its
        hardware queue's dispatches are served before the side chain's), or None."""
        if os.environ.get("ROCFM_MAIN_PRIORITY", "0") != "1":
            return None
        st = getattr(self, "_hp_stream", None)
        if st is None:
            lo, hi = torch.cuda.Stream.priority_range()
            st = self._hp_stream = torch.cuda.Stream(device=self.device, priority=min(lo, hi))
        return st

    def train_step(self) -> None:
        """One optimisation step on the current batch (asynchronous)."""
        self._join_side_chain()
        if not self.fuse_dense_opt:
            raise RuntimeError("train_step() is the single-GPU step; distributed steps live in rocfm.parallel")
        self._m_primed = False
        if not self._primed:
            self.prime()
        p = self._i % 2
        if not self.use_graph or self._warm < 2:
            self._warm += 1
            self._enqueue_step(p)
        else:
            if self._graphs[p] is None:
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize(self.device)
                with torch.cuda.graph(g):
                    self._enqueue_step(p)
                self._graphs[p] = g
            self._graphs[p].replay()
        self._i += 1

    # ---- inference -----------------------------------------------------------------------------
    @torch.no_grad()
    def predict_batch(self, ids: torch.Tensor, vals: torch.Tensor, labels: Optional[torch.Tensor] = None):
        """Probabilities (and per-row losses) for any number of rows; no dropout, no update."""
        self._join_side_chain()
        n = ids.shape[0]
        if n > self.B:
            out = [self.predict_batch(ids[i:i + self.B], vals[i:i + self.B],
                                      None if labels is None else labels[i:i + self.B]) for i in range(0, n, self.B)]
            return torch.cat([o[0] for o in out]), torch.cat([o[1] for o in out])
        self.pred_ids[:n].copy_(ids)
        self.pred_vals[:n].copy_(vals)
        if labels is not None:
            self.pred_labels[:n].copy_(labels)
        else:
            self.pred_labels.zero_()
        rp = self.pred_params
        rp.B = n
        self.H.deepfm_rows(rp, self.stream_ptr)
        return self.pred_prob[:n].clone(), self.pred_loss[:n].clone()

    # ---- state ----------------------------------------------------------------------------------
    def l2_value(self) -> float:
        """λ·(l2_loss(fm_w) + l2_loss(fm_v)) — evaluated on demand (the full-table term of PS:277-278)."""
        nb = 1024
        part = torch.zeros(nb, dtype=torch.float32, device=self.device)
        self.H.emb_sumsq(self.emb.data_ptr(), self.V * self.Kp // 4, self.Kp, self.K1, part.data_ptr(), nb,
                         self.stream_ptr, self.tbl_bf16)
        return float(self.spec.l2_reg * 0.5 * part.double().sum().item())

    def batch_loss(self, include_l2: bool = True) -> float:
        """Loss of the most recent training batch (mean data loss [+ full-table L2 terms])."""
        loss = float(self.loss_rows[: self.B].double().mean().item())
        return loss + (self.l2_value() if include_l2 else 0.0)

    def loss_async(self, include_l2: bool = True):
        """``batch_loss()`` without draining the stream: the reduction and a copy into pinned host
        memory are enqueued on the training stream.  Returns ``(event, host)``; ``host[0]`` holds
        the loss once the event has completed (``event.query()`` / ``synchronize()``)."""
        v = self.loss_rows[: self.B].double().mean()
        if include_l2:
            nb = 1024
            part = torch.zeros(nb, dtype=torch.float32, device=self.device)
            self.H.emb_sumsq(self.emb.data_ptr(), self.V * self.Kp // 4, self.Kp, self.K1, part.data_ptr(), nb,
                             self.stream_ptr, self.tbl_bf16)
            v = v + self.spec.l2_reg * 0.5 * part.double().sum()
        host = torch.empty(1, dtype=torch.float64, pin_memory=True)
        host.copy_(v.view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ev, host

    def last_probs(self) -> torch.Tensor:
        return self.prob[: self.B]

    def global_step(self) -> int:
        return self._i

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        """TF-named variables + optimizer slots + global_step (CPU tensors)."""
        self._join_side_chain()
        torch.cuda.synchronize(self.device)
        self.check()
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        tf = self._tf_views(self.emb, self.dense)
        tf.update(self._bn_views())
        for k, v in tf.items():
            sd[k] = v.detach().float().cpu().clone()  # (a bf16 table is saved as f32: TF layout)
        names = slot_names(self.hp.name)
        for si, sn in enumerate(names):
            sv = self._tf_views(self.emb_slots[si], self.dense_slots[si])
            for k, v in sv.items():
                sd[f"{k}/{sn}"] = v.detach().cpu().clone()
        step = self.global_step()
        sd["global_step"] = torch.tensor(step, dtype=torch.int64)
        if self.hp.name == "Adam":
            sd["beta1_power"] = torch.tensor(self.hp.beta1 ** (step + 1), dtype=torch.float32)
            sd["beta2_power"] = torch.tensor(self.hp.beta2 ** (step + 1), dtype=torch.float32)
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        self._join_side_chain()
        with torch.no_grad():
            self._load_views(sd, "", self.emb, self.dense, strict)
            for k, view in self._bn_views().items():
                if k in sd:
                    view.copy_(sd[k].to(view.device).reshape(view.shape))
                elif strict:
                    raise KeyError(f"checkpoint is missing {k}")
            for si, sn in enumerate(slot_names(self.hp.name)):
                self._load_views(sd, "/" + sn, self.emb_slots[si], self.dense_slots[si], strict)
            if "global_step" in sd:
                self._i = int(sd["global_step"])
        self.refresh_bf16()
        self._graphs = [None, None]
        self._primed = False
        self._m_primed = False
        self._pushed = self._i

    def _tf_views(self, emb_like: torch.Tensor, dense_like: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        v: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        dv = self.layout.views(dense_like)
        v["fm_bias"] = dv.pop("fm_bias")
        v["fm_w"] = emb_like[:, self.K]
        v["fm_v"] = emb_like[:, : self.K]
        v.update(dv)
        return v

    def _load_views(self, sd, suffix, emb_like, dense_like, strict):
        for k, view in self._tf_views(emb_like, dense_like).items():
            key = k + suffix
            if key not in sd:
                if strict:
                    raise KeyError(f"checkpoint is missing {key}")
                continue
            view.copy_(sd[key].to(view.device).reshape(view.shape))

    def _bn_views(self) -> "OrderedDict[str, torch.Tensor]":
        """batch_norm moving moments (non-trainable: no optimizer slots), TF names."""
        v: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        if self.bn:
            for l in range(self.layout.nl):
                n = self.layout.real[l + 1]
                v[f"Deep-part/bn_{l}/moving_mean"] = self.bn_stats[l, 0, :n]
                v[f"Deep-part/bn_{l}/moving_variance"] = self.bn_stats[l, 1, :n]
        return v

    def check(self) -> None:
        """Raise if a batch-norm grid barrier of the row kernel timed out (the step's moments are
        then invalid; a sticky device flag, read with one small copy), or if the device Example
        parser flagged a malformed record (its steps were halted, never trained)."""
        self._join_side_chain()
        self._check_decode(block=True)
        if self.bn and int(self.bn_error[0].item()) != 0:
            raise RuntimeError("deepfm_rows: a batch_norm grid barrier timed out (not every workgroup was resident)")
        if self.row_split > 1 and int(self.xerr[0].item()) != 0:
            self.xctr.zero_()  # (the arrival parity is lost with the timed-out launch)
            self.xerr.zero_()
            raise RuntimeError("deepfm_rows: a row-tile split exchange timed out (its steps' layer-1 inputs are invalid)")
        if getattr(self, "m_eplan", False):
            err = int(self.m_pctr[self.m_plan_nw].item())
            if err:
                raise RuntimeError("step_tail (planned embedding role): "
                                   + ("an item exceeded the plan's bounds " if err & 1 else "")
                                   + ("a split run's head item timed out waiting for its lead items " if err & 2 else "")
                                   + ("an item's head-key slab disagreed with its keys (rows reloaded; a plan "
                                      "kernel bug) " if err & 4 else "")
                                   + "(those rows were not updated)")
        if self.id_guard and int(self.bad_ids.item()) != 0:
            raise ValueError(f"ROCFM_CHECK_IDS: a batch held feature ids outside [0, {self.id_limit}) "
                             "(they were trained as row 0)")

    def parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        tf = self._tf_views(self.emb, self.dense)
        tf.update(self._bn_views())
        return OrderedDict((k, v.detach().float().cpu().clone()) for k, v in tf.items())
