"""Eager PyTorch DeepFM trainer (``engine=torch``).

Runs anywhere PyTorch runs (CPU for tests and BASELINE config 1; on the GPU it is the
PyTorch-eager baseline the fused HIP engine is measured against).  It supports everything the
reference model supports, including ``batch_norm`` (PS:316-338) and every optimizer, and both
embedding semantics:

* ``exact``  — the reference's: loss includes λ·l2_loss over the FULL tables, autograd yields a
  dense [V,K] gradient, the optimizer updates every row.
* ``sparse`` — gather the batch's unique rows, autograd over those rows only, lazy L2 on them,
  row-sparse optimizer (rocfm.optim.apply_rows).

Distributed data parallel hooks (``allreduce_dense``, ``exchange_rows``) are supplied by
rocfm.parallel.dp so the same engine runs under gloo (CPU tests) or RCCL.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Callable, Dict, Optional

import torch

from ..optim import OptHParams, apply_dense, apply_rows, init_slots, slot_names
from .deepfm import ModelSpec, data_loss, forward, full_loss, init_params, is_trainable, l2_terms


class TorchDeepFM:
    def __init__(self, spec: ModelSpec, hp: OptHParams, device="cpu", embedding_update: str = "sparse",
                 params: Optional[Dict[str, torch.Tensor]] = None, seed: int = 1234, dropout_seed: Optional[int] = None):
        self.spec, self.hp = spec, hp
        self.device = torch.device(device)
        self.embedding_update = embedding_update
        P = params if params is not None else init_params(spec, seed)
        self.P: "OrderedDict[str, torch.Tensor]" = OrderedDict(
            (k, v.detach().clone().to(self.device).float()) for k, v in P.items())
        self.trainable = [k for k in self.P if is_trainable(k)]
        self.slots = {k: init_slots(hp, self.P[k]) for k in self.trainable}
        self.t = 0
        self.gen = torch.Generator(device=self.device).manual_seed(seed if dropout_seed is None else dropout_seed)
        self.lr_scale = 1.0
        # distributed hooks (identity on a single process)
        self.allreduce_dense: Optional[Callable[[Dict[str, torch.Tensor]], None]] = None
        self.exchange_rows: Optional[Callable] = None

    # ------------------------------------------------------------------------------------------
    def set_lr_scale(self, s: float) -> None:
        self.lr_scale = s

    def _hp(self) -> OptHParams:
        if self.lr_scale == 1.0:
            return self.hp
        hp = OptHParams(**self.hp.__dict__)
        hp.lr = self.hp.lr * self.lr_scale
        return hp

    def train_step(self, ids: torch.Tensor, vals: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        labels = labels.to(self.device).float()
        step = self.t + 1
        hp = self._hp()
        if self.embedding_update == "exact":
            params = {k: (v.requires_grad_(True) if k in self.trainable else v) for k, v in self.P.items()}
            for v in params.values():
                v.grad = None
            y = forward(params, ids, vals, self.spec, train=True, gen=self.gen)
            loss = full_loss(params, y, labels, self.spec)
            loss.backward()
            grads = {k: params[k].grad for k in self.trainable}
            for k in self.trainable:
                params[k].requires_grad_(False)
            if self.allreduce_dense is not None:
                self.allreduce_dense(grads)
            for k in self.trainable:
                apply_dense(hp, self.P[k], grads[k], self.slots[k], step)
            self.t += 1
            self._last_loss_t, self._last_has_l2 = loss.detach(), True
            return loss.detach()
        # sparse: autograd over the batch's unique rows only
        uniq, inv = torch.unique(ids.reshape(-1), return_inverse=True)
        inv = inv.reshape(ids.shape)
        rw = self.P["fm_w"][uniq].clone().requires_grad_(True)
        rv = self.P["fm_v"][uniq].clone().requires_grad_(True)
        dense_names = [k for k in self.trainable if k not in ("fm_w", "fm_v")]
        params = dict(self.P)
        for k in dense_names:
            params[k] = self.P[k].requires_grad_(True)
            params[k].grad = None
        y = forward(params, ids, vals, self.spec, train=True, gen=self.gen, rows_w=rw[inv], rows_v=rv[inv])
        loss = data_loss(y, labels, self.spec.loss_type)
        loss.backward()
        gw, gv = rw.grad, rv.grad
        dgrads = {k: params[k].grad for k in dense_names}
        for k in dense_names:
            self.P[k].requires_grad_(False)
        if self.exchange_rows is not None:  # (union of ids, rank-averaged data gradients)
            uniq, gw, gv = self.exchange_rows(uniq, gw, gv)
        gw = gw + self.spec.l2_reg * self.P["fm_w"][uniq]  # lazy L2 on touched rows, once
        gv = gv + self.spec.l2_reg * self.P["fm_v"][uniq]
        if self.allreduce_dense is not None:
            self.allreduce_dense(dgrads)
        apply_rows(hp, self.P["fm_w"], uniq, gw, self.slots["fm_w"], step)
        apply_rows(hp, self.P["fm_v"], uniq, gv, self.slots["fm_v"], step)
        for k in dense_names:
            apply_dense(hp, self.P[k], dgrads[k], self.slots[k], step)
        self.t += 1
        self._last_loss_t, self._last_has_l2 = loss.detach(), False
        return loss.detach()

    def batch_loss(self, include_l2: bool = True) -> float:
        """Loss of the most recent training batch (data loss + full-table L2 terms)."""
        if not hasattr(self, "_last_loss_t"):
            return float("nan")
        v = float(self._last_loss_t)
        if include_l2 and not self._last_has_l2:
            v += self.l2_value()
        if not include_l2 and self._last_has_l2:
            v -= self.l2_value()
        return v

    @torch.no_grad()
    def predict_batch(self, ids, vals, labels=None):
        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        y = forward(self.P, ids, vals, self.spec, train=False)
        p = torch.sigmoid(y)
        if labels is None:
            return p, torch.zeros_like(p)
        labels = labels.to(self.device).float()
        if self.spec.loss_type == "log_loss":
            lr = torch.clamp(y, min=0) - y * labels + torch.log1p(torch.exp(-y.abs()))
        else:
            lr = (p - labels) ** 2
        return p, lr

    def l2_value(self) -> float:
        return float(l2_terms(self.P, self.spec.l2_reg))

    def global_step(self) -> int:
        return self.t

    # ---- state ---------------------------------------------------------------------------------
    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        for k, v in self.P.items():
            sd[k] = v.detach().cpu().clone()
        for si, sn in enumerate(slot_names(self.hp.name)):
            for k in self.trainable:
                sd[f"{k}/{sn}"] = self.slots[k][si].detach().cpu().clone()
        sd["global_step"] = torch.tensor(self.t, dtype=torch.int64)
        if self.hp.name == "Adam":
            sd["beta1_power"] = torch.tensor(self.hp.beta1 ** (self.t + 1), dtype=torch.float32)
            sd["beta2_power"] = torch.tensor(self.hp.beta2 ** (self.t + 1), dtype=torch.float32)
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        for k in self.P:
            if k in sd:
                self.P[k].copy_(sd[k].reshape(self.P[k].shape))
            elif strict:
                raise KeyError(f"checkpoint is missing {k}")
        for si, sn in enumerate(slot_names(self.hp.name)):
            for k in self.trainable:
                key = f"{k}/{sn}"
                if key in sd:
                    self.slots[k][si].copy_(sd[key].reshape(self.slots[k][si].shape))
                elif strict:
                    raise KeyError(f"checkpoint is missing {key}")
        if "global_step" in sd:
            self.t = int(sd["global_step"])

    def parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((k, v.detach().cpu().clone()) for k, v in self.P.items())
