"""DeepFM model definition: parameters (TF variable names), initialisers and the eager forward.

This is the math of the reference ``model_fn`` (PS:172-313 ≡ HVD:164-303) in PyTorch:

* variables  ``fm_bias[1]`` (0), ``fm_w[V]``, ``fm_v[V,K]`` (glorot_normal)      PS:188-198
* first order ``y_w = Σ_f w[id]·x``                                              PS:207-209
* second order ``e = V[id]·x``; ``y_v = ½Σ_k((Σ_f e)² − Σ_f e²)``                 PS:211-217
* deep part  ``h0 = reshape(e,[B,F·K])`` → ``fully_connected``×L (ReLU, xavier) → optional BN
  (after ReLU) → dropout(keep_prob) in TRAIN → linear ``deep_out``              PS:219-255
* output ``y = b + y_w + y_v + y_d``, ``prob = σ(y)``                           PS:257-260
* loss  ``mean(sigmoid_CE) + λ·l2_loss(fm_w) + λ·l2_loss(fm_v)``                 PS:275-279
  (the MLP ``weights_regularizer`` at PS:238/251 is never added to the loss — Q2 — and is
  therefore not applied here either).

It serves three purposes: the ``engine=torch`` trainer (CPU, and the PyTorch-eager GPU
baseline), the numerics oracle the HIP kernels are tested against, and the checkpoint layout
(TF names).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as Fn

TRUNC_NORMAL_STD = 0.87962566103423978  # std of a unit normal truncated at ±2σ (TF glorot_normal)


@dataclass
class ModelSpec:
    feature_size: int
    field_size: int
    embedding_size: int
    layers: List[int] = field(default_factory=lambda: [128, 64, 32])
    keep_probs: List[float] = field(default_factory=lambda: [0.5, 0.5, 0.5])
    batch_norm: bool = False
    batch_norm_decay: float = 0.9
    l2_reg: float = 1e-4
    loss_type: str = "log_loss"

    @classmethod
    def from_config(cls, cfg) -> "ModelSpec":
        return cls(feature_size=cfg.feature_size, field_size=cfg.field_size, embedding_size=cfg.embedding_size,
                   layers=cfg.layers, keep_probs=cfg.keep_probs, batch_norm=cfg.batch_norm,
                   batch_norm_decay=cfg.batch_norm_decay, l2_reg=cfg.l2_reg, loss_type=cfg.loss_type)

    @property
    def deep_in(self) -> int:
        return self.field_size * self.embedding_size


def param_shapes(spec: ModelSpec) -> "OrderedDict[str, Tuple[int, ...]]":
    """Trainable + BN variables with their TF names."""
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    s["fm_bias"] = (1,)
    s["fm_w"] = (spec.feature_size,)
    s["fm_v"] = (spec.feature_size, spec.embedding_size)
    d = spec.deep_in
    for i, h in enumerate(spec.layers):
        s[f"Deep-part/mlp{i}/weights"] = (d, h)
        s[f"Deep-part/mlp{i}/biases"] = (h,)
        if spec.batch_norm:
            s[f"Deep-part/bn_{i}/beta"] = (h,)
            s[f"Deep-part/bn_{i}/gamma"] = (h,)
            s[f"Deep-part/bn_{i}/moving_mean"] = (h,)
            s[f"Deep-part/bn_{i}/moving_variance"] = (h,)
        d = h
    s["Deep-part/deep_out/weights"] = (d, 1)
    s["Deep-part/deep_out/biases"] = (1,)
    return s


def is_trainable(name: str) -> bool:
    return not (name.endswith("moving_mean") or name.endswith("moving_variance"))


def glorot_normal_(t: torch.Tensor, fan_in: int, fan_out: int, gen: torch.Generator) -> torch.Tensor:
    """TF 1.x glorot_normal_initializer: truncated normal (±2σ), σ = √(2/(fan_in+fan_out))/0.8796."""
    std = math.sqrt(2.0 / (fan_in + fan_out)) / TRUNC_NORMAL_STD
    with torch.no_grad():
        x = torch.randn(t.shape, generator=gen, dtype=torch.float32)
        bad = x.abs() > 2.0
        while bad.any():  # resample outside ±2σ (TF truncated_normal semantics)
            x[bad] = torch.randn(int(bad.sum()), generator=gen, dtype=torch.float32)
            bad = x.abs() > 2.0
        t.copy_(x * std)
    return t


def init_params(spec: ModelSpec, seed: int = 1234, device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """Initial values with the reference initialisers.

    ``fm_w`` is 1-D: TF's fan computation gives fan_in = fan_out = V.  MLP weights use the
    ``fully_connected`` default xavier *uniform*; biases 0; BN gamma 1, beta 0, moving var 1.
    """
    gen = torch.Generator().manual_seed(seed)
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for name, shape in param_shapes(spec).items():
        t = torch.zeros(shape, dtype=torch.float32)
        if name == "fm_w":
            glorot_normal_(t, spec.feature_size, spec.feature_size, gen)
        elif name == "fm_v":
            glorot_normal_(t, spec.feature_size, spec.embedding_size, gen)
        elif name.endswith("/weights"):
            lim = math.sqrt(6.0 / (shape[0] + shape[1]))
            with torch.no_grad():
                t.uniform_(-lim, lim, generator=gen)
        elif name.endswith("gamma") or name.endswith("moving_variance"):
            t.fill_(1.0)
        out[name] = t.to(device)
    return out


def mlp_names(spec: ModelSpec) -> List[Tuple[str, str]]:
    names = [(f"Deep-part/mlp{i}/weights", f"Deep-part/mlp{i}/biases") for i in range(len(spec.layers))]
    names.append(("Deep-part/deep_out/weights", "Deep-part/deep_out/biases"))
    return names


def batch_norm(h: torch.Tensor, P: Dict[str, torch.Tensor], i: int, train: bool, decay: float,
               eps: float = 1e-3) -> torch.Tensor:
    """contrib.layers.batch_norm(center=True, scale=True, updates_collections=None) (PS:316-338).

    Train: normalise with batch moments, update moving averages in place (decay); the moving
    variance uses the unbiased batch variance like TF's fused batch norm [ext].  Infer: moving stats.
    """
    beta, gamma = P[f"Deep-part/bn_{i}/beta"], P[f"Deep-part/bn_{i}/gamma"]
    mm, mv = P[f"Deep-part/bn_{i}/moving_mean"], P[f"Deep-part/bn_{i}/moving_variance"]
    if train:
        mean = h.mean(0)
        var = h.var(0, unbiased=False)
        with torch.no_grad():
            n = h.shape[0]
            unb = var.detach() * (n / max(n - 1, 1))
            mm.mul_(decay).add_(mean.detach(), alpha=1 - decay)
            mv.mul_(decay).add_(unb, alpha=1 - decay)
    else:
        mean, var = mm, mv
    return (h - mean) * torch.rsqrt(var + eps) * gamma + beta


def forward(P: Dict[str, torch.Tensor], ids: torch.Tensor, vals: torch.Tensor, spec: ModelSpec, train: bool,
            masks: Optional[List[torch.Tensor]] = None, gen: Optional[torch.Generator] = None,
            rows_w: Optional[torch.Tensor] = None, rows_v: Optional[torch.Tensor] = None,
            return_aux: bool = False):
    """Logits y[B].  ``rows_w[B,F]``/``rows_v[B,F,K]`` may be supplied pre-gathered (sparse engine).

    ``masks[i]`` (optional) are explicit 0/1 dropout keep masks for layer i; otherwise dropout
    draws from ``gen``/global RNG.  Dropout is applied only when ``train`` (PS:245-246).
    """
    B, F = ids.shape
    K = spec.embedding_size
    w = P["fm_w"][ids] if rows_w is None else rows_w  # [B,F]
    y_w = (w * vals).sum(1)
    v = P["fm_v"][ids] if rows_v is None else rows_v  # [B,F,K]
    e = v * vals.unsqueeze(-1)
    S = e.sum(1)
    y_v = 0.5 * (S * S - (e * e).sum(1)).sum(1)
    h = e.reshape(B, F * K)
    for i, (wn, bn) in enumerate(mlp_names(spec)[:-1]):
        h = torch.relu(h @ P[wn] + P[bn])
        if spec.batch_norm:
            h = batch_norm(h, P, i, train, spec.batch_norm_decay)
        if train:
            keep = spec.keep_probs[i]
            if masks is not None:
                h = h * masks[i].to(h.dtype) / keep
            elif keep < 1.0:
                if gen is not None:
                    m = (torch.rand(h.shape, generator=gen, device=h.device) < keep).to(h.dtype)
                    h = h * m / keep
                else:
                    h = Fn.dropout(h, p=1.0 - keep, training=True)
    wn, bn = mlp_names(spec)[-1]
    y_d = (h @ P[wn] + P[bn]).reshape(-1)
    y = P["fm_bias"] + y_w + y_v + y_d
    if return_aux:
        return y, {"y_w": y_w, "y_v": y_v, "y_d": y_d, "S": S, "e": e}
    return y


def data_loss(y: torch.Tensor, labels: torch.Tensor, loss_type: str = "log_loss") -> torch.Tensor:
    """Mean per-example loss (without the L2 terms)."""
    if loss_type == "log_loss":
        return Fn.binary_cross_entropy_with_logits(y, labels)  # = TF sigmoid_cross_entropy_with_logits
    return ((torch.sigmoid(y) - labels) ** 2).mean()


def l2_terms(P: Dict[str, torch.Tensor], l2_reg: float) -> torch.Tensor:
    """λ·l2_loss(fm_w) + λ·l2_loss(fm_v) with TF l2_loss(x) = Σx²/2 (PS:277-278)."""
    return l2_reg * 0.5 * ((P["fm_w"] ** 2).sum() + (P["fm_v"] ** 2).sum())


def full_loss(P, y, labels, spec: ModelSpec) -> torch.Tensor:
    return data_loss(y, labels, spec.loss_type) + l2_terms(P, spec.l2_reg)
