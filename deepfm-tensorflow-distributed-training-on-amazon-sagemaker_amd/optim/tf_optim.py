"""TF-1.x-formula optimizers, dense and row-sparse (lazy), on plain tensors.

The reference picks the optimizer at ``model_fn`` (PS:292-307, HVD:281-297):

=========  =====================================================  ==================
name       update (t = global_step + 1)                           TF slot names
=========  =====================================================  ==================
Adam       lr_t = lr·√(1−β2ᵗ)/(1−β1ᵗ); m ← β1m+(1−β1)g;          ``Adam``, ``Adam_1``
           v ← β2v+(1−β2)g²; θ ← θ − lr_t·m/(√v+ε)
Adagrad    acc ← acc+g²; θ ← θ − lr·g/√acc  (acc₀ = 1e-8, PS:297)   ``Adagrad``
Momentum   a ← 0.95a+g; θ ← θ − lr·a  (PS:301)                      ``Momentum``
ftrl       TF FtrlOptimizer defaults (lr_power −0.5, acc₀ 0.1,      ``Ftrl``, ``Ftrl_1``
           l1 = l2 = 0)
GD         θ ← θ − lr·g  (advertised at PS:60 but missing; Q5)      —
=========  =====================================================  ==================

``apply_dense`` is what TF does for every variable in the reference (the full-table L2 makes
the embedding gradients dense).  ``apply_rows`` is the lazy/sparse update used in
``embedding_update=sparse`` mode: only the touched rows and their slots move.  The HIP kernels
(csrc/kernels/optim.h) implement the same formulas; tests compare them against this file.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List

import torch

OPTIMIZERS = ("Adam", "Adagrad", "Momentum", "ftrl", "GD")
OPT_ID = {"Adam": 0, "Adagrad": 1, "Momentum": 2, "ftrl": 3, "GD": 4}


@dataclass
class OptHParams:
    name: str = "Adam"
    lr: float = 0.0005
    beta1: float = 0.9
    beta2: float = 0.999
    eps: float = 1e-8
    adagrad_init: float = 1e-8
    momentum: float = 0.95
    ftrl_lr_power: float = -0.5
    ftrl_init: float = 0.1
    ftrl_l1: float = 0.0
    ftrl_l2: float = 0.0


def slot_names(name: str) -> List[str]:
    return {"Adam": ["Adam", "Adam_1"], "Adagrad": ["Adagrad"], "Momentum": ["Momentum"],
            "ftrl": ["Ftrl", "Ftrl_1"], "GD": []}[name]


def init_slots(hp: OptHParams, param: torch.Tensor) -> List[torch.Tensor]:
    z = lambda: torch.zeros_like(param)  # noqa: E731
    if hp.name == "Adam":
        return [z(), z()]
    if hp.name == "Adagrad":
        return [torch.full_like(param, hp.adagrad_init)]
    if hp.name == "Momentum":
        return [z()]
    if hp.name == "ftrl":
        return [torch.full_like(param, hp.ftrl_init), z()]
    return []


def adam_lr_t(hp: OptHParams, step: int) -> float:
    return hp.lr * math.sqrt(1.0 - hp.beta2 ** step) / (1.0 - hp.beta1 ** step)


@torch.no_grad()
def _update(hp: OptHParams, p: torch.Tensor, g: torch.Tensor, slots: List[torch.Tensor], step: int) -> None:
    """In-place update of (p, slots) given gradient g (all same shape)."""
    if hp.name == "Adam":
        m, v = slots
        m.mul_(hp.beta1).add_(g, alpha=1.0 - hp.beta1)
        v.mul_(hp.beta2).addcmul_(g, g, value=1.0 - hp.beta2)
        p.sub_(adam_lr_t(hp, step) * m / (v.sqrt() + hp.eps))
    elif hp.name == "Adagrad":
        (acc,) = slots
        acc.addcmul_(g, g)
        p.sub_(hp.lr * g / acc.sqrt())
    elif hp.name == "Momentum":
        (a,) = slots
        a.mul_(hp.momentum).add_(g)
        p.sub_(hp.lr * a)
    elif hp.name == "ftrl":
        acc, lin = slots
        acc_new = acc + g * g
        if hp.ftrl_lr_power == -0.5:  # TF's ApplyFtrl special case (sqrt instead of pow)
            pn, po = acc_new.sqrt(), acc.sqrt()
        else:
            pn, po = acc_new.pow(-hp.ftrl_lr_power), acc.pow(-hp.ftrl_lr_power)
        sigma = (pn - po) / hp.lr
        lin.add_(g - sigma * p)
        quad = pn / hp.lr + 2.0 * hp.ftrl_l2
        pnew = torch.where(lin.abs() > hp.ftrl_l1, (torch.sign(lin) * hp.ftrl_l1 - lin) / quad, torch.zeros_like(p))
        p.copy_(pnew)
        acc.copy_(acc_new)
    elif hp.name == "GD":
        p.sub_(hp.lr * g)
    else:
        raise ValueError(hp.name)


@torch.no_grad()
def apply_dense(hp: OptHParams, p: torch.Tensor, g: torch.Tensor, slots: List[torch.Tensor], step: int) -> None:
    _update(hp, p, g, slots, step)


@torch.no_grad()
def apply_rows(hp: OptHParams, p: torch.Tensor, rows: torch.Tensor, g_rows: torch.Tensor,
               slots: List[torch.Tensor], step: int) -> None:
    """Lazy update: rows (unique, int64) of p (first dim) with grads g_rows."""
    pr = p[rows]
    sr = [s[rows] for s in slots]
    _update(hp, pr, g_rows, sr, step)
    p[rows] = pr
    for s, s_r in zip(slots, sr):
        s[rows] = s_r
