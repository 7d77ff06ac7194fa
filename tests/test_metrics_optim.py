import math

import numpy as np
import pytest
import torch

from rocfm.metrics import TFStreamingAUC, exact_auc, logloss, tf_thresholds
from rocfm.optim import OptHParams, adam_lr_t, apply_dense, apply_rows, init_slots


def _pairwise_auc(y, p):
    pos, neg = p[y == 1], p[y == 0]
    gt = (pos[:, None] > neg[None, :]).sum() + 0.5 * (pos[:, None] == neg[None, :]).sum()
    return gt / (len(pos) * len(neg))


def test_exact_auc_matches_pairwise_with_ties():
    g = np.random.default_rng(0)
    y = (g.random(500) < 0.3).astype(np.float32)
    p = np.round(g.random(500) * 20) / 20  # many ties
    assert abs(exact_auc(y, p) - _pairwise_auc(y, p)) < 1e-12
    assert exact_auc([0, 1, 0, 1], [0.1, 0.9, 0.2, 0.8]) == 1.0


def test_tf_auc_formula_and_streaming():
    thr = tf_thresholds(200)
    assert len(thr) == 200 and thr[0] < 0 and thr[-1] > 1 and abs(thr[1] - 1 / 199) < 1e-12
    g = np.random.default_rng(1)
    y = (g.random(3000) < 0.25).astype(np.float32)
    p = np.clip(y * 0.3 + g.random(3000) * 0.7, 0, 1)
    a = TFStreamingAUC()
    for i in range(0, 3000, 700):  # streaming accumulation == one-shot
        a.update(y[i:i + 700], p[i:i + 700])
    b = TFStreamingAUC()
    b.update(y, p)
    assert a.result() == b.result()
    # hand-computed TF formula
    tp = np.array([(p[y == 1] > t).sum() for t in thr], np.float64)
    fp = np.array([(p[y == 0] > t).sum() for t in thr], np.float64)
    fn = (y == 1).sum() - tp
    tn = (y == 0).sum() - fp
    tpr = (tp + 1e-7) / (tp + fn + 1e-7)
    fpr = fp / (fp + tn + 1e-7)
    ref = np.sum((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2)
    assert abs(a.result() - ref) < 1e-12
    assert abs(a.result() - exact_auc(y, p)) < 0.01  # 200-bucket approximation is close


def test_logloss():
    assert abs(logloss([1, 0], [0.9, 0.1]) - (-math.log(0.9))) < 1e-9


def _hand(name, p0, grads, **kw):
    """Scalar re-implementation of the TF update rules, for cross-checking."""
    p = float(p0)
    if name == "Adam":
        m = v = 0.0
        for t, g in enumerate(grads, 1):
            lr_t = kw["lr"] * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
            m = 0.9 * m + 0.1 * g
            v = 0.999 * v + 0.001 * g * g
            p -= lr_t * m / (math.sqrt(v) + 1e-8)
    elif name == "Adagrad":
        acc = 1e-8
        for g in grads:
            acc += g * g
            p -= kw["lr"] * g / math.sqrt(acc)
    elif name == "Momentum":
        a = 0.0
        for g in grads:
            a = 0.95 * a + g
            p -= kw["lr"] * a
    elif name == "GD":
        for g in grads:
            p -= kw["lr"] * g
    elif name == "ftrl":
        acc, lin = 0.1, 0.0
        for g in grads:
            an = acc + g * g
            lin += g - (math.sqrt(an) - math.sqrt(acc)) / kw["lr"] * p
            quad = math.sqrt(an) / kw["lr"]
            p = (-lin) / quad if abs(lin) > 0 else 0.0
            acc = an
    return p


@pytest.mark.parametrize("name", ["Adam", "Adagrad", "Momentum", "GD", "ftrl"])
def test_tf_optimizer_formulas(name):
    hp = OptHParams(name=name, lr=0.05)
    grads = [0.3, -0.1, 0.7, 0.05]
    p = torch.tensor([0.2], dtype=torch.float64)
    slots = [s.double() for s in init_slots(hp, p)]
    for t, g in enumerate(grads, 1):
        apply_dense(hp, p, torch.tensor([g], dtype=torch.float64), slots, t)
    assert abs(float(p) - _hand(name, 0.2, grads, lr=0.05)) < 1e-10


def test_adam_lr_t():
    hp = OptHParams(lr=1e-3)
    assert abs(adam_lr_t(hp, 1) - 1e-3 * math.sqrt(0.001) / 0.1) < 1e-15


@pytest.mark.parametrize("name", ["Adam", "Adagrad", "Momentum", "GD", "ftrl"])
def test_rows_update_equals_dense_when_all_rows_touched(name):
    hp = OptHParams(name=name, lr=0.01)
    g = torch.Generator().manual_seed(0)
    P1 = torch.randn(6, 3, generator=g)
    P2 = P1.clone()
    s1, s2 = init_slots(hp, P1), init_slots(hp, P2)
    for t in range(1, 4):
        grad = torch.randn(6, 3, generator=g)
        apply_dense(hp, P1, grad, s1, t)
        perm = torch.randperm(6, generator=g)
        apply_rows(hp, P2, perm, grad[perm], s2, t)
    assert torch.allclose(P1, P2, atol=1e-6)
    # untouched rows do not move (lazy)
    P3 = P1.clone()
    s3 = [s.clone() for s in s1]
    apply_rows(hp, P3, torch.tensor([1, 4]), torch.ones(2, 3), s3, 5)
    assert torch.equal(P3[[0, 2, 3, 5]], P1[[0, 2, 3, 5]])
