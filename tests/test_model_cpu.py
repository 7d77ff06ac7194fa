"""Eager DeepFM (engine=torch): reference math, autograd, exact-vs-sparse semantics, oracles."""
import math

import numpy as np
import pytest
import torch

from rocfm.models.deepfm import ModelSpec, forward, full_loss, init_params, param_shapes
from rocfm.models.torch_engine import TorchDeepFM
from rocfm.ops import reference as R
from rocfm.optim import OptHParams


def _spec(**kw):
    d = dict(feature_size=50, field_size=6, embedding_size=4, layers=[8, 4], keep_probs=[1.0, 1.0], l2_reg=1e-3)
    d.update(kw)
    return ModelSpec(**d)


def _batch(spec, B, seed=0, V=None):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V or spec.feature_size, (B, spec.field_size), generator=g)
    vals = torch.rand(B, spec.field_size, generator=g)
    labels = (torch.rand(B, generator=g) < 0.4).float()
    return ids, vals, labels


def test_tf_variable_names_and_shapes():
    s = param_shapes(ModelSpec(117581, 39, 32, [128, 64, 32], [0.5] * 3, batch_norm=True))
    assert s["fm_v"] == (117581, 32) and s["fm_w"] == (117581,) and s["fm_bias"] == (1,)
    assert s["Deep-part/mlp0/weights"] == (1248, 128) and s["Deep-part/deep_out/weights"] == (32, 1)
    assert "Deep-part/bn_2/moving_variance" in s
    total = sum(int(np.prod(v)) for k, v in param_shapes(ModelSpec(117581, 39, 32, [128, 64, 32], [0.5] * 3)).items())
    assert total == 4050415


def test_initializers_statistics():
    spec = ModelSpec(20000, 39, 10, [128, 64, 32], [0.5] * 3)
    P = init_params(spec, 0)
    std_v = math.sqrt(2.0 / (20000 + 10))
    v = P["fm_v"]
    assert v.abs().max() <= 2 * std_v / 0.8796256610342398 + 1e-6  # truncated at 2σ
    assert abs(v.std().item() - std_v) / std_v < 0.02  # truncation-corrected std
    lim = math.sqrt(6.0 / (390 + 128))
    W = P["Deep-part/mlp0/weights"]
    assert W.abs().max() <= lim and abs(W.std().item() - lim / math.sqrt(3)) / (lim / math.sqrt(3)) < 0.03
    assert P["fm_bias"].item() == 0 and P["Deep-part/mlp0/biases"].abs().sum() == 0


def test_forward_matches_manual_math():
    spec = _spec()
    P = init_params(spec, 1)
    ids, vals, _ = _batch(spec, 7)
    y, aux = forward(P, ids, vals, spec, train=False, return_aux=True)
    e = P["fm_v"][ids] * vals[..., None]
    ym = (P["fm_w"][ids] * vals).sum(1)
    fm = 0.0
    for k in range(spec.embedding_size):  # ½((Σe)² − Σe²) per k, brute force
        s = e[:, :, k].sum(1)
        fm = fm + 0.5 * (s * s - (e[:, :, k] ** 2).sum(1))
    h = e.reshape(7, -1)
    for i in range(2):
        h = torch.relu(h @ P[f"Deep-part/mlp{i}/weights"] + P[f"Deep-part/mlp{i}/biases"])
    yd = (h @ P["Deep-part/deep_out/weights"]).reshape(-1) + P["Deep-part/deep_out/biases"]
    torch.testing.assert_close(y, P["fm_bias"] + ym + fm + yd)


def test_gradcheck_float64():
    spec = _spec()
    P = {k: v.double() for k, v in init_params(spec, 2).items()}
    ids, vals, labels = _batch(spec, 5)
    vals, labels = vals.double(), labels.double()
    names = ["fm_v", "Deep-part/mlp0/weights", "fm_w"]

    def f(*ts):
        Q = dict(P)
        Q.update(zip(names, ts))
        y = forward(Q, ids, vals, spec, train=False)
        return full_loss(Q, y, labels, spec)

    assert torch.autograd.gradcheck(f, tuple(P[n].clone().requires_grad_(True) for n in names))


@pytest.mark.parametrize("opt", ["Adam", "Adagrad", "Momentum", "ftrl", "GD"])
def test_exact_equals_sparse_when_every_row_is_touched(opt):
    spec = _spec(feature_size=12)  # tiny vocab: every row appears in every batch
    P = init_params(spec, 3)
    hp = OptHParams(name=opt, lr=0.01)
    a = TorchDeepFM(spec, hp, embedding_update="exact", params=P)
    b = TorchDeepFM(spec, hp, embedding_update="sparse", params=P)
    for s in range(3):
        ids, vals, labels = _batch(spec, 64, seed=s)
        assert len(torch.unique(ids)) == 12
        a.train_step(ids, vals, labels)
        b.train_step(ids, vals, labels)
    for k in a.P:
        torch.testing.assert_close(a.P[k], b.P[k], rtol=1e-5, atol=1e-6)


def test_training_reduces_loss_on_learnable_data():
    from rocfm.data.synthetic import SyntheticCriteo

    gen = SyntheticCriteo(3000, 39, seed=0)
    spec = ModelSpec(3000, 39, 8, [32, 16], [1.0, 1.0], l2_reg=1e-5)
    eng = TorchDeepFM(spec, OptHParams(lr=5e-3), params=init_params(spec, 0))
    g = torch.Generator().manual_seed(0)
    ev = gen.batch(2000, "cpu", g)
    p0, l0 = eng.predict_batch(*ev)
    for _ in range(60):
        eng.train_step(*gen.batch(256, "cpu", g))
    p1, l1 = eng.predict_batch(*ev)
    from rocfm.metrics import exact_auc

    assert l1.mean() < l0.mean()
    assert exact_auc(ev[2], p1) > 0.65


def test_dropout_mask_replica_matches_scalar_philox():
    """numpy Philox replica == a direct scalar transcription of csrc/common.h."""
    def philox(c, k0, k1):
        c = list(c)
        for _ in range(10):
            p0 = 0xD2511F53 * c[0]
            p1 = 0xCD9E8D57 * c[2]
            c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
                 p0 & 0xFFFFFFFF]
            k0 = (k0 + 0x9E3779B9) & 0xFFFFFFFF
            k1 = (k1 + 0xBB67AE85) & 0xFFFFFFFF
        return c

    seed, layer, step, keep = 0x1234567890AB, 2, 17, 0.5
    m = R.dropout_masks(seed, layer, step, 8, 5, keep)
    for r in range(8):
        for c in range(5):
            lanes = philox([r >> 2, c, layer, step], seed & 0xFFFFFFFF, seed >> 32)
            u = (lanes[r & 3] >> 8) / 16777216.0
            assert bool(m[r, c]) == (np.float32(u) < np.float32(keep))
    big = R.dropout_masks(7, 0, 0, 256, 128, 0.5)
    assert abs(big.float().mean().item() - 0.5) < 0.02


def test_fused_reference_gradients_vs_autograd():
    """The kernel oracle's backward equals autograd of the same bf16-emulating forward."""
    spec = _spec(feature_size=40, layers=[16, 8])
    P = init_params(spec, 4)
    ids, vals, labels = _batch(spec, 12)
    K = spec.embedding_size
    emb = torch.zeros(40, 8)
    emb[:, :K] = P["fm_v"]
    emb[:, K] = P["fm_w"]
    layers = [{"W": P[f"Deep-part/mlp{i}/weights"], "b": P[f"Deep-part/mlp{i}/biases"]} for i in range(2)]
    w_out = P["Deep-part/deep_out/weights"].reshape(-1)
    ref = R.fused_step_reference(emb, layers, w_out, 0.0, 0.0, ids, vals, labels, K, [1.0, 1.0], None, 1.0 / 12)
    # autograd of the f32 model (no bf16 rounding) — close within bf16 tolerance
    Q = {k: v.clone().requires_grad_(k in ("Deep-part/mlp0/weights", "Deep-part/deep_out/weights")) for k, v in P.items()}
    y = forward(Q, ids, vals, spec, train=False)
    torch.nn.functional.binary_cross_entropy_with_logits(y, labels).backward()
    torch.testing.assert_close(ref["dW"][0], Q["Deep-part/mlp0/weights"].grad, rtol=0.05, atol=2e-3)
    torch.testing.assert_close(ref["dw_out"], Q["Deep-part/deep_out/weights"].grad.reshape(-1), rtol=0.05, atol=2e-3)


@pytest.mark.parametrize("exact", [True, False])
def test_fused_reference_batch_norm_vs_autograd(monkeypatch, exact):
    """The kernel oracle's batch-norm forward/backward (batch moments, γ/β gradients, dz through
    the normalisation) equals autograd of the f32 DeepFM with batch_norm=True: exactly with the
    oracle's bf16 operand rounding switched off, within bf16 tolerance with it (fixed γ/β: at 24
    rows the normalisation amplifies bf16 rounding by up to ~15× for some draws)."""
    if exact:
        monkeypatch.setattr(R, "bf16", lambda x: x)
    spec = _spec(feature_size=40, layers=[16, 8])
    spec.batch_norm = True
    P = init_params(spec, 5)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():  # non-trivial γ / β
        for i in range(2):
            P[f"Deep-part/bn_{i}/gamma"].uniform_(0.5, 1.5, generator=g)
            P[f"Deep-part/bn_{i}/beta"].uniform_(-0.2, 0.2, generator=g)
    ids, vals, labels = _batch(spec, 24)
    K = spec.embedding_size
    emb = torch.zeros(40, 8)
    emb[:, :K] = P["fm_v"]
    emb[:, K] = P["fm_w"]
    layers = [{"W": P[f"Deep-part/mlp{i}/weights"], "b": P[f"Deep-part/mlp{i}/biases"]} for i in range(2)]
    bn = [{"gamma": P[f"Deep-part/bn_{i}/gamma"], "beta": P[f"Deep-part/bn_{i}/beta"]} for i in range(2)]
    w_out = P["Deep-part/deep_out/weights"].reshape(-1)
    ref = R.fused_step_reference(emb, layers, w_out, 0.0, 0.0, ids, vals, labels, K, [1.0, 1.0], None, 1.0 / 24,
                                 bn=bn)
    names = ["Deep-part/mlp0/weights", "Deep-part/mlp1/biases", "Deep-part/bn_0/gamma", "Deep-part/bn_1/beta",
             "Deep-part/bn_0/beta", "Deep-part/bn_1/gamma"]
    Q = {k: v.clone().requires_grad_(k in names) for k, v in P.items()}
    y = forward(Q, ids, vals, spec, train=True)
    torch.nn.functional.binary_cross_entropy_with_logits(y, labels).backward()
    tol = dict(rtol=1e-4, atol=1e-6) if exact else dict(rtol=0.06, atol=3e-3)
    torch.testing.assert_close(ref["dW"][0], Q[names[0]].grad, **tol)
    torch.testing.assert_close(ref["db"][1], Q[names[1]].grad, **tol)
    torch.testing.assert_close(ref["dgamma"][0], Q[names[2]].grad, **tol)
    torch.testing.assert_close(ref["dbeta"][1], Q[names[3]].grad, **tol)
    torch.testing.assert_close(ref["dbeta"][0], Q[names[4]].grad, **tol)
    torch.testing.assert_close(ref["dgamma"][1], Q[names[5]].grad, **tol)
    # the oracle's probabilities match the model's training-mode forward
    ptol = dict(rtol=1e-5, atol=1e-6) if exact else dict(rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(ref["prob"], torch.sigmoid(y.detach()), **ptol)


def test_step_tail_wgrad_plan_fits_one_dispatch_round():
    """The step tail widens the weight-gradient tiles of wide layers while its two roles exceed the
    256 CUs' one round (to 32 × 64 tiles; ROCFM_WGRAD_TW=auto to 32 × 128) (wgrad_body.h wgrad_prepare): the reference's flag defaults
    (39·32 → 256-128-64) and the notebook MLP go from two rounds to one; the bench shape keeps its
    32×32 tiles."""
    import os

    import pytest

    from rocfm.ops import hip

    H = hip()
    if H is None or not hasattr(H, "wgrad_plan"):
        pytest.skip("rocfm._rocfm_hip not built")
    os.environ.pop("ROCFM_WGRAD_TW", None)
    emb = lambda F, B=1024: -(-B * F // H.tail_chunk())  # noqa: E731 — embedding workgroups
    n, tw = H.wgrad_plan([416, 128, 64, 32], 1024, emb(39), 256)  # 39·10 → 128-64-32 (padded to 32)
    assert tw == [1, 1, 1] and n + emb(39) <= 256
    # (the widest tiles are 32 × 128; a few bias / output workgroups may spill past the round)
    # (the default widens up to 32 × 64 tiles; ROCFM_WGRAD_TW=auto up to 32 × 128, below)
    n, tw = H.wgrad_plan([1248, 256, 128, 64], 1024, emb(39), 256)
    assert tw == [2, 2, 2], (n, tw)
    n, tw = H.wgrad_plan([1248, 128, 64, 32], 1024, emb(39), 256)
    assert n + emb(39) <= 256 and tw[0] == 2, (n, tw)
    n0, tw = H.wgrad_plan([1248, 256, 128, 64], 1024, -1, 256)  # standalone launch: plain tiles
    assert tw == [1, 1, 1] and n0 == 39 * 8 + 8 * 4 + 4 * 2 + (256 + 128 + 64) // 32 + 1
    # ROCFM_WGRAD_TW=auto widens exactly as the unset variable does (it used to read as "force 0",
    # i.e. plain tiles); 2 / 4 force a width
    try:
        os.environ["ROCFM_WGRAD_TW"] = "auto"
        n, tw = H.wgrad_plan([1248, 256, 128, 64], 1024, emb(39), 256)
        assert n + emb(39) <= 256 + 8 and tw == [4, 4, 2], (n, tw)
        os.environ["ROCFM_WGRAD_TW"] = "2"
        assert H.wgrad_plan([1248, 256, 128, 64], 1024, emb(39), 256)[1] == [2, 2, 2]
    finally:
        os.environ.pop("ROCFM_WGRAD_TW", None)
