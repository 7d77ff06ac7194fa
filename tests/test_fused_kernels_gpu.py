"""Numerics of the fused HIP kernels vs the plain-PyTorch fp32 oracle (rocfm/ops/reference.py)."""
import numpy as np
import pytest
import torch

from rocfm.models.deepfm import ModelSpec, init_params
from rocfm.models.fused import FusedDeepFM
from rocfm.ops import reference as R
from rocfm.optim import OptHParams, apply_dense, init_slots

pytestmark = pytest.mark.gpu


def _batch(B, F, V, gen, hot=True):
    ids = torch.randint(0, V, (B, F), generator=gen, dtype=torch.int64)
    if hot:  # numeric-style fields: fixed ids 1..13 in every example (extreme duplication)
        ids[:, :13] = torch.arange(1, 14)
        ids[:, 13] = V - 1  # last row
    vals = torch.rand(B, F, generator=gen)
    vals[:, 13:] = 1.0
    labels = (torch.rand(B, generator=gen) < 0.3).float()
    return ids.to(torch.int32), vals, labels


def _ref_inputs(eng: FusedDeepFM, spec: ModelSpec, step: int, keeps):
    sd = eng.parameters_tf()
    emb = eng.emb.detach().cpu()
    layers = []
    for l in range(len(spec.layers)):
        layers.append({"W": sd[f"Deep-part/mlp{l}/weights"].float(), "b": sd[f"Deep-part/mlp{l}/biases"].float()})
    w_out = sd["Deep-part/deep_out/weights"].reshape(-1).float()
    b_out = float(sd["Deep-part/deep_out/biases"])
    fmb = float(sd["fm_bias"])
    masks = []
    L = eng.layout
    for l in range(len(spec.layers)):
        m = R.dropout_masks(eng.seed, l, step, eng.Bp, L.dims[l + 1], keeps[l])
        masks.append(m[: eng.B, : spec.layers[l]])
    return emb, layers, w_out, b_out, fmb, masks


@pytest.mark.parametrize("K,layers,generic,tw", [
    (10, [128, 64, 32], False, 0), (10, [128, 64, 32], True, 0), (32, [256, 128, 64], False, 0), (8, [48, 16], False, 0),
    (10, [64, 32], False, 0), (32, [128, 64, 32], False, 0), (32, [128, 64, 32], True, 0), (32, [256, 128, 64], True, 0),
    # wide weight-gradient tiles (32 × 64 / 32 × 128: the step tail's one-dispatch-round layout for
    # wide layers, forced here on every layer they divide)
    (32, [256, 128, 64], False, 4), (10, [128, 64, 32], False, 2), (32, [128, 64, 32], True, 4)])
def test_fused_step_gradients_match_oracle(K, layers, generic, tw, monkeypatch):
    if tw:
        monkeypatch.setenv("ROCFM_WGRAD_TW", str(tw))
    torch.manual_seed(0)
    dev = torch.device("cuda")
    V, F, B = 5000, 39, 192
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=layers,
                     keep_probs=[0.5] * len(layers), l2_reg=1e-3)
    hp = OptHParams(name="GD", lr=1.0)
    eng = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 7), use_graph=False,
                      force_generic_kernels=generic)
    gen = torch.Generator().manual_seed(1)
    ids, vals, labels = _batch(B, F, V, gen)
    emb, lays, w_out, b_out, fmb, masks = _ref_inputs(eng, spec, 0, spec.keep_probs)
    before_dense = eng.parameters_tf()
    eng.load_batch(ids.to(dev), vals.to(dev), labels.to(dev))
    eng.train_step()
    torch.cuda.synchronize()
    ref = R.fused_step_reference(emb, lays, w_out, b_out, fmb, ids, vals, labels, K, spec.keep_probs, masks,
                                 1.0 / B, train=True)
    # forward
    torch.testing.assert_close(eng.prob[:B].cpu(), ref["prob"], rtol=2e-3, atol=2e-4)
    after = eng.parameters_tf()
    # dense grads = before - after (GD lr=1)
    for l in range(len(layers)):
        dW = before_dense[f"Deep-part/mlp{l}/weights"] - after[f"Deep-part/mlp{l}/weights"]
        torch.testing.assert_close(dW, ref["dW"][l], rtol=2e-2, atol=2e-5)
        db = before_dense[f"Deep-part/mlp{l}/biases"] - after[f"Deep-part/mlp{l}/biases"]
        torch.testing.assert_close(db, ref["db"][l], rtol=2e-2, atol=2e-5)
    dwo = (before_dense["Deep-part/deep_out/weights"] - after["Deep-part/deep_out/weights"]).reshape(-1)
    torch.testing.assert_close(dwo, ref["dw_out"], rtol=2e-3, atol=1e-6)
    dbo = float(before_dense["Deep-part/deep_out/biases"] - after["Deep-part/deep_out/biases"])
    assert abs(dbo - float(ref["d_bout"])) < 1e-5
    assert abs(float(before_dense["fm_bias"] - after["fm_bias"]) - float(ref["d_bout"])) < 1e-5
    # embedding: touched rows move by Σcontrib + λθ (lazy L2); untouched rows do not move
    uniq, acc = R.emb_grad_reference(ids, ref["contrib"])
    emb_after = eng.emb.detach().cpu()
    delta = emb[:, : K + 1] - emb_after[:, : K + 1]
    exp = acc + spec.l2_reg * emb[uniq, : K + 1]
    torch.testing.assert_close(delta[uniq], exp, rtol=5e-3, atol=2e-6)
    mask = torch.ones(V, dtype=torch.bool)
    mask[uniq] = False
    assert torch.equal(emb_after[mask], emb[mask])


def test_fused_adam_two_steps_and_graph_replay():
    dev = torch.device("cuda")
    V, F, K, B = 3000, 39, 10, 128
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[128, 64, 32],
                     keep_probs=[1.0, 1.0, 1.0], l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=1e-3)
    gen = torch.Generator().manual_seed(3)
    ids, vals, labels = _batch(B, F, V, gen)
    a = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 11), use_graph=False)
    b = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 11), use_graph=True)
    batch = (ids.to(dev), vals.to(dev), labels.to(dev))
    for eng in (a, b):
        for _ in eng.train_on([batch] * 5):  # graph engine: 2 eager warm-up steps, capture, replays
            pass
    torch.cuda.synchronize()
    # deterministic kernels (no atomics): graph replay == eager, bitwise
    assert torch.equal(a.emb, b.emb)
    assert torch.equal(a.dense, b.dense)
    assert a.global_step() == b.global_step() == 5


def test_fused_adam_matches_tf_formula_one_step():
    dev = torch.device("cuda")
    V, F, K, B = 2000, 39, 10, 64
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=1e-4)
    P = init_params(spec, 5)
    gen = torch.Generator().manual_seed(9)
    ids, vals, labels = _batch(B, F, V, gen)
    ref_eng = FusedDeepFM(spec, OptHParams(name="GD", lr=1.0), B, dev, params=P, use_graph=False)
    adam = FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, dev, params=P, use_graph=False)
    before = ref_eng.parameters_tf()
    for eng in (ref_eng, adam):
        eng.load_batch(ids.to(dev), vals.to(dev), labels.to(dev))
        eng.train_step()
    torch.cuda.synchronize()
    grads = {k: before[k] - v for k, v in ref_eng.parameters_tf().items()}
    got = adam.parameters_tf()
    hp = OptHParams(name="Adam", lr=1e-3)
    for name in ("Deep-part/mlp0/weights", "Deep-part/mlp1/biases", "Deep-part/deep_out/weights"):
        p = before[name].clone()
        apply_dense(hp, p, grads[name], init_slots(hp, p), 1)
        torch.testing.assert_close(got[name], p, rtol=1e-3, atol=1e-5)


def test_device_auc_matches_streaming_auc():
    from rocfm.metrics import DeviceAUC, TFStreamingAUC

    g = torch.Generator().manual_seed(5)
    ref = TFStreamingAUC()
    dev = DeviceAUC("cuda")
    tot = 0.0
    for n in (1000, 4097, 1):
        p = torch.rand(n, generator=g)
        p[: n // 10] = torch.round(p[: n // 10] * 199) / 199  # exactly on thresholds
        y = (torch.rand(n, generator=g) < p).float()
        l = torch.rand(n, generator=g)
        tot += float(l.double().sum())
        ref.update(y, p)
        dev.update(y.cuda(), p.cuda(), l.cuda())
    np.testing.assert_array_equal(dev.state(), ref.state())
    assert abs(dev.streaming().result() - ref.result()) < 1e-12
    s, c = dev.loss_total()
    assert c == 5098 and abs(s - tot) < 1e-3


@pytest.mark.parametrize("sort", ["composite", "wide"])
@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_multi_step_graph_equals_per_step(update, sort, monkeypatch):
    """The multi-step pipeline (S steps per graph, one batched sort per graph, eager first graph,
    tail graph of S' < S) trains bit-identically to per-step eager training.  sort=wide: 64-bit
    step|id keys — the path of vocabularies too wide for the 32-bit composite key (100M-1B rows),
    forced here on a small one."""
    monkeypatch.setenv("ROCFM_SORT", sort)
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.7, 0.8],
                     l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=2e-3)
    g = torch.Generator().manual_seed(9)
    NB, B = 5, 128
    pool = [_batch(B, 39, 3000, g) for _ in range(NB)]
    ids = torch.stack([p[0] for p in pool]).cuda()
    vals = torch.stack([p[1] for p in pool]).cuda()
    labels = torch.stack([p[2] for p in pool]).cuda()
    a = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), embedding_update=update, use_graph=True)
    b = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), embedding_update=update, use_graph=False)
    a.attach_pool(ids, vals, labels)
    b.attach_pool(ids, vals, labels)
    a.train_steps(21, 8)  # 8 eager + 8 graph + 5 tail graph
    assert a.m_composite == (sort == "composite")
    for _ in range(21):
        b.train_step()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 21
    assert torch.equal(a.emb, b.emb) and torch.equal(a.dense, b.dense)
    assert torch.equal(a.emb_slots[1], b.emb_slots[1])
    # switching back to per-step training continues from the same global step / batch
    a.train_step()
    b.train_step()
    torch.cuda.synchronize()
    assert torch.equal(a.emb, b.emb)


def test_lean_launch_and_capture_first_equal_per_step(monkeypatch):
    """ROCFM_LEAN_LAUNCH=3 (reused launch events, no wait on a completed side graph, lazy trailing
    side-chain join) with the bench's capture-first warm-up order (precapture of a list of runs,
    bench.warm_capture_first), interleaved with per-step steps, a prediction and a state read,
    trains bit-identically to per-step eager training."""
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.7, 0.8],
                     l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=2e-3)
    g = torch.Generator().manual_seed(11)
    NB, B = 5, 128
    pool = [_batch(B, 39, 3000, g) for _ in range(NB)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    monkeypatch.setenv("ROCFM_LEAN_LAUNCH", "3")
    a = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True)
    monkeypatch.setenv("ROCFM_LEAN_LAUNCH", "0")
    b = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=False)
    assert a._lean_launch == 3
    a.attach_pool(ids, vals, labels)
    b.attach_pool(ids, vals, labels)
    a.train_steps(1, 8)  # eager first launch
    a.precapture([4, 8, 8], 8)  # the graphs of the next three calls, captured up front
    a.train_steps(4, 8)
    a.train_steps(8, 8)
    a.train_steps(8, 8)
    a.train_step()  # per-step path right behind a lazily joined side chain
    a.train_steps(5, 8)
    p_a = a.predict_batch(ids[0], vals[0], labels[0])[0].clone()
    for _ in range(27):
        b.train_step()
    p_b = b.predict_batch(ids[0], vals[0], labels[0])[0].clone()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == 27
    sa, sb = a.state_dict(), b.state_dict()
    for k in sb:
        assert torch.equal(sa[k], sb[k]), k
    assert torch.equal(p_a, p_b)
    a.check()


def test_train_stream_equals_per_step():
    """Host batches streamed through the HBM ring + multi-step graphs (two calls, the second
    starting mid-ring with a partial tail graph) train bit-identically to per-step training."""
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.7, 0.8],
                     l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=2e-3)
    g = torch.Generator().manual_seed(11)
    NB, B = 45, 128
    host = [tuple(t.pin_memory() for t in _batch(B, 39, 3000, g)) for _ in range(NB)]
    a = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True)
    b = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=False)
    seen = []
    assert a.train_stream(iter(host[:21]), 4, after_steps=lambda s, n: seen.append((s, n))) == 21
    assert seen[0] == (0, 4) and seen[-1] == (20, 1)
    assert a.train_stream(iter(host[21:]), 4) == 24
    b.attach_pool(torch.stack([h[0] for h in host]).cuda(), torch.stack([h[1] for h in host]).cuda(),
                  torch.stack([h[2] for h in host]).cuda())
    for _ in range(NB):
        b.train_step()
    torch.cuda.synchronize()
    assert a.global_step() == b.global_step() == NB
    assert torch.equal(a.emb, b.emb) and torch.equal(a.dense, b.dense)
    assert torch.equal(a.emb_slots[1], b.emb_slots[1])


def test_fp8_input_layer_matches_fp8_oracle():
    """compute_dtype=fp8: the input layer's forward GEMM and its dgrad (dz1·W0ᵀ, the embedding
    gradient's MLP part) run on fp8-e4m3 MFMA — activations / dz quantised per row in the kernel,
    the weights pre-quantised by the refresh with one per-tensor scale; the step matches an oracle
    with the same quantisation (and differs from the bf16 one by more than the comparison tolerance)."""
    torch.manual_seed(0)
    dev = torch.device("cuda")
    V, F, K, B = 5000, 39, 10, 192
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[128, 64, 32],
                     keep_probs=[1.0, 1.0, 1.0], l2_reg=1e-3)
    hp = OptHParams(name="GD", lr=1.0)
    eng = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 7), use_graph=False, compute_dtype="fp8")
    gen = torch.Generator().manual_seed(1)
    ids, vals, labels = _batch(B, F, V, gen)
    emb, lays, w_out, b_out, fmb, masks = _ref_inputs(eng, spec, 0, spec.keep_probs)
    before = eng.parameters_tf()
    eng.load_batch(ids.to(dev), vals.to(dev), labels.to(dev))
    eng.train_step()
    torch.cuda.synchronize()
    args = (emb, lays, w_out, b_out, fmb, ids, vals, labels, K, spec.keep_probs, masks, 1.0 / B)
    ref8 = R.fused_step_reference(*args, train=True, fp8=True)
    ref16 = R.fused_step_reference(*args, train=True, fp8=False)
    got = eng.prob[:B].cpu()
    torch.testing.assert_close(got, ref8["prob"], rtol=1e-3, atol=1e-4)
    assert (got - ref8["prob"]).abs().max() < 0.2 * (ref16["prob"] - ref8["prob"]).abs().max()
    after = eng.parameters_tf()
    for l in range(3):
        dW = before[f"Deep-part/mlp{l}/weights"] - after[f"Deep-part/mlp{l}/weights"]
        torch.testing.assert_close(dW, ref8["dW"][l], rtol=3e-2, atol=3e-5)
    # embedding rows (GD, lazy L2): the fp8 dgrad's quantisation shows in their update
    uniq, acc8 = R.emb_grad_reference(ids, ref8["contrib"])
    _, acc16 = R.emb_grad_reference(ids, ref16["contrib"])
    delta = (emb[:, : K + 1] - eng.emb.detach().cpu()[:, : K + 1])[uniq] - spec.l2_reg * emb[uniq, : K + 1]
    # a 1-ulp bf16 difference in dz (f32 accumulation order) can flip one fp8 rounding (≈6 % of one
    # product), hence the loose element tolerance; the second check separates fp8 from bf16 dgrad
    # (measured: |Δ − fp8 oracle| 1.1e-4, |Δ − bf16 oracle| 8.8e-4, rows up to 0.24)
    torch.testing.assert_close(delta, acc8, rtol=3e-2, atol=3e-4)
    assert (delta - acc8).abs().max() < 0.3 * (acc16 - acc8).abs().max()


def _frag_swz_index(R, C):
    """common.h frag_swz(r, c, C) for every (r, c) of an R×C matrix → int64 [R, C]."""
    r = torch.arange(R)[:, None]
    c = torch.arange(C)[None, :]
    nt, rl, u, cc = r >> 4, r & 15, c >> 5, c & 31
    return ((nt * (C >> 5) + u) * 64 + rl + 16 * (cc >> 3)) * 8 + (cc & 7)


def test_fp8_prequantised_copies_track_weights():
    """Delayed per-tensor scaling of the fp8 input-layer copies (deepfm_rows.h Fp8W0) through
    multi-step graphs with Adam: after n steps the amax slot of parity n holds max|W0| of the current
    master weights (accumulated by the last refresh), the de-scale is the previous weights' max / 448,
    and both swizzled fp8 copies equal the current weights quantised with it."""
    dev = torch.device("cuda")
    V, F, K, B = 5000, 39, 10, 256
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[128, 64, 32],
                     keep_probs=[0.8, 0.8, 0.8], l2_reg=1e-3)
    eng = FusedDeepFM(spec, OptHParams(name="Adam", lr=5e-3), B, dev, params=init_params(spec, 7), use_graph=True,
                      compute_dtype="fp8")
    g = torch.Generator().manual_seed(3)
    pool = [_batch(B, F, V, g) for _ in range(4)]
    eng.attach_pool(*(torch.stack([p[i] for p in pool]).to(dev) for i in range(3)))
    n = 11
    eng.train_steps(n, 4)
    torch.cuda.synchronize()
    L = eng.layout
    Din, Dout = L.dims[0], L.dims[1]
    W0 = eng.dense[L.offW[0]: L.offW[0] + Din * Dout].view(Din, Dout).cpu()
    f8, b8, amax, inv = (t.cpu() for t in eng.w8)
    assert amax[n & 1].item() == W0.abs().max().item()
    prev = inv.item() * 448.0
    assert prev > 0 and abs(prev / W0.abs().max().item() - 1) < 0.05  # one Adam step earlier
    q = (W0 * (448.0 / prev)).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    fwd = f8[_frag_swz_index(Dout, Din).reshape(-1)].view(Dout, Din).t()
    bwd = b8[_frag_swz_index(Din, Dout).reshape(-1)].view(Din, Dout)
    assert torch.equal(fwd, q) and torch.equal(bwd, q)


def test_fp8_training_tracks_bf16():
    """30 Adam steps with dropout: fp8 and bf16 engines from the same start stay close (loss within
    2 %, predictions within 0.05, 0.01 on average; measured 0.028 / 0.004) — the delayed weight
    scale does not drift."""
    dev = torch.device("cuda")
    V, F, K, B = 5000, 39, 10, 512
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[128, 64, 32],
                     keep_probs=[0.8, 0.8, 0.8], l2_reg=1e-4)
    g = torch.Generator().manual_seed(5)
    pool = [_batch(B, F, V, g) for _ in range(6)]
    out = {}
    for dt in ("bf16", "fp8"):
        e = FusedDeepFM(spec, OptHParams(name="Adam", lr=2e-3), B, dev, params=init_params(spec, 9), use_graph=True,
                        compute_dtype=dt)
        e.attach_pool(*(torch.stack([p[i] for p in pool]).to(dev) for i in range(3)))
        e.train_steps(30, 8)
        torch.cuda.synchronize()
        out[dt] = (float(e.loss_rows[:B].mean()), e.prob[:B].clone())
    assert abs(out["fp8"][0] - out["bf16"][0]) < 0.02 * out["bf16"][0]
    d = (out["fp8"][1] - out["bf16"][1]).abs()
    assert d.max() < 0.05 and d.mean() < 0.01


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _bn_spec(layers, keep):
    return ModelSpec(feature_size=5000, field_size=39, embedding_size=10, layers=layers,
                     keep_probs=[keep] * len(layers), l2_reg=1e-3, batch_norm=True, batch_norm_decay=0.9)


def _bn_params(spec, seed):
    P = init_params(spec, seed)
    g = torch.Generator().manual_seed(seed)
    for i in range(len(spec.layers)):  # non-trivial γ / β / moving moments
        n = spec.layers[i]
        P[f"Deep-part/bn_{i}/gamma"] = 0.5 + torch.rand(n, generator=g)
        P[f"Deep-part/bn_{i}/beta"] = 0.2 * torch.rand(n, generator=g) - 0.1
        P[f"Deep-part/bn_{i}/moving_mean"] = 0.1 * torch.rand(n, generator=g)
        P[f"Deep-part/bn_{i}/moving_variance"] = 0.5 + torch.rand(n, generator=g)
    return P


@pytest.mark.parametrize("layers,keep,generic", [([128, 64, 32], 0.5, False), ([128, 64, 32], 0.5, True),
                                                ([64, 32], 1.0, False), ([64, 32], 1.0, True)])
def test_fused_batch_norm_matches_oracle(layers, keep, generic):
    """batch_norm=True on the fused row kernel (batch moments via in-launch grid reductions):
    forward, MLP / γ / β / embedding gradients and the moving-moment updates match the fp32
    oracle with the same bf16 rounding points and dropout masks; inference uses the moving
    moments.  B=192 leaves 4 all-padding workgroups in the grid.  Both the compile-time-shape
    kernel (PS:316-338 batch_norm on the fast path) and the runtime-shape one."""
    dev = torch.device("cuda")
    spec = _bn_spec(layers, keep)
    B, K = 192, 10
    P = _bn_params(spec, 7)
    eng = FusedDeepFM(spec, OptHParams(name="GD", lr=1.0), B, dev, params=P, use_graph=False,
                      force_generic_kernels=generic)
    assert eng.H.deepfm_rows_static(eng.rows_params[0]) == (not generic)
    assert eng.H.deepfm_rows_tile(eng.rows_params[0]) == 16
    gen = torch.Generator().manual_seed(2)
    ids, vals, labels = _batch(B, 39, 5000, gen)
    emb, lays, w_out, b_out, fmb, masks = _ref_inputs(eng, spec, 0, spec.keep_probs)
    bn = [{"gamma": P[f"Deep-part/bn_{i}/gamma"], "beta": P[f"Deep-part/bn_{i}/beta"]} for i in range(len(layers))]
    before = eng.parameters_tf()
    eng.load_batch(ids.to(dev), vals.to(dev), labels.to(dev))
    eng.train_step()
    torch.cuda.synchronize()
    eng.check()
    ref = R.fused_step_reference(emb, lays, w_out, b_out, fmb, ids, vals, labels, K, spec.keep_probs, masks,
                                 1.0 / B, train=True, bn=bn)
    # BN rescales each column to unit variance, so a 1-ulp bf16 flip of an activation (f32
    # accumulation order differs between MFMA and the oracle) moves outputs more than without BN:
    # compare by relative norm, which a wrong moment / gradient formula would miss by far
    errs = {"prob": _rel(eng.prob[:B].cpu(), ref["prob"])}
    after = eng.parameters_tf()
    for l in range(len(layers)):
        for name, key in ((f"mlp{l}/weights", "dW"), (f"mlp{l}/biases", "db"), (f"bn_{l}/gamma", "dgamma"),
                          (f"bn_{l}/beta", "dbeta")):
            d = before[f"Deep-part/{name}"] - after[f"Deep-part/{name}"]
            errs[name] = _rel(d, ref[key][l])
        mm = 0.9 * before[f"Deep-part/bn_{l}/moving_mean"] + 0.1 * ref["bn_mean"][l]
        mv = 0.9 * before[f"Deep-part/bn_{l}/moving_variance"] + 0.1 * ref["bn_var"][l] * B / (B - 1)
        torch.testing.assert_close(after[f"Deep-part/bn_{l}/moving_mean"], mm, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(after[f"Deep-part/bn_{l}/moving_variance"], mv, rtol=1e-4, atol=1e-5)
    uniq, acc = R.emb_grad_reference(ids, ref["contrib"])
    delta = emb[:, : K + 1] - eng.emb.detach().cpu()[:, : K + 1]
    errs["emb"] = _rel(delta[uniq], acc + spec.l2_reg * emb[uniq, : K + 1])
    bad = {k: v for k, v in errs.items() if not v < 2e-2}
    assert not bad, f"relative errors vs the oracle: {errs}"
    # inference: the moving moments, no dropout
    emb2, lays2, w2, b2, f2, _ = _ref_inputs(eng, spec, 0, [1.0] * len(layers))
    bn2 = [{"gamma": after[f"Deep-part/bn_{i}/gamma"], "beta": after[f"Deep-part/bn_{i}/beta"],
            "mean": after[f"Deep-part/bn_{i}/moving_mean"], "var": after[f"Deep-part/bn_{i}/moving_variance"]}
           for i in range(len(layers))]
    prob, _ = eng.predict_batch(ids[:100].to(dev), vals[:100].to(dev))
    ref2 = R.fused_step_reference(emb2, lays2, w2, b2, f2, ids[:100], vals[:100], labels[:100], K,
                                  [1.0] * len(layers), None, 1.0 / 100, train=False, bn=bn2)
    assert _rel(prob.cpu(), ref2["prob"]) < 2e-3


@pytest.mark.parametrize("layers", [[64, 32], [128, 64, 32]])
def test_fused_batch_norm_multistep_graph_equals_per_step(layers):
    """Grid-barrier counters reset between launches: multi-step graph replays of the batch-norm
    row kernel train bit-identically to per-step eager launches."""
    spec = _bn_spec(layers, 0.7)
    g = torch.Generator().manual_seed(4)
    pool = [_batch(128, 39, 5000, g) for _ in range(5)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    hp = OptHParams(name="Adam", lr=2e-3)
    a = FusedDeepFM(spec, hp, 128, "cuda", params=_bn_params(spec, 3), use_graph=True)
    b = FusedDeepFM(spec, hp, 128, "cuda", params=_bn_params(spec, 3), use_graph=False)
    a.attach_pool(ids, vals, labels)
    b.attach_pool(ids, vals, labels)
    a.train_steps(21, 8)
    for _ in range(21):
        b.train_step()
    torch.cuda.synchronize()
    a.check()
    b.check()
    assert torch.equal(a.dense, b.dense) and torch.equal(a.emb, b.emb) and torch.equal(a.bn_stats, b.bn_stats)


@pytest.mark.parametrize("update", ["sparse", "exact"])
@pytest.mark.parametrize("opt", ["Adam", "Adagrad", "Momentum", "ftrl", "GD"])
def test_fused_optimizers_match_tf_formulas(opt, update):
    """Every HIP optimizer (MLP dense apply inside the step tail, embedding row update, exact-mode
    full-table update) against optim/tf_optim.py over two steps.  Each step's gradients come from
    a GD(lr=1) engine started from the optimizer engine's current variables; the TF formula is
    then applied to the variables and slots read back from the optimizer engine."""
    from rocfm.optim import apply_dense, slot_names

    dev = torch.device("cuda")
    V, F, K, B = 3000, 39, 10, 128
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=1e-3)
    hp = OptHParams(name=opt, lr=1e-2)
    eng = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 21), use_graph=False, embedding_update=update)
    gen = torch.Generator().manual_seed(4)
    batches = [_batch(B, F, V, gen) for _ in range(2)]
    names = slot_names(opt)
    # g is recovered as (θ − θ_GD) / 1024 from a GD(lr = 1024) step: the f32 rounding of θ_GD then
    # costs ≈ ulp(θ)/1024 of g.  Adam / Adagrad / FTRL normalise by |g|, so elements with tiny |g|
    # may still move by a slightly different fraction of lr: 0.5 % of one step is allowed
    # (a wrong formula term is off by ≫ 1 %)
    glr = 1024.0
    atol = 5e-3 * hp.lr if opt in ("Adam", "Adagrad", "ftrl") else 2e-6
    for step, (ids, vals, labels) in enumerate(batches, start=1):
        sd0 = eng.state_dict()
        params0 = {k: v for k, v in sd0.items() if "/" not in k or k.startswith("Deep-part/")}
        params0 = {k: v for k, v in params0.items() if not any(k.endswith("/" + n) for n in names)}
        params0.pop("global_step", None)
        params0.pop("beta1_power", None)
        params0.pop("beta2_power", None)
        gd = FusedDeepFM(spec, OptHParams(name="GD", lr=glr), B, dev, params=params0, use_graph=False,
                         embedding_update=update)
        for e in (gd, eng):
            e.load_batch(ids.to(dev), vals.to(dev), labels.to(dev))
            e.train_step()
        torch.cuda.synchronize()
        gdp = gd.parameters_tf()
        got = eng.state_dict()
        for name, p0 in params0.items():
            g = (p0 - gdp[name]) / glr  # this step's gradient (incl. the lazy / dense L2 term of the tables)
            p = p0.clone()
            slots = [sd0[f"{name}/{n}"].clone() for n in names]
            if name in ("fm_v", "fm_w") and update == "sparse":
                rows = torch.unique(ids.long())
                pr, sr = p[rows], [t[rows] for t in slots]
                apply_dense(hp, pr, g[rows], sr, step)
                p[rows] = pr
                for t, tr in zip(slots, sr):
                    t[rows] = tr
            else:
                apply_dense(hp, p, g, slots, step)
            torch.testing.assert_close(got[name], p, rtol=2e-4, atol=atol, msg=lambda m: f"{opt} {name}: {m}")
            for n, t in zip(names, slots):
                torch.testing.assert_close(got[f"{name}/{n}"], t, rtol=2e-3, atol=max(atol, 1e-6),
                                           msg=lambda m: f"{opt} {name}/{n}: {m}")


def test_device_id_guard(monkeypatch):
    """ROCFM_CHECK_IDS=1: out-of-range ids are caught on the device (sticky flag; fetched as row 0
    so no kernel reads outside the table) and check() raises; in-range batches pass."""
    monkeypatch.setenv("ROCFM_CHECK_IDS", "1")
    dev = torch.device("cuda")
    V, F, K, B = 1000, 39, 10, 128
    spec = ModelSpec(feature_size=V, field_size=F, embedding_size=K, layers=[64, 32], keep_probs=[1.0, 1.0])
    gen = torch.Generator().manual_seed(2)
    good = [_batch(B, F, V, gen) for _ in range(4)]
    bad = [tuple(t.clone() for t in b) for b in good]
    bad[2][0][5, 7] = V + 12345
    bad[3][0][9, 3] = -4
    for batches, should_fail in ((good, False), (bad, True)):
        eng = FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, dev, params=init_params(spec, 1))
        eng.attach_pool(*[torch.stack([b[i] for b in batches]).to(dev) for i in range(3)])
        eng.train_steps(8, 4)
        torch.cuda.synchronize()
        if should_fail:
            with pytest.raises(ValueError, match="ROCFM_CHECK_IDS"):
                eng.check()
        else:
            eng.check()
        assert torch.isfinite(eng.emb).all()


@pytest.mark.parametrize("K,layers,dtype,generic", [(10, [128, 64, 32], "bf16", False), (32, [128, 64, 32], "bf16", False),
                                                    (10, [128, 64, 32], "fp8", False), (10, [64, 32], "bf16", False),
                                                    (10, [128, 64, 32], "bf16", True), (32, [256, 128, 64], "bf16", False)])
def test_row_tile_8_equals_16(K, layers, dtype, generic, monkeypatch):
    """8 or 4 examples per row-kernel workgroup (2× / 4× the workgroups) computes every valid row
    with the same arithmetic as 16 (padding rows of the MFMA tile are zero and never stored): Adam
    + dropout through multi-step graphs, a batch that is not a multiple of 16 — bitwise equal.
    The runtime-shape kernel (generic, or the reference's 256-128-64 default) takes 16 and 8."""
    monkeypatch.setenv("ROCFM_DEDUP", "0")  # (dedup groups depend on the row tile: test_dedup_*)
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=K, layers=layers,
                     keep_probs=[0.7] * len(layers), l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=2e-3)
    g = torch.Generator().manual_seed(21)
    B = 200
    pool = [_batch(B, 39, 3000, g) for _ in range(5)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    out = {}
    tiles = (16, 8) if (generic or layers[0] > 128) else (16, 8, 4)
    for rt in tiles:
        monkeypatch.setenv("ROCFM_ROW_TILE", str(rt))
        e = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True, compute_dtype=dtype,
                        force_generic_kernels=generic)
        assert e.H.deepfm_rows_tile(e.rows_params[0]) == rt
        e.attach_pool(ids, vals, labels)
        e.train_steps(13, 4)
        torch.cuda.synchronize()
        e.check()
        out[rt] = (e.emb.clone(), e.dense.clone(), [s.clone() for s in e.emb_slots], e.prob[:B].clone())
    a = out[16]
    for rt in tiles[1:]:
        b = out[rt]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[3], b[3]), rt
        assert all(torch.equal(x, y) for x, y in zip(a[2], b[2])), rt


def _dedup_ref(ids_sorted, pos_sorted, F, rt):
    """numpy reference of the per-tile dedup of one sorted batch."""
    n = len(ids_sorted)
    tile = (pos_sorted // F) // rt
    head = np.ones(n, bool)
    head[1:] = (ids_sorted[1:] != ids_sorted[:-1]) | (tile[1:] != tile[:-1])
    c = np.cumsum(head) - 1
    pos = np.zeros(n, np.int64)
    nxt = np.full(n, -1, np.int64)
    pos[pos_sorted] = np.where(head, c, ~c)
    more = np.zeros(n, bool)
    more[:-1] = ~head[1:]
    nxt[pos_sorted[:-1][more[:-1]]] = pos_sorted[1:][more[:-1]]
    return pos, nxt, ids_sorted[head], int(head.sum())


@pytest.mark.parametrize("rt,chunk", [(8, 512), (16, 256), (4, 512)])
def test_dedup_kernel_matches_reference(rt, chunk):
    """batch.hip dedup: group index / next-member links / compacted keys / count / per-chunk run
    ends and run heads of a sorted batch with hot ids (fixed ids in every row, a hot id in two
    fields of one row) equal a numpy reference."""
    from rocfm.ops import require_hip

    H = require_hip()
    B, F, V = 300, 39, 5000
    g = torch.Generator().manual_seed(rt)
    ids, _, _ = _batch(B, F, V, g)
    ids[:, 20] = ids[:, 21]  # the same id twice in one row
    n = B * F
    dev = torch.device("cuda")
    flat = ids.reshape(-1).cuda()
    sk, sv = torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev)
    temp = torch.zeros(max(H.sort_pairs_temp_bytes(n, 13), 16), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    H.sort_pairs_iota(temp.data_ptr(), temp.numel(), flat.data_ptr(), sk.data_ptr(), sv.data_ptr(), n, 13, s)
    nch = (n + chunk - 1) // chunk
    out = {k: torch.full((n,), -7, dtype=torch.int32, device=dev) for k in ("pos", "nxt", "ck")}
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    cend, chd = (torch.zeros(nch, dtype=torch.int32, device=dev) for _ in range(2))
    bc = torch.zeros(H.dedup_scratch_ints(n, 1), dtype=torch.int32, device=dev)
    d = H.DedupParams()
    d.skeys, d.svals, d.n, d.S, d.F, d.rt, d.val_base_step = sk.data_ptr(), sv.data_ptr(), n, 1, F, rt, 0
    d.pos, d.nxt, d.ckeys = out["pos"].data_ptr(), out["nxt"].data_ptr(), out["ck"].data_ptr()
    d.count, d.bcount, d.chunk = cnt.data_ptr(), bc.data_ptr(), chunk
    d.chunk_end, d.chunk_heads = cend.data_ptr(), chd.data_ptr()
    H.dedup(d, s)
    torch.cuda.synchronize()
    pos, nxt, ck, c = _dedup_ref(sk.cpu().numpy().astype(np.int64), sv.cpu().numpy().astype(np.int64), F, rt)
    assert int(cnt.item()) == c
    np.testing.assert_array_equal(out["pos"].cpu().numpy(), pos)
    np.testing.assert_array_equal(out["nxt"].cpu().numpy(), nxt)
    np.testing.assert_array_equal(out["ck"].cpu().numpy()[:c], ck)
    for j in range(nch):  # run end of each compacted chunk's last run, run heads per chunk
        lo = j * chunk
        if lo >= c:
            assert int(cend[j]) == c
            continue
        last = min(lo + chunk, c) - 1
        e = last + 1
        while e < c and ck[e] == ck[last]:
            e += 1
        assert int(cend[j]) == e, j
        seg = ck[lo:min(lo + chunk, c)]
        heads = sum(1 for i in range(lo, min(lo + chunk, c)) if i == 0 or ck[i] != ck[i - 1])
        assert int(chd[j]) == heads, (j, seg[:4])


@pytest.mark.parametrize("rt", ["8", "16"])
@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_dedup_equals_no_dedup(rt, update, monkeypatch):
    """Per-tile dedup changes only the summation order of each id's gradient rows: with Momentum
    every element matches the un-deduplicated engine to fp32 reorder bounds, and the multi-step
    graphs equal the per-step launches bitwise (both dedup)."""
    monkeypatch.setenv("ROCFM_ROW_TILE", rt)
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=10, layers=[128, 64, 32],
                     keep_probs=[0.8] * 3, l2_reg=1e-3)
    hp = OptHParams(name="Momentum", lr=0.02)
    g = torch.Generator().manual_seed(5)
    B = 256
    pool = [_batch(B, 39, 3000, g) for _ in range(5)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    out = {}
    for dd, graphs in ((False, True), (True, True), (True, False)):
        e = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=graphs, embedding_update=update,
                        dedup=dd)
        assert e.dedup == dd
        e.attach_pool(ids, vals, labels)
        if graphs:
            e.train_steps(13, 4)
        else:
            for _ in range(13):
                e.train_step()
        torch.cuda.synchronize()
        e.check()
        out[(dd, graphs)] = (e.emb.clone(), e.dense.clone(), [x.clone() for x in e.emb_slots])
    a, b, c = out[(False, True)], out[(True, True)], out[(True, False)]
    assert torch.equal(b[0], c[0]) and torch.equal(b[1], c[1])
    for x, y in [(a[0], b[0]), (a[1], b[1])] + list(zip(a[2], b[2])):
        d = (x - y).abs()
        assert bool((d <= 1e-7 + 1e-5 * y.abs()).all()), d.max().item()


@pytest.mark.parametrize("W,mode", [(2, 0), (3, 1), (8, 0)])
def test_merge_range_equals_search(W, mode):
    """merge.hip range mode (bucket directories, LDS-staged matching; one bucket holds more
    entries than the LDS stage and takes the global-search fallback) sums every key's rows in the
    search mode's rank order: the dense-gradient rows (mode 1) are bitwise equal; after the Adam
    update (mode 0) the two kernels' instruction selection may differ in the last bit."""
    from rocfm.ops import require_hip
    from rocfm.parallel.dp import range_merge_buckets

    H = require_hip()
    dev = torch.device("cuda")
    V, Kp = 2_000_000, 12
    g = torch.Generator().manual_seed(W)
    lists = []
    for r in range(W):
        hot = torch.arange(0, 600)  # bucket 0 crowded in every rank (> the LDS stage in total)
        rnd = torch.randint(0, V, (3000 + 500 * r,), generator=g)
        lists.append(torch.unique(torch.cat([hot, rnd])))
    cap = (max(len(x) for x in lists) + 3) // 4 * 4
    keys = torch.full((W, cap), -1, dtype=torch.int32)
    for r, x in enumerate(lists):
        keys[r, : len(x)] = x.to(torch.int32)
    keys = keys.to(dev)
    counts = torch.tensor([len(x) for x in lists], dtype=torch.int32, device=dev)
    rows = torch.randn(W, cap, Kp, generator=g).to(dev)
    nb = range_merge_buckets(W, cap)
    div = (V + nb - 1) // nb
    dirs = torch.stack([torch.searchsorted(x, torch.arange(nb + 1) * div).to(torch.int32) for x in lists]).to(dev)
    assert int((dirs[:, 1] - dirs[:, 0]).sum()) > H.merge_range_lds_entries(Kp)  # the fallback bucket
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    outs = []
    for rng in (False, True):
        emb = torch.randn(V, Kp, generator=torch.Generator().manual_seed(1)).to(dev)
        s0, s1 = torch.zeros_like(emb), torch.zeros_like(emb)
        dg, touched = torch.zeros_like(emb), torch.zeros(V, dtype=torch.int32, device=dev)
        p = H.MergeParams()
        p.keys, p.key_stride, p.rows, p.row_stride = keys.data_ptr(), cap, rows.data_ptr(), cap * Kp
        p.counts, p.count_stride = counts.data_ptr(), 1
        p.W, p.cap, p.Kp, p.K1, p.key_div, p.Vmap = W, cap, Kp, Kp - 1, 1, V
        p.emb, p.s0, p.s1, p.l2, p.grad_scale = emb.data_ptr(), s0.data_ptr(), s1.data_ptr(), 1e-3, 1.0 / W
        o = H.OptParams()
        o.type, o.lr, o.beta1, o.beta2, o.eps = 0, 1e-3, 0.9, 0.999, 1e-8  # Adam
        lrt = torch.full((1,), 1e-3, device=dev)
        o.lrt = lrt.data_ptr()
        p.opt, p.step, p.mode = o, step.data_ptr(), mode
        p.dense_grad, p.touched = dg.data_ptr(), touched.data_ptr()
        p.dirs, p.dir_stride, p.nb, p.bucket_div = dirs.data_ptr(), nb + 1, nb, div
        s = torch.cuda.current_stream().cuda_stream
        if rng:
            H.merge_range_apply(p, None, s)
        else:
            H.merge_search_apply(p, None, s)
        torch.cuda.synchronize()
        outs.append((emb.cpu(), s0.cpu(), s1.cpu(), dg.cpu(), touched.cpu()))
    for a, b in zip(*outs):
        if mode == 1:
            assert torch.equal(a, b)
        else:
            assert bool(((a.float() - b.float()).abs() <= 1e-6 * b.float().abs() + 1e-9).all())


@pytest.mark.parametrize("dedup", [False, True])
def test_wide_static_kernel_equals_runtime_shape(dedup, monkeypatch):
    """The reference's flag defaults (k=32, 256-128-64; PS:52,62) run a compile-time-shape row
    kernel whose layer-0 forward streams two tiles per wave through one tile's registers and whose
    layer-1 backward owns two tiles per wave.  Its k-order per tile is the runtime-shape kernel's,
    so Adam + dropout through multi-step graphs match it to fp32 reorder bounds (dedup: the
    per-tile gradient-row sums, which only the static kernel's LDS has room for at this shape)."""
    monkeypatch.setenv("ROCFM_DEDUP", "1" if dedup else "0")
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=32, layers=[256, 128, 64],
                     keep_probs=[0.7] * 3, l2_reg=1e-3)
    hp = OptHParams(name="Momentum", lr=0.02)
    g = torch.Generator().manual_seed(33)
    B = 200
    pool = [_batch(B, 39, 3000, g) for _ in range(5)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    out = {}
    for generic in (True, False):
        e = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True,
                        force_generic_kernels=generic)
        assert e.dedup == (dedup and not generic)
        e.attach_pool(ids, vals, labels)
        e.train_steps(13, 4)
        torch.cuda.synchronize()
        e.check()
        out[generic] = (e.emb.clone(), e.dense.clone(), e.prob[:B].clone())
    for x, y in zip(out[True], out[False]):
        d = (x - y).abs()
        assert bool((d <= 1e-6 + 1e-4 * y.abs()).all()), d.max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("tbl,graph", [("f32", True), ("bf16", True), ("f32", False)])
def test_row_split_equals_unsplit(tbl, graph, monkeypatch):
    """The row-tile split (ROCFM_ROW_SPLIT=2: two workgroups per 8-row tile, each streaming half of
    W0 and computing its half of layer 0's outputs and its fields' dgrad, with an in-launch exchange
    of the outputs) ≡ one workgroup per tile, bitwise: the reference's flag-default shape (39 × 32 →
    256-128-64), Adam + dropout, a batch that is not a multiple of 8, multi-step graphs and per-step
    launches, f32 and bf16 tables; the exchange's error word stays clear."""
    monkeypatch.setenv("ROCFM_DEDUP", "0")
    spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=32, layers=[256, 128, 64],
                     keep_probs=[0.7] * 3, l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=2e-3)
    g = torch.Generator().manual_seed(5)
    B = 200
    pool = [_batch(B, 39, 3000, g) for _ in range(5)]
    ids, vals, labels = (torch.stack([p[i] for p in pool]).cuda() for i in range(3))
    out = {}
    for split in ("1", "2"):
        monkeypatch.setenv("ROCFM_ROW_SPLIT", split)
        e = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=graph, table_dtype=tbl)
        assert e.H.deepfm_rows_split(e.rows_params[0]) == int(split)
        e.attach_pool(ids, vals, labels)
        if graph:
            e.train_steps(13, 4)
        else:
            for _ in range(7):
                e.train_step()
        torch.cuda.synchronize()
        e.check()
        out[split] = (e.emb.clone(), e.dense.clone(), [s.clone() for s in e.emb_slots], e.prob[:B].clone())
    a, b = out["1"], out["2"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[3], b[3])
    assert all(torch.equal(x, y) for x, y in zip(a[2], b[2]))
