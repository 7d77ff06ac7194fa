"""bf16 embedding-table storage (table_dtype="bf16"): the fused kernels read bf16
rows, update them in f32 with stochastic rounding, and keep f32 optimizer slots."""
import pytest
import torch

from rocfm.models.deepfm import ModelSpec, init_params
from rocfm.models.fused import FusedDeepFM
from rocfm.optim import OptHParams

pytestmark = pytest.mark.gpu


def _spec(K=10, V=5003):
    return ModelSpec(feature_size=V, field_size=39, embedding_size=K, layers=[128, 64, 32], keep_probs=[1.0] * 3,
                     l2_reg=1e-4)


def _pool(V, B=256, n=6, seed=3):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (n, B, 39), generator=g, dtype=torch.int64)
    ids[:, :, :13] = torch.arange(1, 14)
    vals = torch.rand(n, B, 39, generator=g)
    labels = (torch.rand(n, B, generator=g) < 0.3).float()
    return ids.to(torch.int32).cuda(), vals.cuda(), labels.cuda()


def _bf16_round(P):
    out = dict(P)
    for k in ("fm_v", "fm_w"):
        out[k] = P[k].to(torch.bfloat16).float()
    return out


@pytest.mark.parametrize("K,generic", [(10, False), (10, True), (32, False)])
def test_bf16_table_forward_equals_f32_on_rounded_table(K, generic):
    """Gathering bf16 rows is exact: predictions equal the f32 engine's on the bf16-rounded table."""
    spec = _spec(K)
    P = init_params(spec, 1)
    hp = OptHParams("Adam", 1e-3)
    a = FusedDeepFM(spec, hp, 256, "cuda", params=P, table_dtype="bf16", use_graph=False,
                    force_generic_kernels=generic)
    b = FusedDeepFM(spec, hp, 256, "cuda", params=_bf16_round(P), use_graph=False, force_generic_kernels=generic)
    assert a.emb.dtype == torch.bfloat16 and a.emb_slots[0].dtype == torch.float32
    ids, vals, _ = _pool(spec.feature_size, n=1)
    pa, _ = a.predict_batch(ids[0], vals[0])
    pb, _ = b.predict_batch(ids[0], vals[0])
    torch.testing.assert_close(pa, pb, rtol=0, atol=0)
    assert abs(a.l2_value() - b.l2_value()) <= 1e-6 * abs(b.l2_value())


@pytest.mark.parametrize("update", ["sparse", "exact"])
def test_bf16_table_training_tracks_f32(update):
    """20 Adam steps: the bf16-table run stays within a few bf16 ulps of the f32 run, is
    reproducible (stochastic rounding hashed from element and step), and saves f32 checkpoints."""
    spec = _spec()
    P = init_params(spec, 2)
    hp = OptHParams("Adam", 1e-3)
    pool = _pool(spec.feature_size)
    runs = []
    for dt in ("bf16", "bf16", "f32"):
        e = FusedDeepFM(spec, hp, 256, "cuda", params=P if dt == "f32" else P, table_dtype=dt,
                        embedding_update=update)
        e.attach_pool(*pool)
        e.train_steps(20, 8)
        torch.cuda.synchronize()
        runs.append((e.parameters_tf(), e.batch_loss()))
    (a, la), (a2, _), (f, lf) = runs
    for k in a:
        torch.testing.assert_close(a[k], a2[k], rtol=0, atol=0)  # reproducible
    assert a["fm_v"].dtype == torch.float32
    dv = (a["fm_v"] - f["fm_v"]).abs()
    # (Adam normalises near-zero gradients, so a few rows whose gradient sign flips under the bf16
    #  forward move by up to 2·lr per step; the bulk stays within bf16 rounding noise)
    print("bf16 vs f32 table: max", dv.max().item(), "mean", dv.mean().item())
    assert dv.max().item() < 2e-2 and dv.mean().item() < 6e-4
    assert abs(la - lf) < 5e-3


def test_bf16_stochastic_rounding_is_unbiased():
    """GD steps far below half a bf16 ulp: round-to-nearest would freeze the rows; stochastic
    rounding moves them by the f32 amount on average."""
    spec = ModelSpec(feature_size=64, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[1.0, 1.0],
                     l2_reg=0.0)
    P = init_params(spec, 5)
    P["fm_v"] = torch.full_like(P["fm_v"], 0.5)  # bf16 ulp at 0.5 is 2^-8 ≈ 3.9e-3
    hp = OptHParams("GD", 2e-3)
    pool = _pool(64, B=256, n=4)
    out = {}
    for dt in ("bf16", "f32"):
        e = FusedDeepFM(spec, hp, 256, "cuda", params=P, table_dtype=dt)
        e.attach_pool(*pool)
        e.train_steps(40, 8)
        torch.cuda.synchronize()
        out[dt] = e.parameters_tf()["fm_v"]
    moved_f32 = (out["f32"] - 0.5).mean().item()
    moved_bf = (out["bf16"] - 0.5).mean().item()
    assert abs(moved_f32) > 1e-4
    assert abs(moved_bf - moved_f32) < 0.2 * abs(moved_f32)


def test_bf16_table_dp_and_rowshard_world1_match_single():
    """The DP merge and the row-shard owner update write bf16 rows with the same stochastic
    rounding.  (fma contraction differs between the merge and the single-GPU update, and a last-bit
    f32 difference can flip a rounding draw, so the runs agree to bf16 precision, not bitwise.)"""
    from rocfm.parallel.dp import FusedDataParallel
    from rocfm.parallel.emb_shard import FusedRowShard

    spec = _spec()
    P = init_params(spec, 4)
    hp = OptHParams("Adam", 1e-3)
    pool = _pool(spec.feature_size)
    ref = FusedDeepFM(spec, hp, 256, "cuda", params=P, table_dtype="bf16")
    ref.attach_pool(*pool)
    ref.train_steps(12, 4)
    exp = ref.parameters_tf()
    for cls in (FusedDataParallel, FusedRowShard):
        eng = cls(spec, hp, 256, torch.device("cuda"), params=P, table_dtype="bf16")
        eng.attach_pool(*pool)
        eng.train_steps(12, 4)
        torch.cuda.synchronize()
        got = eng.parameters_tf()
        for k in exp:
            if k in ("fm_v", "fm_w"):  # a handful of rows diverge (Adam on near-zero gradients)
                d = (got[k] - exp[k]).abs()
                print(cls.__name__, k, "max", d.max().item(), "mean", d.mean().item())
                assert d.max().item() < 1e-2 and d.mean().item() < 1e-4, (cls.__name__, k, d.max(), d.mean())
            else:
                torch.testing.assert_close(got[k], exp[k], rtol=2e-2, atol=2e-3)
