"""Every engine's side/main multi-step graph pairs are free of shared written buffers
(ROCFM_HAZARD=1, rocfm/utils/hazard.py), and an injected shared write is caught."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(opt="Momentum"):
    from rocfm.models.deepfm import ModelSpec
    from rocfm.optim import OptHParams

    spec = ModelSpec(feature_size=4001, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.8, 0.8],
                     l2_reg=1e-3)
    return spec, OptHParams(name=opt, lr=0.01)


def _pool(B=128, n=6, seed=5):
    from rocfm.data.synthetic import SyntheticCriteo

    g = torch.Generator().manual_seed(seed)
    gen = SyntheticCriteo(4001, 39, seed=seed)
    bs = [gen.batch(B, "cpu", g) for _ in range(n)]
    return [torch.stack([b[i] for b in bs]).cuda() for i in range(3)]


def _make(kind):
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.parallel.dp import FusedDataParallel
    from rocfm.parallel.emb_shard import FusedRowShard

    spec, hp = _cfg("Adam" if "adam" in kind else "Momentum")
    P = init_params(spec, 3)
    dev = torch.device("cuda")
    if kind.startswith("single"):
        e = FusedDeepFM(spec, hp, 128, dev, params=P, use_graph=True,
                        embedding_update="exact" if "exact" in kind else "sparse",
                        dedup="dedup" in kind)
        return e, e
    if kind.startswith("dp") or kind.startswith("dense_dp"):
        mode = "dense_dp" if kind.startswith("dense_dp") else "dp"
        e = FusedDataParallel(spec, hp, 128, dev, params=P, mode=mode, use_graph=True,
                              embedding_update="exact" if ("exact" in kind or mode == "dense_dp") else "sparse")
        return e, e.eng
    e = FusedRowShard(spec, hp, 128, dev, params=P, use_graph=True,
                      embedding_update="exact" if "exact" in kind else "sparse",
                      hot_rows=64 if "hot" in kind else 0, staleness=1 if "stale" in kind else 0)
    return e, e.eng


@pytest.mark.parametrize("kind", ["single", "single_exact", "single_dedup_adam", "dp", "dp_exact", "dense_dp",
                                  "rs", "rs_exact_hot", "rs_hot_adam", "rs_stale"])
def test_side_and_main_graphs_share_no_written_buffer(kind, monkeypatch):
    monkeypatch.setenv("ROCFM_HAZARD", "1")
    monkeypatch.setenv("ROCFM_MERGE", "direct")
    drv, eng = _make(kind)
    assert eng._hazard is not None
    drv.attach_pool(*_pool())
    drv.train_steps(13, 4)  # eager pair, two captured parities, the 1-step remainder pair
    torch.cuda.synchronize()
    drv.check()
    assert eng._hazard.checked >= 3
    # the checker saw both chains' launches and the engine's buffers
    names = {n for n, _ in eng._hazard.calls["side"]} | {n for n, _ in eng._hazard.calls["main"]}
    assert {"fetch_multi", "deepfm_rows"} <= names, names


def test_injected_shared_write_is_caught(monkeypatch):
    from rocfm.utils.hazard import HazardError

    monkeypatch.setenv("ROCFM_HAZARD", "1")
    drv, eng = _make("single")
    orig = type(eng)._prepare_multi

    def bad(self, q, advance, stream):
        orig(self, q, advance, stream)
        # a side-chain write into the positions the CONCURRENT main graph reads (parity q)
        self._hazard.note("injected_write", (self.m_pos[q].data_ptr(),))

    monkeypatch.setattr(type(eng), "_prepare_multi", bad)
    drv.attach_pool(*_pool())
    with pytest.raises(HazardError, match=r"injected_write\.arg0 W eng\.m_pos\+0 +<->  deepfm_rows\.contrib_pos R"):
        drv.train_steps(8, 4)
    torch.cuda.synchronize()


@pytest.mark.parametrize("raw", [False, True])
def test_train_stream_three_stream_plan(raw, monkeypatch, tmp_path):
    """The streamed loop's copy (H2D + device parse into the HBM ring), side (fetch + sort of the
    next graph's batches) and main streams, checked for unordered overlapping accesses after every
    graph (utils/hazard.py StreamPlan); a refill that waits one side graph too early
    (ROCFM_HAZARD_INJECT=ring) is caught."""
    from rocfm.data import tfrecord as T
    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.models.deepfm import init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.utils.hazard import HazardError

    monkeypatch.setenv("ROCFM_HAZARD", "1")
    f = str(tmp_path / "tr.tfrecords")
    write_synthetic_tfrecord(f, 128 * 40, 4001, 39, seed=2)
    spec, hp = _cfg("Adam")

    def run():
        e = FusedDeepFM(spec, hp, 128, torch.device("cuda"), params=init_params(spec, 3))
        ds = T.TFRecordDataset([f], 39, 128, 4001, num_threads=2)
        src = ds.raw_groups(4, hold=2) if raw else ds.groups(4, hold=2)
        n = e.train_stream(src, 4, hold=2)
        torch.cuda.synchronize()
        run.observed = e.hazard_observed
        return n

    assert run() == 40
    if not raw:  # the H2D copies into the ring were also observed as torch writes on the copy stream
        assert run.observed >= 30
    monkeypatch.setenv("ROCFM_HAZARD_INJECT", "ring")
    with pytest.raises(HazardError, match="ring"):
        run()
    torch.cuda.synchronize()
    # the copy stream no longer waits for the ring's zero fill on the compute stream (the 1B-row race)
    monkeypatch.setenv("ROCFM_HAZARD_INJECT", "ring_init")
    with pytest.raises(HazardError, match="ring allocation"):
        run()
    torch.cuda.synchronize()
