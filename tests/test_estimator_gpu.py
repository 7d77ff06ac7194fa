"""Estimator on the GPU with the fused HIP engine: train → evaluate (device AUC histogram) →
checkpoint/restore → predict → export/serve, and the row-shard engine through the same API."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path_factory.mktemp("gdata")
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 8192, 5000, seed=1)
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 2048, 5000, seed=2)
    write_synthetic_tfrecord(str(d / "te.tfrecords"), 1024, 5000, seed=3)
    return str(d)


def _cfg(data_dir, model_dir, **kw):
    from rocfm.config import parse_flags

    argv = ["--feature_size", "5000", "--field_size", "39", "--embedding_size", "10", "--deep_layers", "64,32",
            "--dropout", "0.9,0.9", "--batch_size", "512", "--learning_rate", "0.003", "--l2_reg", "0.00001",
            "--training_data_dir", data_dir, "--val_data_dir", data_dir, "--model_dir", model_dir,
            "--log_steps", "4", "--engine", "fused", "--num_threads", "4", "--save_checkpoints_secs", "0"]
    for k, v in kw.items():
        argv += [f"--{k}", str(v)]
    return parse_flags(argv)


@pytest.mark.parametrize("par", ["auto", "rowshard", "auto+batch_norm"])
def test_fused_estimator_end_to_end(data_dir, tmp_path, par):
    from rocfm import checkpoint as ckpt
    from rocfm.estimator import Estimator
    from rocfm.serving import Predictor

    md = str(tmp_path / "m")
    kw = dict(parallelism=par.split("+")[0])
    if par.endswith("batch_norm"):
        kw["batch_norm"] = "true"
    est = Estimator(_cfg(data_dir, md, **kw))
    assert est.engine_name == "fused"
    ev0 = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    out = est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=2)
    assert out["steps"] == 2 * (8192 // 512)
    ev = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    assert ev["loss"] < ev0["loss"] and ev["auc_exact"] > 0.65
    assert abs(ev["auc"] - ev["auc_exact"]) < 0.02 and ev["examples"] == 2048
    prefix = ckpt.latest_checkpoint(md)
    assert ckpt.checkpoint_step(prefix) == est.global_step
    b = Estimator(_cfg(data_dir, md, **kw))
    assert b.global_step == est.global_step
    evb = b.evaluate([os.path.join(data_dir, "va.tfrecords")])
    assert abs(evb["auc_exact"] - ev["auc_exact"]) < 1e-6
    probs = est.predict([os.path.join(data_dir, "te.tfrecords")], str(tmp_path / "pred.txt"))
    assert len(probs) == 1024 and len(open(tmp_path / "pred.txt").read().splitlines()) == 1024
    exp = est.export(str(tmp_path / "export"))
    pr = Predictor(exp, engine="fused")
    from rocfm.data.tfrecord import decode_file

    _, ids, vals = decode_file(os.path.join(data_dir, "te.tfrecords"), 39, 5000)
    torch.testing.assert_close(pr.predict(ids, vals), probs, rtol=1e-4, atol=1e-5)
    est.close()
    b.close()


def test_streamed_training_equals_per_step_and_resumes(data_dir, tmp_path):
    """Single-GPU Estimator training streams loader groups through multi-step graphs; it trains
    bit-identically to the per-step path (use_hip_graph=false), also when resumed with
    skip_batches, and still writes its loss log lines."""
    import json

    from rocfm.estimator import Estimator

    tr = [os.path.join(data_dir, "tr.tfrecords")]
    mf = str(tmp_path / "metrics.jsonl")
    a = Estimator(_cfg(data_dir, str(tmp_path / "a"), use_hip_graph="true", metrics_file=mf))
    b = Estimator(_cfg(data_dir, "", use_hip_graph="false"))
    c = Estimator(_cfg(data_dir, "", use_hip_graph="true"))
    assert a.train(tr, num_epochs=2, max_steps=21)["steps"] == 21
    assert b.train(tr, num_epochs=2, max_steps=21)["steps"] == 21
    c.train(tr, num_epochs=2, max_steps=5)
    c.train(tr, num_epochs=2, max_steps=16, skip_batches=5)
    sa, sb, sc = a.eng.state_dict(), b.eng.state_dict(), c.eng.state_dict()

    def diff(x, y):
        bad = [k for k in x if not torch.equal(x[k], y[k])]
        return {k: (float((x[k].double() - y[k].double()).abs().max()),
                    int((x[k] != y[k]).sum())) for k in bad}

    assert not diff(sa, sb), diff(sa, sb)
    assert not diff(sa, sc), diff(sa, sc)
    logs = [json.loads(line) for line in open(mf)]
    train = [r for r in logs if r.get("event") == "train"]
    # logged asynchronously after each graph (16 steps, then the 5-step tail) that crosses log_steps=4
    assert [r["global_step"] for r in train] == [16, 21] and all(r["loss"] == r["loss"] for r in train)
    for e in (a, b, c):
        e.close()


def test_hbm_epoch_cache_equals_streaming(data_dir, tmp_path):
    """hbm_cache: epoch 1 streams from the loader into an HBM ring sized for the epoch, epochs 2..
    replay it from HBM through multi-step graphs — bit-identical to streaming every epoch (no
    shuffle: every epoch presents the same batches in the same order, PS:147-165)."""
    import json

    from rocfm.estimator import Estimator

    tr = [os.path.join(data_dir, "tr.tfrecords")]
    mf = str(tmp_path / "metrics.jsonl")
    a = Estimator(_cfg(data_dir, "", hbm_cache="true", metrics_file=mf))
    b = Estimator(_cfg(data_dir, "", hbm_cache="false"))
    ra, rb = a.train(tr, num_epochs=3), b.train(tr, num_epochs=3)
    assert ra["steps"] == rb["steps"] == 3 * (8192 // 512)
    sa, sb = a.eng.state_dict(), b.eng.state_dict()
    bad = [k for k in sa if not torch.equal(sa[k], sb[k])]
    assert not bad, bad
    logs = [json.loads(line) for line in open(mf)]
    assert any(r.get("event") == "hbm_cache" and r["epochs_from_cache"] == 2 for r in logs)
    assert [r["global_step"] for r in logs if r.get("event") == "train"][-1] == 48
    for e in (a, b):
        e.close()


def test_device_decode_equals_host_decode(data_dir, tmp_path):
    """device_decode (default): the loader hands the graphs' copy stream undecoded Example payloads
    and the GPU parses them (csrc/kernels/decode.hip) — bit-identical training to host parsing."""
    from rocfm.estimator import Estimator

    tr = [os.path.join(data_dir, "tr.tfrecords")]
    a = Estimator(_cfg(data_dir, "", device_decode="true", hbm_cache="false"))
    b = Estimator(_cfg(data_dir, "", device_decode="false", hbm_cache="false"))
    assert a.train(tr, num_epochs=2)["steps"] == b.train(tr, num_epochs=2)["steps"] == 32
    sa, sb = a.eng.state_dict(), b.eng.state_dict()
    assert not [k for k in sa if not torch.equal(sa[k], sb[k])]
    for e in (a, b):
        e.close()


def _two_rank_cache_worker(rank, world, port, data_dir, out_path):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), ROCFM_SHADOW_STEPS="3")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from rocfm.estimator import Estimator

    tr = [os.path.join(data_dir, "tr2.tfrecords")]
    res = {}
    for cache in ("true", "false"):
        est = Estimator(_cfg(data_dir, "", hbm_cache=cache, parallelism="dp", batch_size=512),
                        device=torch.device("cuda", 0))  # (both ranks share the box's one GPU)
        out = est.train(tr, num_epochs=3)
        torch.cuda.synchronize()
        sd = est.eng.state_dict()
        res[cache] = (out["steps"], {k: v.cpu() for k, v in sd.items()}, est.eng.shadow.status)
        est.close()
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_hbm_epoch_cache_equals_streaming(tmp_path):
    """World 2 (ranks sharing the GPU, p2p DP, device-side parsing, a 3-step shadow window): the
    ranks agree on a per-epoch batch count (rank 0's shard holds one batch more, dropped every
    epoch), epoch 1 streams into each rank's HBM cache and epochs 2-3 replay it — bit-identical to
    streaming all three epochs from the loader."""
    import torch.multiprocessing as mp

    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path / "data2"
    d.mkdir()
    write_synthetic_tfrecord(str(d / "tr2.tfrecords"), 9215, 5000, seed=5)  # shards 4608 / 4607 → 9 / 8 batches
    out = str(tmp_path / "cache2.pt")
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_two_rank_cache_worker, args=(2, port, str(d), out), nprocs=2, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    (na, sa, sha), (nb, sb, shb) = r["true"], r["false"]
    assert na == nb == 3 * 8 and sha == shb == "ok", (na, nb, sha, shb)
    assert not [k for k in sa if not torch.equal(sa[k], sb[k])]
