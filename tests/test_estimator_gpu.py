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


@pytest.mark.parametrize("par", ["auto", "rowshard"])
def test_fused_estimator_end_to_end(data_dir, tmp_path, par):
    from rocfm import checkpoint as ckpt
    from rocfm.estimator import Estimator
    from rocfm.serving import Predictor

    md = str(tmp_path / "m")
    est = Estimator(_cfg(data_dir, md, parallelism=par))
    ev0 = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    out = est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=2)
    assert out["steps"] == 2 * (8192 // 512)
    ev = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    assert ev["loss"] < ev0["loss"] and ev["auc_exact"] > 0.65
    assert abs(ev["auc"] - ev["auc_exact"]) < 0.02 and ev["examples"] == 2048
    prefix = ckpt.latest_checkpoint(md)
    assert ckpt.checkpoint_step(prefix) == est.global_step
    b = Estimator(_cfg(data_dir, md, parallelism=par))
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
