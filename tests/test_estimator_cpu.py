"""End-to-end Estimator on CPU (BASELINE config 1 plumbing): train on a synthetic train file +
the bundled val file's schema, evaluate, checkpoint/resume bit-exactness, export, pred.txt."""
import json
import os

import numpy as np
import pytest
import torch

from rocfm import checkpoint as ckpt
from rocfm.config import parse_flags
from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.estimator import Estimator


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("data")
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 6000, 2000, seed=1)
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 1500, 2000, seed=2)
    write_synthetic_tfrecord(str(d / "te.tfrecords"), 700, 2000, seed=3)
    return str(d)


def _cfg(data_dir, model_dir, **kw):
    argv = ["--feature_size", "2000", "--field_size", "39", "--embedding_size", "8", "--deep_layers", "32,16",
            "--dropout", "1.0,1.0", "--batch_size", "256", "--learning_rate", "0.005", "--l2_reg", "0.00001",
            "--training_data_dir", data_dir, "--val_data_dir", data_dir, "--model_dir", model_dir,
            "--log_steps", "5", "--engine", "torch", "--num_threads", "2", "--save_checkpoints_secs", "0"]
    for k, v in kw.items():
        argv += [f"--{k}", str(v)]
    return parse_flags(argv)


def test_train_eval_checkpoint_export(data_dir, tmp_path):
    md = str(tmp_path / "m")
    est = Estimator(_cfg(data_dir, md))
    ev0 = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    out = est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=2)
    assert out["steps"] == 2 * (6000 // 256)
    ev1 = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    assert ev1["loss"] < ev0["loss"] and ev1["auc_exact"] > 0.7 and abs(ev1["auc"] - ev1["auc_exact"]) < 0.02
    assert ev1["examples"] == (1500 // 256) * 256  # drop_remainder on eval too (reference input_fn)
    prefix = ckpt.latest_checkpoint(md)
    assert prefix and ckpt.checkpoint_step(prefix) == est.global_step
    sd = ckpt.load_checkpoint(prefix)
    assert "fm_v/Adam" in sd and "Deep-part/mlp0/weights/Adam_1" in sd and int(sd["global_step"]) == est.global_step
    # resume: a fresh estimator restores the checkpoint and continues bit-exactly
    a = Estimator(_cfg(data_dir, md))
    assert a.global_step == est.global_step
    b_sd = est.state_dict()
    for k, v in a.state_dict().items():
        assert torch.equal(v, b_sd[k]), k
    # export + servable predictions == estimator predictions
    exp = est.export(str(tmp_path / "export"))
    meta = json.load(open(os.path.join(exp, "model.json")))
    assert meta["signatures"]["serving_default"]["inputs"]["feat_ids"]["shape"] == [None, 39]
    from rocfm.serving import Predictor

    pr = Predictor(str(tmp_path / "export"))
    from rocfm.data.tfrecord import decode_file

    L, I, V = decode_file(os.path.join(data_dir, "te.tfrecords"), 39)
    p_est = est.predict([os.path.join(data_dir, "te.tfrecords")], str(tmp_path / "pred.txt"))
    p_srv = pr.predict(I[: len(p_est)], V[: len(p_est)])
    torch.testing.assert_close(p_srv, p_est, rtol=1e-5, atol=1e-6)
    lines = open(tmp_path / "pred.txt").read().splitlines()
    assert len(lines) == (700 // 256) * 256 and all(len(x.split(".")[1]) == 6 for x in lines)


def test_keep_checkpoint_max(tmp_path):
    md = str(tmp_path / "k")
    sd = {"w": torch.zeros(3)}
    for s in range(1, 9):
        ckpt.save_checkpoint(md, sd, s, keep_max=3)
    assert ckpt.list_checkpoints(md) == ["model.ckpt-6", "model.ckpt-7", "model.ckpt-8"]
    assert not any(f.startswith("model.ckpt-5.") for f in os.listdir(md))


def test_sharded_checkpoint_reshard(tmp_path):
    md = str(tmp_path / "s")
    full = torch.arange(40, dtype=torch.float32).view(10, 4)
    for r in range(2):  # 2 shards, id % 2 == r
        rows = torch.arange(r, 10, 2)
        ckpt.save_checkpoint(md, {"fm_v": full[rows]}, 7, shard=(r, 2), row_sets={"fm_v": rows},
                             write_index=(r == 0), global_rows={"fm_v": 10})
    p = ckpt.latest_checkpoint(md)
    assert torch.equal(ckpt.load_checkpoint(p)["fm_v"], full)
    sub = ckpt.load_checkpoint(p, rows_for={"fm_v": torch.tensor([9, 0, 4])})["fm_v"]
    assert torch.equal(sub, full[[9, 0, 4]])


def test_cli_train_infer(data_dir, tmp_path):
    from rocfm.cli import run

    md = str(tmp_path / "cli")
    cfg = _cfg(data_dir, md, num_epochs=1, servable_model_dir=str(tmp_path / "exp"), task_type="train")
    res = run(cfg)
    assert res["epochs"][0]["eval_auc"] > 0.6 and os.path.isdir(res["export"])
    res = run(_cfg(data_dir, md, task_type="infer"))
    assert os.path.exists(os.path.join(data_dir, "pred.txt")) and res["infer"]["n"] == 512
    os.remove(os.path.join(data_dir, "pred.txt"))


def test_sagemaker_pipe_mode_channels(data_dir, tmp_path, monkeypatch):
    """pipe_mode=1: channels bound from SM_CHANNELS (evaluation = channels[0], training =
    channels[1 + local_rank], HVD:420-445), one FIFO per channel and epoch under
    SM_INPUT_DIR/data/<channel>_<epoch> (PipeModeDataset), streamed by writer threads."""
    import threading

    from rocfm.cli import run

    base = tmp_path / "input"
    (base / "data").mkdir(parents=True)
    monkeypatch.setenv("SM_INPUT_DIR", str(base))
    monkeypatch.setenv("SM_CHANNELS", json.dumps(["evaluation", "training", "training-1"]))
    src = {"training": os.path.join(data_dir, "tr.tfrecords"), "evaluation": os.path.join(data_dir, "va.tfrecords")}
    fifos = [("training", 0), ("training", 1), ("evaluation", 0)]
    writers = []
    for ch, ep in fifos:
        path = str(base / "data" / f"{ch}_{ep}")
        os.mkfifo(path)

        def feed(path=path, ch=ch):
            with open(path, "wb") as w, open(src[ch], "rb") as r:  # open blocks until the reader opens
                w.write(r.read())

        t = threading.Thread(target=feed, daemon=True)
        t.start()
        writers.append(t)
    cfg = _cfg(data_dir, str(tmp_path / "m"), pipe_mode=1, num_epochs=2)
    out = run(cfg)
    for t in writers:
        t.join(timeout=30)
        assert not t.is_alive()
    assert out["channels"]["train"] == [str(base / "data" / "training_0"), str(base / "data" / "training_1")]
    assert out["channels"]["eval"] == [str(base / "data" / "evaluation_0")]
    assert out["train"]["steps"] == 2 * (6000 // 256)
    assert out["eval"]["examples"] == (1500 // 256) * 256


def test_tensorboard_event_files(data_dir, tmp_path):
    """Estimator summaries: TF event files in model_dir (train) and model_dir/eval, readable back
    (TFRecord framing with valid CRCs, Event/Summary protobuf encoding)."""
    import glob

    from rocfm.utils.tensorboard import encode_event, frame, read_scalars

    md = str(tmp_path / "m")
    est = Estimator(_cfg(data_dir, md))
    est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=1)
    res = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    est.close()
    tr = glob.glob(os.path.join(md, "events.out.tfevents.*"))
    ev = glob.glob(os.path.join(md, "eval", "events.out.tfevents.*"))
    assert len(tr) == 1 and len(ev) == 1
    s = read_scalars(tr[0])
    losses = [(st, v) for st, tag, v in s if tag == "loss"]
    assert [st for st, _ in losses] == list(range(5, 6000 // 256 + 1, 5))
    assert all(np.isfinite(v) for _, v in losses)
    assert {"global_step/sec", "examples/sec"} <= {tag for _, tag, _ in s}
    e = {tag: v for _, tag, v in read_scalars(ev[0])}
    assert abs(e["auc"] - res["auc"]) < 1e-6 and abs(e["loss"] - res["loss"]) < 1e-5
    # byte-level encoding of one event (field numbers / wire types of tensorflow.Event)
    b = encode_event(1.5, 7, {"x": 2.0})
    assert b == (b"\x09" + np.float64(1.5).tobytes() + b"\x10\x07" + b"\x2a\x0a\x0a\x08\x0a\x01x\x15"
                 + np.float32(2.0).tobytes())
    assert len(frame(b)) == len(b) + 16


def test_fused_only_options_fail_loudly_on_the_torch_engine(data_dir, tmp_path):
    """Options only the fused engines implement are refused on the eager engine (not ignored)."""
    for kw in ({"table_dtype": "bf16"}, {"parallelism": "rowshard", "hot_rows": 8},
               {"parallelism": "rowshard", "ps_staleness": 1}):
        with pytest.raises(ValueError):
            Estimator(_cfg(data_dir, str(tmp_path / "m"), **kw))


def test_remaining_steps_is_a_global_target():
    """max_steps counts global steps in both file and pipe mode: a restarted job that restored a
    checkpoint trains only up to it (and not at all once it is reached)."""
    from rocfm.cli import _remaining_steps

    assert _remaining_steps(0, 40) is None
    assert _remaining_steps(100, 40) == 60
    assert _remaining_steps(100, 100) == 0 and _remaining_steps(100, 130) == 0
