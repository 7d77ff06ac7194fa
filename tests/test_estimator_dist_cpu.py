"""Multi-rank Estimator on CPU (gloo, 2 ranks): unequal data shards still run in lockstep (agreed
step count), eval/predict are collective for the row-sharded table, sharded checkpoints are written
by every rank and restore on one process (reshard 2 → 1)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _argv(data_dir, model_dir, par):
    return ["--feature_size", "2000", "--field_size", "39", "--embedding_size", "8", "--deep_layers", "32,16",
            "--dropout", "1.0,1.0", "--batch_size", "128", "--learning_rate", "0.005", "--l2_reg", "0.00001",
            "--training_data_dir", data_dir, "--val_data_dir", data_dir, "--model_dir", model_dir,
            "--log_steps", "5", "--engine", "torch", "--num_threads", "2", "--save_checkpoints_secs", "0",
            "--parallelism", par]


def _worker(rank, world, port, data_dir, model_dir, par, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rocfm.config import parse_flags
    from rocfm.estimator import Estimator

    est = Estimator(parse_flags(_argv(data_dir, model_dir, par)))
    tr = est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=1)
    ev = est.evaluate([os.path.join(data_dir, "va.tfrecords")])
    probs = est.predict([os.path.join(data_dir, "te.tfrecords")])
    full = est.eng.parameters_tf()
    os.environ["ROCFM_EXPORT_CHUNK_ROWS"] = "300"  # row-shard export streams 7 gathered ranges
    path = est.export(os.path.join(model_dir, "export"))
    if rank == 0:
        torch.save({"tr": tr, "ev": ev, "probs": probs, "fm_v": full["fm_v"], "step": est.global_step,
                    "full": dict(full), "export": path}, out)
    est.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("par", ["rowshard", "dp"])
def test_estimator_two_ranks(tmp_path, par):
    from rocfm import checkpoint as ckpt
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path / "data"
    d.mkdir()
    # 1700 records → shard sizes 850/850 → 6 batches each; 700 test records → 350 each → 2 + 2 batches
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 1700, 2000, seed=1)
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 600, 2000, seed=2)
    write_synthetic_tfrecord(str(d / "te.tfrecords"), 700, 2000, seed=3)
    md = str(tmp_path / "m")
    out = str(tmp_path / "o.pt")
    mp.start_processes(_worker, args=(2, _port(), str(d), md, par, out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["step"] == 1700 // 2 // 128
    assert got["ev"]["examples"] == 2 * (300 // 128) * 128
    assert len(got["probs"]) == 2 * (350 // 128) * 128
    prefix = ckpt.latest_checkpoint(md)
    assert prefix and ckpt.checkpoint_step(prefix) == got["step"]
    sd = ckpt.load_checkpoint(prefix)  # both shards reassembled (row-shard) or the replicated table (dp)
    torch.testing.assert_close(sd["fm_v"], got["fm_v"])
    # servable export (row-shard: streamed range by range into the bundle) ≡ the gathered variables
    meta, params = ckpt.load_servable(got["export"])
    assert set(params) == set(got["full"])
    for k, v in got["full"].items():
        torch.testing.assert_close(params[k], v.float())
    # a single-process estimator restores it
    from rocfm.config import parse_flags
    from rocfm.estimator import Estimator

    one = Estimator(parse_flags(_argv(str(d), md, "auto")))
    assert one.global_step == got["step"]
    torch.testing.assert_close(one.eng.P["fm_v"], got["fm_v"])


def test_unequal_shards_lockstep(tmp_path):
    """Shards of different length: ranks agree on the shorter count (no hang)."""
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path / "data"
    d.mkdir()
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 1023, 2000, seed=1)  # 512 / 511 records: 4 vs 3 batches
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 300, 2000, seed=2)
    write_synthetic_tfrecord(str(d / "te.tfrecords"), 300, 2000, seed=3)
    out = str(tmp_path / "o.pt")
    mp.start_processes(_worker, args=(2, _port(), str(d), str(tmp_path / "m"), "rowshard", out), nprocs=2,
                       join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    assert got["step"] == 3


def _ckpt_worker(rank, world, port, data_dir, model_dir, out):
    """Time-based checkpoints with skewed rank clocks: rank 1 is slow every step, so each rank's own
    clock would cross save_checkpoints_secs on different steps (deadlock)."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rocfm.config import parse_flags
    from rocfm.estimator import Estimator

    argv = _argv(data_dir, model_dir, "dp")
    i = argv.index("--save_checkpoints_secs")
    argv[i + 1] = "1"
    argv += ["--ckpt_poll_steps", "1", "--keep_checkpoint_max", "100"]
    est = Estimator(parse_flags(argv))
    saved = []
    orig = est._save

    def spy():
        saved.append(est.global_step)
        return orig()

    est._save = spy

    def slow(e, step):
        time.sleep(0.35 if rank == 1 else 0.0)

    est.train([os.path.join(data_dir, "tr.tfrecords")], num_epochs=1, hooks=[slow])
    torch.save(saved, out + f".{rank}")
    est.close()
    dist.barrier()
    dist.destroy_process_group()


def test_time_based_checkpoint_is_collective(tmp_path):
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path / "data"
    d.mkdir()
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 2 * 128 * 8, 2000, seed=1)  # 8 steps per rank
    out = str(tmp_path / "o.pt")
    mp.start_processes(_ckpt_worker, args=(2, _port(), str(d), str(tmp_path / "m"), out), nprocs=2, join=True,
                       start_method="spawn")
    s0, s1 = torch.load(out + ".0"), torch.load(out + ".1")
    assert s0 == s1, (s0, s1)  # every rank saved at the same steps
    assert len(s0) >= 2  # at least one time-based save before the final one


def _resume_worker(rank, world, port, data_dir, model_dir, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rocfm.config import parse_flags
    from rocfm.estimator import Estimator

    est = Estimator(parse_flags(_argv(data_dir, model_dir, "dp")))
    rp = est.resume_point([os.path.join(data_dir, "tr.tfrecords")], 2)
    torch.save({"step": est.global_step, "rp": rp}, out + f".{rank}")
    est.close()
    dist.barrier()
    dist.destroy_process_group()


def test_resume_point_agreed_over_unequal_shards(tmp_path):
    """512 / 511 records at batch 128 → 4 vs 3 batches per epoch; a job restored at step 5 must
    split (epoch, skip) with the agreed count 3 on both ranks: (1, 2)."""
    from rocfm import checkpoint as ckpt
    from rocfm.config import parse_flags
    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.estimator import Estimator

    d = tmp_path / "data"
    d.mkdir()
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 1023, 2000, seed=1)
    md = str(tmp_path / "m")
    one = Estimator(parse_flags(_argv(str(d), md, "auto")))
    sd = one.state_dict()
    sd["global_step"] = torch.tensor(5, dtype=torch.int64)
    ckpt.save_checkpoint(md, sd, 5)
    out = str(tmp_path / "o.pt")
    mp.start_processes(_resume_worker, args=(2, _port(), str(d), md, out), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = torch.load(out + ".0"), torch.load(out + ".1")
    assert r0["step"] == r1["step"] == 5
    assert tuple(r0["rp"]) == tuple(r1["rp"]) == (1, 2)
