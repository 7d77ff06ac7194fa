"""Asynchronous parameter server (rocfm.parallel.async_ps) on CPU over RPC: one worker is the
single-process sparse engine step for step (1 and 2 PS tasks); two workers train asynchronously
(every push applied once, global step = all workers' steps, the gathered state reloads into the
eager engine); the CLI job (1 PS + 2 workers) trains, checkpoints and evaluates."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from rocfm.models.deepfm import ModelSpec, init_params
from rocfm.optim import OptHParams

SPEC = dict(feature_size=3000, field_size=39, embedding_size=8, layers=[32, 16], keep_probs=[0.5, 0.5], l2_reg=1e-3)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(seed, n, B=64):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, SPEC["feature_size"], (B, 39), generator=g)
        ids[:, :5] = torch.arange(1, 6)  # hot ids shared by every example (and every worker)
        out.append((ids, torch.rand(B, 39, generator=g), (torch.rand(B, generator=g) < 0.3).float()))
    return out


def _job(rank, world, port, n_ps, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)  # the reference run below uses one thread too: same reduction order
    from torch.distributed import rpc

    from rocfm.parallel import async_ps as A

    spec = ModelSpec(**SPEC)
    hp = OptHParams(name="Adam", lr=0.01)
    if rank < n_ps:
        A._SHARD = A.ParameterShard(spec, hp, rank, n_ps, seed=11)
        A._rpc_init(A.ps_name(rank), rank, world, 60.0)
        rpc.shutdown()
        return
    w, nw = rank - n_ps, world - n_ps
    A._rpc_init(A.worker_name(w), rank, world, 60.0)
    eng = A.AsyncPSWorker(spec, hp, n_ps, dropout_seed=100 + w)
    losses = [float(eng.train_step(*b)) for b in _batches(7 + w, steps)]
    eng.flush()
    if w == 0:
        while eng.global_step() < nw * steps:  # the other workers' pushes
            import time

            time.sleep(0.02)
        sd = eng.state_dict()
        b = _batches(99, 1)[0]
        p, _ = eng.predict_batch(b[0], b[1], b[2])
        torch.save({"sd": dict(sd), "losses": losses, "pred": p, "step": eng.global_step()}, out)
    rpc.shutdown()


def _run(tmp_path, n_ps, n_workers, steps):
    out = str(tmp_path / "o.pt")
    world = n_ps + n_workers
    mp.start_processes(_job, args=(world, _port(), n_ps, steps, out), nprocs=world, join=True, start_method="spawn")
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("n_ps", [1, 2])
def test_one_worker_equals_sparse_engine(tmp_path, n_ps):
    from rocfm.models.torch_engine import TorchDeepFM

    got = _run(tmp_path, n_ps, 1, 6)
    spec = ModelSpec(**SPEC)
    ref = TorchDeepFM(spec, OptHParams(name="Adam", lr=0.01), params=init_params(spec, 11), dropout_seed=100)
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # (Adam turns reduction-order rounding of near-zero gradients into lr-sized steps)
    try:
        losses = [float(ref.train_step(*b)) for b in _batches(7, 6)]
    finally:
        torch.set_num_threads(nt)
    assert got["losses"] == losses
    assert got["step"] == 6
    sd = ref.state_dict()
    for k, v in sd.items():
        assert torch.equal(got["sd"][k], v), k


def test_two_workers_asynchronous(tmp_path):
    from rocfm.models.torch_engine import TorchDeepFM

    got = _run(tmp_path, 1, 2, 10)
    assert got["step"] == 20  # every push of both workers applied once
    assert int(got["sd"]["global_step"]) == 20
    init = init_params(ModelSpec(**SPEC), 11)
    assert not torch.equal(got["sd"]["fm_v"], init["fm_v"])
    assert all(torch.isfinite(v).all() for v in got["sd"].values())
    # the gathered variables + slots reload into the eager engine and predict the same
    spec = ModelSpec(**SPEC)
    eng = TorchDeepFM(spec, OptHParams(name="Adam", lr=0.01))
    eng.load_state_dict(got["sd"])
    b = _batches(99, 1)[0]
    p, _ = eng.predict_batch(b[0], b[1], b[2])
    torch.testing.assert_close(p, got["pred"])


def test_cli_async_ps_job(tmp_path):
    """torchrun --nproc-per-node 3 -m rocfm.cli --parallelism async_ps --num_ps 1: both workers
    train their file shard, the chief evaluates and writes the final checkpoint."""
    from rocfm import checkpoint as ckpt
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tmp_path / "data"
    d.mkdir()
    write_synthetic_tfrecord(str(d / "tr0.tfrecords"), 640, 2000, seed=1)
    write_synthetic_tfrecord(str(d / "tr1.tfrecords"), 640, 2000, seed=2)
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 256, 2000, seed=3)
    md = tmp_path / "m"
    argv = ["--feature_size", "2000", "--field_size", "39", "--embedding_size", "8", "--deep_layers", "32,16",
            "--dropout", "1.0,1.0", "--batch_size", "64", "--learning_rate", "0.005", "--training_data_dir", str(d),
            "--val_data_dir", str(d), "--model_dir", str(md), "--log_steps", "5", "--num_threads", "2",
            "--save_checkpoints_secs", "0", "--parallelism", "async_ps", "--num_ps", "1", "--num_epochs", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "-m", "rocfm.cli"] + argv
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    prefix = ckpt.latest_checkpoint(str(md))
    assert prefix is not None
    assert ckpt.checkpoint_step(prefix) == 2 * (640 // 64)  # both workers' steps: one shared global step
    sd = ckpt.load_checkpoint(prefix)
    assert int(sd["global_step"]) == 20


def _fail_job(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    torch.set_num_threads(1)
    from torch.distributed import rpc

    from rocfm.config import parse_flags
    from rocfm.parallel import async_ps as A

    cfg = parse_flags(["--feature_size", "3000", "--field_size", "39", "--embedding_size", "8", "--deep_layers",
                       "32,16", "--dropout", "1.0,1.0", "--batch_size", "64", "--parallelism", "async_ps", "--num_ps", "1",
                       "--dist_timeout_s", "120", "--log_steps", "0"])

    def task(est, w, nw):
        if w == 1:
            raise ValueError("injected worker failure")
        A._wait_ps0(lambda: rpc.rpc_sync(A.ps_name(0), A._done_count) >= nw, "the workers", cfg.dist_timeout_s)
        return {}

    try:
        A.run_job(cfg, task_fn=task)
        res = "ok"
    except BaseException as e:  # noqa: BLE001
        res = f"{type(e).__name__}: {e}"
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(res)


def test_a_failing_worker_fails_the_chief_instead_of_hanging(tmp_path):
    """A worker that raises reports to ps0; the chief's wait for every worker raises (well within
    dist_timeout_s) instead of spinning forever, and the failing worker's error propagates."""
    import time

    t0 = time.time()
    mp.start_processes(_fail_job, args=(3, _port(), str(tmp_path)), nprocs=3, join=True, start_method="spawn")
    assert time.time() - t0 < 100
    chief = open(tmp_path / "r1.txt").read()
    worker = open(tmp_path / "r2.txt").read()
    assert "a worker failed" in chief, chief
    assert "injected worker failure" in worker, worker
