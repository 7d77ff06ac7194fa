"""Auxiliary subsystems on CPU: fault injection + restart-and-resume, watchdog, loader CRC policy,
profiler window, numerics / id guards."""
import json
import os
import subprocess
import sys

import pytest
import torch

from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.utils import fault

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def data_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("udata")
    write_synthetic_tfrecord(str(d / "tr.tfrecords"), 2048, 2000, seed=1)
    write_synthetic_tfrecord(str(d / "va.tfrecords"), 512, 2000, seed=2)
    return str(d)


def _cli(data_dir, model_dir, *extra):
    return ["--feature_size", "2000", "--field_size", "39", "--embedding_size", "8", "--deep_layers", "16",
            "--dropout", "1.0", "--batch_size", "128", "--training_data_dir", data_dir, "--val_data_dir", data_dir,
            "--model_dir", model_dir, "--engine", "torch", "--num_threads", "2", "--save_checkpoints_secs", "0",
            "--eval_every_epoch", "False", "--log_steps", "1", "--num_epochs", "1"] + list(extra)


def _run(args, env_extra, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable] + args, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def test_fault_spec_parse():
    assert fault.parse("kill_rank:1@step:5,nan_loss@step:3") == [("kill_rank", 1, 5), ("nan_loss", -1, 3)]
    with pytest.raises(ValueError):
        fault.parse("explode@now")


def test_kill_restart_resume(data_dir, tmp_path):
    md = str(tmp_path / "m")
    r = _run(["-m", "rocfm.launch", "--nproc", "1", "--max_restarts", "1", "--"] +
             _cli(data_dir, md, "--save_checkpoints_steps", "4"), {"ROCFM_FAULT": "kill_rank:0@step:6"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "restart 1/1" in r.stderr
    assert '"event": "restore"' in r.stderr and '"global_step": 4' in r.stderr  # resumed from step 4
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["train"]["global_step"] == 2048 // 128  # the resumed epoch re-reads from the start, steps 4 → 16


def test_watchdog_fires_on_hang(data_dir, tmp_path):
    r = _run(["-m", "rocfm.cli"] + _cli(data_dir, str(tmp_path / "m"), "--watchdog_s", "3"),
             {"ROCFM_FAULT": "hang_rank:0@step:2"}, timeout=120)
    assert r.returncode == 3
    assert "watchdog: no progress" in r.stderr and "Thread" in r.stderr


def test_nan_loss_guard(data_dir, tmp_path):
    r = _run(["-m", "rocfm.cli"] + _cli(data_dir, str(tmp_path / "m")), {"ROCFM_FAULT": "nan_loss@step:3"})
    assert r.returncode != 0 and "NonFiniteLoss" in r.stderr


def test_corrupt_record_policy(tmp_path):
    from rocfm.data.tfrecord import TFRecordDataset

    p = str(tmp_path / "tr.tfrecords")
    write_synthetic_tfrecord(p, 300, 2000, seed=4)
    fault.corrupt_record(p, 7)
    with pytest.raises(Exception):
        for _ in TFRecordDataset([p], 39, 100, 2000, verify_crc=True, skip_bad=False, num_threads=1):
            pass
    ds = TFRecordDataset([p], 39, 100, 2000, verify_crc=True, skip_bad=True, num_threads=1)
    n = sum(int(b[0].shape[0]) for b in ds)
    assert n == 200 and ds.bad_records == 1  # 299 good records → 2 full batches (drop_remainder)


def test_profile_window(data_dir, tmp_path):
    md = str(tmp_path / "m")
    r = _run(["-m", "rocfm.cli"] + _cli(data_dir, md, "--profile_steps", "2:4"), {})
    assert r.returncode == 0, r.stderr[-2000:]
    assert os.path.exists(os.path.join(md, "profile", "trace.json"))
    assert os.path.getsize(os.path.join(md, "profile", "kernel_table.txt")) > 0


def test_id_guard(monkeypatch):
    from rocfm.utils.numerics import check_ids

    check_ids(torch.tensor([[0, 5]]), 6)
    with pytest.raises(ValueError):
        check_ids(torch.tensor([[0, 6]]), 6)


def test_rank_info_from_env(monkeypatch):
    """torchrun env (RANK / WORLD_SIZE / LOCAL_*) and the SageMaker host list (SM_HOSTS,
    SM_CURRENT_HOST — what the reference's dead set_dist_env read) → rank / host layout."""
    from rocfm.parallel.dist import rank_info_from_env

    monkeypatch.setenv("RANK", "5")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.delenv("SM_HOSTS", raising=False)
    r = rank_info_from_env()
    assert (r.rank, r.world, r.local_rank, r.local_world, r.host_index, r.num_hosts) == (5, 8, 1, 4, 1, 2)
    assert not r.is_chief and r.distributed
    monkeypatch.setenv("SM_HOSTS", '["algo-1", "algo-2"]')
    monkeypatch.setenv("SM_CURRENT_HOST", "algo-2")
    r = rank_info_from_env()
    assert r.num_hosts == 2 and r.host_index == 1
    r = rank_info_from_env(worker_per_host=2)
    assert r.local_world == 2


def test_pyproject_packages_exist():
    """pyproject.toml installs `rocfm` from the hyphenated source directory (no symlink needed):
    every listed package maps to a directory with an __init__.py."""
    import os

    import tomli

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = tomli.load(open(os.path.join(root, "pyproject.toml"), "rb"))["tool"]["setuptools"]
    src = os.path.join(root, cfg["package-dir"]["rocfm"])
    assert os.path.isdir(src) and not os.path.islink(src)
    for pkg in cfg["packages"]:
        d = os.path.join(src, *pkg.split(".")[1:])
        assert os.path.isfile(os.path.join(d, "__init__.py")), pkg
    on_disk = {os.path.relpath(r, src) for r, _, fs in os.walk(src) if "__init__.py" in fs and "__pycache__" not in r}
    listed = {os.path.join(*p.split(".")[1:]) if "." in p else "." for p in cfg["packages"]}
    assert on_disk == listed, (on_disk, listed)


def test_gpu_state_snapshot_never_raises():
    """utils/gpu_state.snapshot: a read-only diagnostic — a dict of numbers, {} without a GPU."""
    from rocfm.utils.gpu_state import snapshot
    s = snapshot()
    assert isinstance(s, dict) and all(isinstance(v, (int, float)) for v in s.values())


def test_numa_cpulist_and_binding_are_safe():
    """utils/numa: sysfs cpulist parsing; without a GPU (or sysfs) nothing is bound."""
    import os

    from rocfm.utils.numa import _parse_cpulist, bind_to_gpu_node, gpu_local_cpus
    assert _parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    before = os.sched_getaffinity(0)
    if gpu_local_cpus() is None:
        assert bind_to_gpu_node() is None and os.sched_getaffinity(0) == before
