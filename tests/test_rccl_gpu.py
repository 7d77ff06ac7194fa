"""The multi-GPU transports on one MI355X, as the 8-GPU node will run them.

* RCCL at world 1 with ROCFM_FORCE_COLLECTIVES=1: the dp / dense_dp / row-shard engines run their
  real ``all_gather_into_tensor`` / ``all_reduce`` / ``all_to_all_single`` calls (captured into the
  multi-step HIP graphs and replayed) and must be bitwise equal to the same engine taking the
  world-1 shortcut.
* ``bench.py --gpus 4`` rehearsal: 4 ranks sharing the GPU over gloo + the p2p push; the JSON line
  must report the world, backend and exchange the run really used.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CASES = [("dp", "sparse"), ("dp", "exact"), ("dense_dp", "exact"), ("rowshard", "sparse"), ("rowshard", "exact")]


def _build(kind, upd, force):
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.optim import OptHParams

    os.environ["ROCFM_FORCE_COLLECTIVES"] = "1" if force else "0"
    spec = ModelSpec(feature_size=5000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.5, 0.5],
                     l2_reg=1e-3)
    hp = OptHParams(name="Adam", lr=1e-3)
    dev = torch.device("cuda", 0)
    if kind == "rowshard":
        from rocfm.parallel.emb_shard import FusedRowShard

        return FusedRowShard(spec, hp, 128, dev, params=init_params(spec, 3), embedding_update=upd, use_graph=True)
    from rocfm.parallel.dp import FusedDataParallel

    return FusedDataParallel(spec, hp, 128, dev, params=init_params(spec, 3), embedding_update=upd, mode=kind,
                             use_graph=True)


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from rocfm.data.synthetic import SyntheticCriteo

    gen = SyntheticCriteo(5000, 39, seed=5)
    g = torch.Generator().manual_seed(5)
    bs = [gen.batch(128, "cpu", g) for _ in range(6)]
    pool = [torch.stack([b[i] for b in bs]).cuda() for i in range(3)]
    res = {}
    for kind, upd in CASES:
        outs = []
        for force in (False, True):
            eng = _build(kind, upd, force)
            eng.attach_pool(*pool)
            eng.train_steps(21, 8)  # 8 + 8 + 5: eager first graph, captured graphs, a remainder graph
            torch.cuda.synchronize()
            eng.check()
            outs.append((eng.emb.cpu(), eng.dense.cpu(), getattr(eng, "exchange", None), eng.global_step()))
            eng.close()
        (e0, d0, x0, s0), (e1, d1, x1, s1) = outs
        res[f"{kind}/{upd}"] = {"emb_equal": bool(torch.equal(e0, e1)), "dense_equal": bool(torch.equal(d0, d1)),
                                "exchange": x1, "steps": (s0, s1)}
    torch.save(res, out)
    dist.destroy_process_group()


def test_rccl_world1_collectives_in_graphs_bitwise(tmp_path):
    out = str(tmp_path / "r.pt")
    mp.start_processes(_worker, args=(_port(), out), nprocs=1, join=True, start_method="spawn")
    res = torch.load(out, weights_only=True)
    for case, r in res.items():
        assert r["steps"] == (21, 21), (case, r)
        assert r["exchange"] == "rccl", (case, r)
        assert r["emb_equal"] and r["dense_equal"], (case, r)


def _bench(args, env_extra, timeout=300):
    env = dict(os.environ)
    env.update(env_extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0]), r.stdout + r.stderr


@pytest.mark.timeout(600)
def test_bench_rehearsal_4_ranks_gloo_p2p():
    """bench.py --gpus 4 relaunches itself under torch.distributed.run; 4 ranks share the GPU (gloo
    bootstrap), the DP exchange is the p2p push through multi-step graphs."""
    j, log = _bench(["--gpus", "4", "--steps", "32", "--warmup", "8", "--steps_per_graph", "16"],
                    {"ROCFM_BENCH_BACKEND": "gloo", "ROCFM_BENCH_AB": "1"}, timeout=600)
    assert j["n_gpus"] == 4 and j["world_size"] == 4 and j["backend"] == "gloo", j
    # ranks sharing the GPU: the copy push (the fused one is the default with one GPU per rank)
    assert j["config"]["exchange"] == "p2p" and j["config"]["fused_push"] is False, (j, log[-2000:])
    assert j["config"]["parallelism"] == "dp4" and j["config"]["global_batch"] == 4096, j
    assert j["value"] > 0 and j["rank_ms_per_step"]["max"] >= j["rank_ms_per_step"]["min"] > 0, j
    assert "falling back" not in log, log[-2000:]
    # the node run's attribution: per-rank phase times of the headline step, what ran, and the
    # secondary windows (collective transport A/B, config 4 at 100M rows) each with its own checks
    ph = j["phase_ms"]
    for k in ("rows", "tail", "merge", "exchange", "step"):
        assert ph[k]["max"] >= ph[k]["min"], (k, ph)
    assert ph["step"]["min"] > 0 and ph["merge_mode"] and ph["cap"] > 0 and ph["push"] == "copy", ph
    assert not [k for k in j if k.endswith("_error")], j
    for w in ("rccl", "rowshard", "merge_plan"):
        assert j[f"{w}_examples_per_sec"] > 0 and j[f"{w}_replicas_consistent"] is True, (w, j)
    # the merge A/B window (forced here on the shared GPU): the plan-ahead merge below PLAN_MIN_W
    assert j["merge_plan_phase_ms"]["merge_mode"] == "plan" and "merge_noplan_examples_per_sec" not in j, j
    assert j["rowshard_exchange"] == "p2p" and j["rowshard_shadow_exchange"] == "ok", j
    assert j["rowshard_feature_size"] == 100_000_000, j
    # TFRecord-fed DP under the reference's record sharding (each rank reads its records through
    # the record index; the GPU parses the payloads)
    assert j["tfrecord_examples_per_sec"] > 0 and j["tfrecord_replicas_consistent"] is True, j
    assert j["tfrecord_shadow_exchange"] == "ok" and j["tfrecord_decode"] == "device", j


def test_bench_rehearsal_2_ranks_fused_push():
    """The fused push (producers store into the peers' slots from the step tail) through bench.py
    at the reference batch, 2 ranks sharing the GPU (forced: ROCFM_DP_PUSH=1)."""
    j, log = _bench(["--gpus", "2", "--steps", "32", "--warmup", "8", "--steps_per_graph", "16"],
                    {"ROCFM_BENCH_BACKEND": "gloo", "ROCFM_DP_PUSH": "1",
                     # forced producer push on a shared GPU: a starved wait ends in ≈4 s with the
                     # sticky error flag (check() raises, bench exits non-zero) instead of hanging
                     "ROCFM_SPIN_LIMIT": str(1 << 26)})
    assert j["n_gpus"] == 2 and j["config"]["exchange"] == "p2p" and j["config"]["fused_push"] is True, j
    assert j["value"] > 0 and "falling back" not in log, log[-2000:]


@pytest.mark.parametrize("extra", [[], ["--hot_rows", "256", "--ps_staleness", "1"]])
def test_bench_rehearsal_4_ranks_rowshard(extra):
    """The PS-equivalent bench at 4 ranks sharing the GPU: p2p all-to-alls, owner merge through
    position maps (W > SEARCH_MAX_W), optionally replicated hot rows and bounded staleness."""
    j, log = _bench(["--gpus", "4", "--parallelism", "rowshard", "--steps", "32", "--warmup", "8",
                     "--steps_per_graph", "16"] + extra, {"ROCFM_BENCH_BACKEND": "gloo"})
    assert j["n_gpus"] == 4 and j["config"]["parallelism"] == "rowshard4", j
    assert j["config"]["exchange"] == "p2p", (j, log[-2000:])
    assert j["value"] > 0 and "falling back" not in log, log[-2000:]


@pytest.mark.parametrize("par", ["dp", "rowshard"])
def test_bench_nccl_world1_forced_collectives(par):
    """The bench's RCCL path at world 1: nccl process group, collectives captured in the graphs."""
    j, _ = _bench(["--parallelism", par, "--steps", "24", "--warmup", "8", "--steps_per_graph", "8"],
                  {"ROCFM_FORCE_COLLECTIVES": "1"})
    assert j["backend"] == "nccl" and j["world_size"] == 1, j
    assert j["config"]["exchange"] == "rccl", j
