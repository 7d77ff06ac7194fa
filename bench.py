#!/usr/bin/env python3
"""rocfm benchmark: DeepFM training throughput (examples/sec, whole job) on 1..8 MI355X.

Config (BASELINE.json config 2/3): DeepFM on Criteo-shape data — 39 fields (13 numeric with fixed
ids + 26 categorical), 1M-row hashed vocabulary, embedding_size k=10, deep_layers 128,64,32,
dropout keep 0.5, Adam lr 5e-4 (× world size, HVD:171), l2 1e-4, per-GPU batch 1024 (the
reference's per-worker batch, NB-HVD:96), bf16 MFMA MLP with f32 master weights.  Weak scaling:
every rank trains its own 1024-example batches; N>1 runs one process per GPU over RCCL.

Data is synthetic (rocfm.data.synthetic: Zipf ids with the bundled data's field layout),
generated once into an HBM-resident pool of batches; each timed step copies its batch into the
engine's input buffers and runs a FULL optimisation step (forward, backward, MLP + embedding
optimizer, cross-rank exchange).  Weights are random-init (TF initialisers).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--engine fused|torch]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "examples/sec (whole node) DeepFM Criteo-39-field at 1/2/4/8 MI355X"
# PyTorch-eager (engine=torch, same semantics, same shapes) measured on one MI355X; see BASELINE.md.
# Measured 2026-10 on one MI355X: bench.py --engine torch [--embedding_update exact], B=1024, 1M vocab, k=10.
EAGER_BASELINE = {"sparse": 439405.8, "exact": 535396.5}


def _human(n: int) -> str:
    for div, suf in ((10**9, "B"), (10**6, "M"), (10**3, "K")):
        if n >= div and n % (div // 10) == 0:
            v = n / div
            return (f"{v:.0f}" if v == int(v) else f"{v:.1f}") + suf
    return str(n)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch_size", type=int, default=1024, help="per-GPU batch")
    ap.add_argument("--feature_size", type=int, default=1_000_000)
    ap.add_argument("--field_size", type=int, default=39)
    ap.add_argument("--embedding_size", type=int, default=10)
    ap.add_argument("--deep_layers", default="128,64,32")
    ap.add_argument("--dropout", default="0.5,0.5,0.5")
    ap.add_argument("--optimizer", default="Adam")
    ap.add_argument("--learning_rate", type=float, default=0.0005)
    ap.add_argument("--l2_reg", type=float, default=0.0001)
    ap.add_argument("--engine", default="fused", choices=["fused", "torch"])
    ap.add_argument("--compute_dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: the MLP input layer's forward GEMM on fp8-e4m3 MFMA (dynamic scales)")
    ap.add_argument("--table_dtype", default="f32", choices=["f32", "bf16"],
                    help="embedding table storage (bf16: stochastic-rounded updates, f32 optimizer slots)")
    ap.add_argument("--embedding_update", default="sparse", choices=["sparse", "exact"])
    ap.add_argument("--parallelism", default="auto", choices=["auto", "dp", "dense_dp", "rowshard", "dp_owner"])
    ap.add_argument("--pool", type=int, default=32, help="distinct device-resident batches to cycle")
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--dp_exchange", default="auto", choices=["auto", "p2p", "rccl"],
                    help="N>1 exchanges (dp all-gather, row-shard all-to-all + all-reduce): p2p push over "
                         "IPC-mapped peer buffers (one node) or RCCL")
    ap.add_argument("--steps_per_graph", type=int, default=0,
                    help="fused engine: steps captured per HIP graph (0 = min(64, steps): a graph's side chain "
                         "prepares exactly the next graph's batches, none beyond the timed window)")
    ap.add_argument("--capacity", default="auto",
                    help="rows per rank (dp) / per owner (rowshard) in the exchange buffers: 'auto' = the exact max "
                         "over the batch pool, 'safe' = batch_size*field_size (never overflows), or a number")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--hot_rows", type=int, default=0,
                    help="rowshard: replicate the N most frequent ids on every rank (gradients ride the MLP bucket)")
    ap.add_argument("--ps_staleness", type=int, default=0, choices=[0, 1],
                    help="rowshard: 1 = bounded-staleness (async-PS) row serving, 0 = synchronous")
    ap.add_argument("--input", default="pool", choices=["pool", "tfrecord"],
                    help="pool: HBM-resident batch pool; tfrecord: synthetic Criteo-shape TFRecord files written "
                         "before timing, fed through the C++ loader -> pinned ring -> HBM ring -> multi-step graphs "
                         "(one GPU)")
    ap.add_argument("--data_dir", default="", help="--input tfrecord: directory for the generated files (default: a "
                                                   "temporary directory, removed afterwards)")
    ap.add_argument("--loader_threads", type=int, default=8)
    ap.add_argument("--host_decode", action="store_true",
                    help="--input tfrecord: parse the Examples on the host (default: raw payloads, parsed on the GPU)")
    ap.add_argument("--loader_hold", type=int, default=2,
                    help="--input tfrecord: decoded groups held ahead of the GPU (pinned ring of (hold+2)*S batches)")
    ap.add_argument("--json_out", default="")
    ap.add_argument("--no_secondary", action="store_true",
                    help="one GPU: skip the secondary windows (exact-mode and TFRecord-fed rates) reported "
                         "next to the headline")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus > 1 and world == 1:
        # re-launch under torch.distributed.run (exec before touching the GPU)
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000), __file__] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    # ROCFM_BENCH_BACKEND=gloo rehearses the N>1 code path with ranks sharing the visible GPUs
    # (host-staged collectives); the real multi-GPU run uses nccl (= RCCL over xGMI), one GPU per rank.
    backend = os.environ.get("ROCFM_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # ROCFM_NUMA_BIND (default 1): this process's threads (and the loader threads it starts) on the CPUs of
    # its GPU's NUMA node (utils/numa.py; profiles/r5_stream_queues.md)
    numa_cpus = None
    if os.environ.get("ROCFM_NUMA_BIND", "1") == "1":
        from rocfm.utils.numa import bind_to_gpu_node
        numa_cpus = bind_to_gpu_node(local)
    # ROCFM_FORCE_COLLECTIVES=1 (one process): a 1-rank process group whose exchanges still run the
    # backend's collectives (rehearses the RCCL calls the multi-GPU node captures)
    pg = world > 1 or os.environ.get("ROCFM_FORCE_COLLECTIVES", "0") == "1"
    if pg:
        if world == 1:  # plain `python bench.py` (no launcher): a local 1-rank rendezvous
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.optim import OptHParams

    layers = [int(x) for x in a.deep_layers.split(",")]
    keeps = [float(x) for x in a.dropout.split(",")]
    spec = ModelSpec(a.feature_size, a.field_size, a.embedding_size, layers, keeps, l2_reg=a.l2_reg)
    hp = OptHParams(name=a.optimizer, lr=a.learning_rate)
    if a.parallelism in ("rowshard", "dp_owner") or (a.engine == "fused" and a.feature_size > 20_000_000):
        params = None  # tables drawn on the device (each rank's own shard in rowshard mode): a
        #                100M-1B-row table never materialises on the host
    else:
        params = init_params(spec, a.seed)  # identical on every rank (= rank-0 broadcast, HVD:418)

    B = a.batch_size
    gen = SyntheticCriteo(a.feature_size, a.field_size, seed=a.seed)
    g = torch.Generator(device=dev).manual_seed(a.seed * 1000 + rank)
    pool = [gen.batch(B, dev, g) for _ in range(a.pool)]
    pool_ids = torch.stack([x[0] for x in pool])
    pool_vals = torch.stack([x[1] for x in pool])
    pool_labels = torch.stack([x[2] for x in pool])

    if a.input == "tfrecord":
        return bench_tfrecord(a, spec, hp, params, dev, rank)

    explicit_dp = a.parallelism in ("dp", "dense_dp")
    parallelism = a.parallelism
    if parallelism == "auto":
        parallelism = "dp"  # either update; dense_dp (dense all-reduce) only when asked for
    cap = None
    sharded = parallelism in ("rowshard", "dp_owner")  # owner-routed row gradients (emb_shard)
    if a.engine == "fused" and (world > 1 or a.parallelism in ("dp", "rowshard", "dp_owner")) and parallelism != "dense_dp":
        if a.capacity == "auto":
            from rocfm.parallel.dp import pool_exchange_capacity

            cap = pool_exchange_capacity(pool_ids, world if sharded else 1)
        elif a.capacity != "safe":
            cap = int(a.capacity)
    if a.engine == "fused":
        if sharded:
            from rocfm.parallel.emb_shard import FusedRowShard

            eng = FusedRowShard(spec, hp, B, dev, params=params, embedding_update=a.embedding_update, seed=a.seed,
                                use_graph=not a.no_graph, capacity=cap, compute_dtype=a.compute_dtype, table_dtype=a.table_dtype,
                                exchange=a.dp_exchange, staleness=a.ps_staleness, hot_rows=a.hot_rows,
                                replicate_table=parallelism == "dp_owner")
        elif world > 1 or explicit_dp:
            from rocfm.parallel.dp import FusedDataParallel

            eng = FusedDataParallel(spec, hp, B, dev, params=params, embedding_update=a.embedding_update,
                                    mode=parallelism, seed=a.seed, use_graph=not a.no_graph, capacity=cap,
                                    compute_dtype=a.compute_dtype, table_dtype=a.table_dtype, exchange=a.dp_exchange)
        else:
            from rocfm.models.fused import FusedDeepFM

            eng = FusedDeepFM(spec, hp, B, dev, embedding_update=a.embedding_update, params=params, seed=a.seed,
                              use_graph=not a.no_graph, compute_dtype=a.compute_dtype, table_dtype=a.table_dtype)

        eng.attach_pool(pool_ids, pool_vals, pool_labels)

        def run(n):
            if hasattr(eng, "train_steps"):
                eng.train_steps(n, a.steps_per_graph)
            else:
                for _ in range(n):
                    eng.train_step()
    else:
        from rocfm.models.torch_engine import TorchDeepFM

        if sharded:  # (dp_owner: the same synchronous mathematics as rowshard in eager PyTorch)
            from rocfm.parallel.emb_shard import TorchRowShard

            eng = TorchRowShard(spec, hp, dev, embedding_update=a.embedding_update, params=params, seed=a.seed)
        else:
            eng = TorchDeepFM(spec, hp, dev, embedding_update=a.embedding_update, params=params, seed=a.seed)
        if world > 1 and not sharded:
            from rocfm.parallel.dp import attach_torch_dp

            attach_torch_dp(eng, a.embedding_update)

        def run(n, _it=[0]):
            for _ in range(n):
                ids, vals, labels = pool[_it[0] % len(pool)]
                eng.train_step(ids, vals, labels)
                _it[0] += 1

    if world > 1 and hasattr(eng, "set_lr_scale"):
        eng.set_lr_scale(float(world))  # Horovod linear LR scaling (HVD:171)

    if a.steps_per_graph <= 0:
        a.steps_per_graph = max(2, min(64, a.steps))
    shadow = getattr(eng, "shadow", None)
    if not warm_capture_first(eng, run, a.warmup, a.steps, a.steps_per_graph):
        run(a.warmup)
        while shadow is not None and shadow.active:  # p2p self-validation window: always untimed
            eng.train_step()
        if hasattr(eng, "precapture"):
            eng.precapture(a.steps, a.steps_per_graph)  # graph captures stay out of the timed region
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # every rank's own timed window → the slowest (reported) and fastest rank
    t = torch.tensor([dt, -dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if pg:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, dt_min = float(t[0].item()), -float(t[1].item())
    replicas_ok = None
    if hasattr(eng, "verify_replicas"):
        eng.check(replicas=False)  # sticky device flags (exchange overflow, p2p peer timeout): fail loudly
        # collective digest of every replicated tensor: a fast but wrong multi-GPU run shows here
        replicas_ok = bool(eng.verify_replicas()) if world > 1 else None
    elif hasattr(eng, "check"):
        eng.check()  # sticky device flags (BN barrier, id guard): fail loudly
    ms = dt / a.steps * 1e3
    value = B * world * a.steps / dt
    base = EAGER_BASELINE.get(a.embedding_update)
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "examples/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        # the reference publishes no numbers, so there is no baseline ratio; the
        # in-house PyTorch-eager engine of the same model is reported separately for context
        "vs_baseline": None,
        "vs_eager_pytorch": (round(value / (base * world), 3) if base else None),
        # (relative to a STORED constant: the eager engine's rate measured once, EAGER_BASELINE above,
        # not re-measured in this run)
        "vs_eager_pytorch_basis": "stored constant (EAGER_BASELINE, bench.py --engine torch, one MI355X)",
        "dtype": a.compute_dtype if a.engine == "fused" else "fp32",
        "data": "synthetic Criteo-shape (39 fields, Zipf ids, HBM-resident batch pool), random-init weights",
        "config": {
            "model": f"DeepFM Criteo-shape ({a.field_size} fields, {_human(a.feature_size)}-hash vocab, k={a.embedding_size}, "
                     f"mlp {a.deep_layers}, dropout keep {a.dropout}, {a.optimizer})",
            "global_batch": B * world,
            "seq_len": a.field_size,
            "parallelism": f"{parallelism}{world}" if (world > 1 or a.parallelism != "auto") else "dp1",
            "engine": a.engine,
            "embedding_update": a.embedding_update,
            "table_dtype": a.table_dtype,
            "exchange_capacity": cap,
            "ps_staleness": a.ps_staleness if parallelism == "rowshard" else None,
            "hot_rows": a.hot_rows if parallelism == "rowshard" else None,
            "exchange": getattr(eng, "exchange", None) if pg else None,
            "fused_push": bool(getattr(eng, "fused_push", False)) if pg else None,
            # the planned step tail (emb_plan.hip): embedding workgroups per step, or null (fixed chunks)
            "emb_plan_workgroups": (getattr(eng, "m_plan_nw", None) if getattr(eng, "m_eplan", False) else None),
        },
        "world_size": dist.get_world_size() if pg else 1,
        "backend": (dist.get_backend() if pg else None),
        "rank_ms_per_step": {"max": round(ms, 4), "min": round(dt_min / a.steps * 1e3, 4)},
        "numa_bind_cpus": (len(numa_cpus) if numa_cpus else None),
        # self-validation (rocfm.parallel.validate): replicas bit-identical across ranks after the
        # timed steps; the p2p exchange's first steps checked bitwise against the collective
        "replicas_consistent": replicas_ok,
        "shadow_exchange": (shadow.status if shadow is not None else None),
    }
    wd = None
    if world > 1 and a.engine == "fused" and not a.no_secondary:
        wd = _Watchdog(out, rank, a.json_out)  # bounds everything after the headline
    if (world > 1 and a.engine == "fused" and hasattr(eng, "phase_windows") and not a.no_secondary):
        wd.window = "phase_ms"
        try:  # per-rank device phase times of the headline's DP step (diagnostic windows, after it)
            out["phase_ms"] = eng.phase_windows(64, a.steps_per_graph)
        except Exception as e:  # noqa: BLE001 — a diagnostic never costs the headline
            out["phase_ms_error"] = f"{type(e).__name__}: {e}"[:300]
        _ctrl_barrier()
    if hasattr(eng, "close"):
        eng.close()  # graphs holding RCCL collectives must go before the process group
    if (not pg and a.engine == "fused" and a.parallelism == "auto" and not a.no_secondary
            and a.feature_size <= 20_000_000):
        del eng, run
        out.update(secondary_windows(a, spec, hp, params, dev, (pool_ids, pool_vals, pool_labels)))
    elif world > 1 and a.engine == "fused" and a.parallelism == "auto" and not a.no_secondary:
        del eng, run
        multi_gpu_windows(a, spec, hp, params, dev, (pool_ids, pool_vals, pool_labels), world, rank, backend, out,
                          wd)
    if wd is not None:
        wd.cancel()
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if pg:
        dist.barrier()
        dist.destroy_process_group()


_CTRL = []


def warm_capture_first(eng, run, warmup: int, steps: int, spg: int) -> bool:
    """Warm-up order: capture every graph the LAST warm-up steps and the timed window will launch,
    then run those warm-up steps — so the timed window starts right behind graph-replayed warm-up
    steps instead of behind the capture's idle gap (a 20-step window measured ≈2 µs/step slower
    there; profiles/r6_window_fixed_cost.md).  Same W untimed steps, same K timed steps.

    * single-GPU fused engine: warm-up step 1 (eager: code objects load), capture, steps 2..W;
    * DP / row-shard engines: warm-up steps 1..W-m (p2p shadow-validated steps and the eager first
      graph among them), capture, the last m = W // 2 steps; if the multi-step path has not
      launched by then (all of them were shadow steps) the round-5 order is kept.
    ROCFM_BENCH_CAPTURE_FIRST=0: capture after the warm-up (the round-5 order).  Returns False when
    not applied (the caller then runs the warm-up and captures itself)."""
    from rocfm.models.fused import FusedDeepFM

    if (warmup < 2 or spg < 2 or not hasattr(eng, "precapture")
            or os.environ.get("ROCFM_BENCH_CAPTURE_FIRST", "1") != "1"):
        return False
    if type(eng) is FusedDeepFM:
        run(1)
        eng.precapture([warmup - 1, steps], spg)
        run(warmup - 1)
        return True
    m = warmup // 2
    run(warmup - m)
    shadow = getattr(eng, "shadow", None)
    while shadow is not None and shadow.active:  # p2p self-validation window: always untimed
        eng.train_step()
    if getattr(getattr(eng, "eng", eng), "_m_warm", 0) < 1:  # the multi-step path has not launched yet
        run(m)
        eng.precapture(steps, spg)
        return True
    eng.precapture([m, steps], spg)
    run(m)
    return True


def _ctrl_barrier():
    """Host-side barrier on a gloo group (never queued behind GPU work)."""
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return
    if not _CTRL:
        _CTRL.append(dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else None)
    dist.barrier(group=_CTRL[0])


def _rank_span(dt, dev, backend):
    """(max, min) over ranks of a timed window."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([dt, -dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0].item()), -float(t[1].item())


class _Watchdog:
    """N > 1: bounds the work after the headline (phase windows, secondary windows) — on expiry
    (ROCFM_BENCH_SECONDARY_S, default 300 s) rank 0 prints the JSON gathered so far with the name
    of the window that overran, and every rank exits, so a hung secondary never loses the headline."""

    def __init__(self, out, rank, json_out):
        import threading

        self.out, self.rank, self.json_out, self.window, self.done = out, rank, json_out, None, False
        self.budget = float(os.environ.get("ROCFM_BENCH_SECONDARY_S", "300"))
        self.t = threading.Timer(self.budget, self._expire)
        self.t.daemon = True
        self.t.start()

    def _expire(self):
        if self.done:
            return
        if self.rank == 0:
            h = dict(self.out)
            h["secondary_error"] = f"watchdog: window {self.window} overran {self.budget:.0f} s"
            print(json.dumps(h), flush=True)
            if self.json_out:
                with open(self.json_out, "w") as f:
                    f.write(json.dumps(h) + "\n")
        os._exit(0)

    def cancel(self):
        self.done = True
        self.t.cancel()


def multi_gpu_windows(a, spec, hp, params, dev, pool, world, rank, backend, out, wd):
    """N > 1: secondary windows beside the headline (DP over the p2p push), each on a fresh engine
    and fenced — a window that fails becomes an error string in ``out``, one that overruns trips
    the watchdog; either way the headline is printed:

    * ``rccl``: the same DP step with the exchange on RCCL (all-gather captured in the graphs), the
      transport A/B of the node;
    * ``merge_plan`` (below PLAN_MIN_W ranks) / ``merge_noplan`` (from PLAN_MIN_W): the headline's DP
      step with the other row merge than the default (``ROCFM_MERGE``), and ``push_copy`` (when the
      headline used the fused producer push): with the copy push (``ROCFM_DP_PUSH=0``), each with
      ``phase_ms`` beside the headline's — the A/Bs behind ``dp.PLAN_MIN_W`` and the push default
      (only with one GPU per rank unless ``ROCFM_BENCH_AB=1``; ``=0`` skips them);
    * ``rowshard``: config 4 — the PS-equivalent row-sharded table at 100M rows
      (``…multiInstance.py:461-521``), p2p all-to-alls.
    Every window reports its own replica check and p2p shadow status."""
    import torch

    S = a.steps_per_graph
    B = a.batch_size

    def run_window(name, build, env=None, phases=False):
        wd.window = name
        t_w = time.perf_counter()
        if rank == 0:
            print(f"[bench] window {name} ...", file=sys.stderr, flush=True)
        err = None
        res = {}
        eng = None
        saved = {k: os.environ.get(k) for k in (env or {})}
        os.environ.update(env or {})
        try:
            eng = build()
            eng.attach_pool(*pool)
            eng.set_lr_scale(float(world))
            eng.train_steps(a.warmup, S)
            while getattr(eng, "shadow", None) is not None and eng.shadow.active:
                eng.train_step()
            eng.precapture(a.steps, S)
            torch.cuda.synchronize()
            _ctrl_barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.train_steps(a.steps, S)
            torch.cuda.synchronize()
            _ctrl_barrier()
            dt = time.perf_counter() - t0
            dmax, dmin = _rank_span(dt, dev, backend)
            eng.check(replicas=False)
            res = {"examples_per_sec": round(B * world * a.steps / dmax, 1),
                   "ms_per_step": round(dmax / a.steps * 1e3, 4),
                   "rank_ms_per_step_min": round(dmin / a.steps * 1e3, 4),
                   "replicas_consistent": bool(eng.verify_replicas()),
                   "shadow_exchange": eng.shadow.status if getattr(eng, "shadow", None) is not None else None,
                   "exchange": getattr(eng, "exchange", None),
                   "fused_push": bool(getattr(eng, "fused_push", False))}
            if phases:  # per-rank device phase times (diagnostic, after the timed steps)
                try:
                    res["phase_ms"] = eng.phase_windows(64, S)
                except Exception as e:  # noqa: BLE001
                    res["phase_ms_error"] = f"{type(e).__name__}: {e}"[:300]
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:300]
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            if eng is not None and hasattr(eng, "close"):
                try:
                    eng.close()
                except Exception:  # noqa: BLE001
                    pass
            del eng
            torch.cuda.empty_cache()
        _ctrl_barrier()
        if err is not None:
            out[f"{name}_error"] = err
        for k, v in res.items():
            out[f"{name}_{k}"] = v
        if rank == 0:
            print(f"[bench] window {name}: {time.perf_counter() - t_w:.1f} s{' (error)' if err else ''}",
                  file=sys.stderr, flush=True)

    from rocfm.parallel.dp import PLAN_MIN_W, FusedDataParallel, pool_exchange_capacity
    from rocfm.parallel.emb_shard import FusedRowShard

    pool_ids = pool[0]
    cap = pool_exchange_capacity(pool_ids, 1)
    run_window("rccl", lambda: FusedDataParallel(spec, hp, B, dev, params=params, mode="dp", seed=a.seed,
                                                 capacity=cap, compute_dtype=a.compute_dtype, exchange="rccl"))

    # the headline's DP step with each row merge and each push form, every one with its phase times:
    # the node's measurement behind PLAN_MIN_W (dp.py) and the fused push default (p2p.py)
    def dp_default():
        return FusedDataParallel(spec, hp, B, dev, params=params, mode="dp", seed=a.seed, capacity=cap,
                                 compute_dtype=a.compute_dtype, exchange=a.dp_exchange)

    # (the headline runs the default; each A/B window runs the other choice: the plan-ahead merge
    # from PLAN_MIN_W ranks, the fused push wherever every rank has a GPU of its own)
    # (only where every rank has a GPU of its own, or when asked for: on a shared GPU the windows
    # measure the processes' contention — and the forced fused push of a rehearsal can starve there)
    ab = os.environ.get("ROCFM_BENCH_AB", "auto")
    if ab == "1" or (ab == "auto" and torch.cuda.device_count() >= world):
        if world >= PLAN_MIN_W:
            run_window("merge_noplan", dp_default, env={"ROCFM_MERGE": "noplan"}, phases=True)
        else:
            run_window("merge_plan", dp_default, env={"ROCFM_MERGE": "plan"}, phases=True)
        if out.get("config", {}).get("fused_push"):
            run_window("push_copy", dp_default, env={"ROCFM_DP_PUSH": "0"}, phases=True)
    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec

    V4 = 100_000_000
    spec4 = ModelSpec(V4, spec.field_size, spec.embedding_size, spec.layers, spec.keep_probs, l2_reg=spec.l2_reg)
    gen = SyntheticCriteo(V4, spec.field_size, seed=a.seed)
    g = torch.Generator(device=dev).manual_seed(a.seed * 1000 + rank)
    p4 = [gen.batch(B, dev, g) for _ in range(min(a.pool, 16))]
    pool = (torch.stack([x[0] for x in p4]), torch.stack([x[1] for x in p4]), torch.stack([x[2] for x in p4]))
    cap4 = pool_exchange_capacity(pool[0], world)
    run_window("rowshard", lambda: FusedRowShard(spec4, hp, B, dev, params=None, seed=a.seed, capacity=cap4,
                                                 compute_dtype=a.compute_dtype))
    out["rowshard_feature_size"] = V4
    del pool, p4
    torch.cuda.empty_cache()
    tfrecord_window(a, spec, hp, params, dev, world, rank, backend, out, wd)


def tfrecord_window(a, spec, hp, params, dev, world, rank, backend, out, wd):
    """N > 1, TFRecord-fed DP under the reference's default record sharding
    (``dataset.shard(hvd.size(), hvd.rank())``, HVD:132-133): every rank writes one synthetic
    Criteo-shape file (with its record index) in parallel, then reads every P-th record of the
    concatenated file list — only its own records, through the index — as undecoded payloads that
    its GPU parses (raw loader mode + decode.hip), streamed through the DP multi-step graphs with the
    exchange inline.  The files hold 256 batches per rank; the window repeats them as epochs."""
    import shutil
    import tempfile

    import torch
    import torch.distributed as dist

    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.data.tfrecord import TFRecordDataset
    from rocfm.parallel.dp import FusedDataParallel

    wd.window = "tfrecord"
    B, F, S = a.batch_size, spec.field_size, 16
    nb = 256  # batches per rank per epoch
    steps, warm = max(1024, a.steps), 64
    obj = [tempfile.mkdtemp(prefix="rocfm_bench_mtf_") if rank == 0 else None]
    _ctrl_barrier()
    dist.broadcast_object_list(obj, src=0, group=_CTRL[0] if _CTRL and _CTRL[0] is not None else None)
    d = obj[0]
    err, res, eng = None, {}, None
    try:
        t0 = time.perf_counter()
        write_synthetic_tfrecord(os.path.join(d, f"tr{rank}.tfrecords"), nb * B, spec.feature_size, F,
                                 seed=a.seed + 17 * rank)
        gen_s = time.perf_counter() - t0
        _ctrl_barrier()
        files = [os.path.join(d, f"tr{r}.tfrecords") for r in range(world)]

        def groups(skip, limit):
            ds = TFRecordDataset(files, F, B, spec.feature_size, num_epochs=-(-(skip + limit) // nb) + 1,
                                 shard_count=world, shard_index=rank, num_threads=4, hold=2)
            return ds.raw_groups(S, hold=2, skip=skip, limit=limit)

        eng = FusedDataParallel(spec, hp, B, dev, params=params, mode="dp", seed=a.seed,
                                compute_dtype=a.compute_dtype)
        eng.set_lr_scale(float(world))
        eng.train_stream(groups(0, warm), S, hold=2)  # shadow window + graph captures
        torch.cuda.synchronize()
        _ctrl_barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = eng.train_stream(groups(warm, steps), S, hold=2)
        torch.cuda.synchronize()
        _ctrl_barrier()
        dt = time.perf_counter() - t0
        dmax, dmin = _rank_span(dt, dev, backend)
        eng.check(replicas=False)
        if done != steps:
            raise RuntimeError(f"trained {done} steps, expected {steps}")
        res = {"examples_per_sec": round(B * world * steps / dmax, 1), "ms_per_step": round(dmax / steps * 1e3, 4),
               "rank_ms_per_step_min": round(dmin / steps * 1e3, 4), "steps": steps,
               "replicas_consistent": bool(eng.verify_replicas()), "shadow_exchange": eng.shadow.status,
               "exchange": eng.exchange, "shard": "record (Dataset.shard(P, rank), record index)",
               "decode": "device", "data_gen_s": round(gen_s, 2)}
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"[:300]
    finally:
        if eng is not None:
            try:
                eng.close()
            except Exception:  # noqa: BLE001
                pass
        del eng
        torch.cuda.empty_cache()
    _ctrl_barrier()
    if rank == 0:
        shutil.rmtree(d, ignore_errors=True)
    if err is not None:
        out["tfrecord_error"] = err
    for k, v in res.items():
        out[f"tfrecord_{k}"] = v


def secondary_windows(a, spec, hp, params, dev, pool):
    """One GPU, same config and window length as the headline: (1) the reference-faithful
    ``embedding_update=exact`` step (dense full-table L2 + Adam over every row, PS:277-278, 307) and
    (2) the loader-fed rate (synthetic Criteo-shape TFRecord files → C++ loader → HBM ring →
    multi-step graphs), so both are driver-observed, not only builder-run."""
    import gc

    import torch

    from rocfm.models.fused import FusedDeepFM

    out = {}

    def tf_window(prefix="tfrecord_"):
        # the loader-fed window: >= 2048 steps streamed from the TFRecord files (several epochs of a
        # 512-batch file set), warm-up with the same ring and graph set, so the window holds no
        # graph rebuild or capture; the time to the first graph is reported separately
        import copy

        ta = copy.copy(a)
        # (warm-up >= 4 graphs: the first launch is eager, so both parities' graphs get captured)
        # (32 steps per graph: 27.9-29.9 M ex/s vs 26.7-28.0 M at 16, profiles/r4_seg_sort.md)
        ta.steps, ta.warmup, ta.steps_per_graph = max(2048, a.steps), max(128, a.warmup), 32
        state = os.environ.get("ROCFM_BENCH_GPU_STATE", "0") == "1"  # diagnostics: device clocks / temperature
        if state:
            from rocfm.utils.gpu_state import snapshot
            out[prefix + "gpu_before"] = snapshot()
        try:
            t = measure_tfrecord(ta, spec, hp, params, dev)
            if state:
                out[prefix + "gpu_after"] = snapshot()
            out[prefix + "steps"] = ta.steps
            for k in ("value", "ms_per_step", "steady_examples_per_sec", "fill_ms", "input_stall_fraction",
                      "loader_alone_examples_per_sec", "host_decode_loader_alone_examples_per_sec", "decode",
                      "copy_stream_ms_per_group", "copy_stream_GBps", "copy_stream_busy_fraction",
                      "copy_stream_h2d_ms_per_group", "copy_stream_parse_ms_per_group", "copy_stream_h2d_GBps",
                      "gpu_stall_fraction", "gpu_side_stall_fraction", "gpu_main_busy_fraction", "host_copy_wait_s"):
                out[prefix + ("examples_per_sec" if k == "value" else k)] = t.get(k)
        except Exception as e:  # a secondary window never costs the headline
            out[prefix + "error"] = f"{type(e).__name__}: {e}"[:400]

    # the TFRecord window runs first: after the other windows it measured 20 % slower than in a
    # process of its own (profiles/r4_radix_ab.md); ROCFM_BENCH_TF_FIRST=0 restores the old order
    tf_first = os.environ.get("ROCFM_BENCH_TF_FIRST", "1") == "1"
    if tf_first:
        tf_window()
    eng = FusedDeepFM(spec, hp, a.batch_size, dev, embedding_update="exact", params=params, seed=a.seed,
                      compute_dtype=a.compute_dtype, table_dtype=a.table_dtype)
    eng.attach_pool(*pool)
    S = a.steps_per_graph
    if not warm_capture_first(eng, lambda n: eng.train_steps(n, S), a.warmup, a.steps, S):
        eng.train_steps(a.warmup, S)
        eng.precapture(a.steps, S)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.train_steps(a.steps, S)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.check()
    out["exact_examples_per_sec"] = round(a.batch_size * a.steps / dt, 1)
    out["exact_ms_per_step"] = round(dt / a.steps * 1e3, 4)
    del eng
    gc.collect()
    torch.cuda.empty_cache()
    # the reference's own shapes (sparse update, same window): the notebook job (117,581 × 32,
    # MLP 128-64-32; deepfm-sagemaker-hvd-gpu.ipynb:94-103) and the scripts' flag defaults
    # (embedding_size 32, deep_layers 256,128,64; …multiInstance.py:52,62)
    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec, init_params

    for name, layers in (("notebook", [128, 64, 32]), ("refdefaults", [256, 128, 64])):
        try:
            sp = ModelSpec(117581, a.field_size, 32, layers, [0.5] * 3, l2_reg=spec.l2_reg)
            gen = SyntheticCriteo(117581, a.field_size, seed=a.seed)
            g = torch.Generator(device=dev).manual_seed(a.seed)
            pb = [gen.batch(a.batch_size, dev, g) for _ in range(a.pool)]
            e2 = FusedDeepFM(sp, hp, a.batch_size, dev, params=init_params(sp, a.seed), seed=a.seed,
                             compute_dtype=a.compute_dtype, table_dtype=a.table_dtype)
            e2.attach_pool(torch.stack([x[0] for x in pb]), torch.stack([x[1] for x in pb]),
                           torch.stack([x[2] for x in pb]))
            if not warm_capture_first(e2, lambda n: e2.train_steps(n, S), a.warmup, a.steps, S):
                e2.train_steps(a.warmup, S)
                e2.precapture(a.steps, S)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e2.train_steps(a.steps, S)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            e2.check()
            out[f"{name}_examples_per_sec"] = round(a.batch_size * a.steps / dt, 1)
            out[f"{name}_ms_per_step"] = round(dt / a.steps * 1e3, 4)
            del e2, pb
        except Exception as e:  # noqa: BLE001 — a secondary window never costs the headline
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"[:300]
        gc.collect()
        torch.cuda.empty_cache()
    if not tf_first:
        tf_window()
    out.update(scale_windows(a, spec, hp, dev))
    if os.environ.get("ROCFM_BENCH_TF_TWICE", "0") == "1":  # diagnostics: the same window again, last
        tf_window("tfrecord_last_")
    return out


def scale_windows(a, spec, hp, dev):
    """One GPU, the bench config's model at the vocabulary scales of BASELINE.json configs 4 and 5,
    each window fenced (a failure becomes ``<name>_error``) and timed like the headline (same
    warm-up, steps, steps per graph; full optimisation steps):

    * ``rowshard100m``: config 4's PS-equivalent row-sharded table at 100M rows (the owner-routed
      lookup / gradient exchange at world 1, ``…multiInstance.py:461-521``);
    * ``capacity``: config 5 — the largest table with f32 Adam slots that fits this GPU's HBM next to
      the step's buffers (≈90 %: 1.8B rows × (k+1 → 12 floats) × {table, m, v} ≈ 259 GB on a
      288 GB MI355X), with the fp8-e4m3 MFMA MLP input layer; reports the rows and the bytes
      resident."""
    import gc

    import torch

    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec

    out = {}
    S = a.steps_per_graph
    B = a.batch_size

    def pool_for(V, n):
        gen = SyntheticCriteo(V, spec.field_size, seed=a.seed)
        g = torch.Generator(device=dev).manual_seed(a.seed)
        pb = [gen.batch(B, dev, g) for _ in range(n)]
        return tuple(torch.stack([x[i] for x in pb]) for i in range(3))

    def window(name, V, build, **extra):
        eng, pool = None, None
        try:
            t0 = time.perf_counter()
            sp = ModelSpec(V, spec.field_size, spec.embedding_size, spec.layers, spec.keep_probs, l2_reg=spec.l2_reg)
            pool = pool_for(V, min(a.pool, 16))
            eng = build(sp, pool)
            torch.cuda.synchronize()
            build_s = time.perf_counter() - t0
            resident = torch.cuda.memory_allocated(dev)
            eng.attach_pool(*pool)
            if not warm_capture_first(eng, lambda n: eng.train_steps(n, S), a.warmup, a.steps, S):
                eng.train_steps(a.warmup, S)
                eng.precapture(a.steps, S)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.train_steps(a.steps, S)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            eng.check() if not hasattr(eng, "verify_replicas") else eng.check(replicas=False)
            out[f"{name}_examples_per_sec"] = round(B * a.steps / dt, 1)
            out[f"{name}_ms_per_step"] = round(dt / a.steps * 1e3, 4)
            out[f"{name}_feature_size"] = V
            out[f"{name}_bytes_resident"] = int(resident)
            out[f"{name}_build_s"] = round(build_s, 2)
            out.update({f"{name}_{k}": v for k, v in extra.items()})
        except Exception as e:  # noqa: BLE001 — a secondary window never costs the headline
            out[f"{name}_error"] = f"{type(e).__name__}: {e}"[:300]
        finally:
            if eng is not None and hasattr(eng, "close"):
                try:
                    eng.close()
                except Exception:  # noqa: BLE001
                    pass
            del eng, pool
            gc.collect()
            torch.cuda.empty_cache()

    from rocfm.parallel.dp import pool_exchange_capacity
    from rocfm.parallel.emb_shard import FusedRowShard

    def rowshard(sp, pool):
        return FusedRowShard(sp, hp, B, dev, params=None, seed=a.seed, capacity=pool_exchange_capacity(pool[0], 1),
                             compute_dtype=a.compute_dtype)

    window("rowshard100m", 100_000_000, rowshard, parallelism="rowshard1")

    from rocfm.models.fused import FusedDeepFM

    free, total = torch.cuda.mem_get_info(dev)
    kp = (spec.embedding_size + 1 + 3) // 4 * 4
    per_row = kp * 4 * 3  # f32 table + Adam m, v
    # ≈90 % of the device for the table + slots, ids < 2^31, at most what is free now minus 6 GB
    rows = min(int(0.9 * total) // per_row, (free - (6 << 30)) // per_row, (1 << 31) - 1)
    rows = rows // 1_000_000 * 1_000_000

    def capacity(dtype):
        return lambda sp, pool: FusedDeepFM(sp, hp, B, dev, params=None, seed=a.seed, compute_dtype=dtype)

    if rows >= 1_000_000:
        # config 5 as BASELINE.json names it (fp8 MFMA MLP input layer), then the same table with the
        # bf16 MLP beside it: the fp8 layer's cost / gain at this shape, driver-observed
        for name, dtype in (("capacity", "fp8"), ("capacity_bf16", "bf16")):
            window(name, rows, capacity(dtype), table_bytes=rows * per_row, hbm_total_bytes=int(total),
                   hbm_fraction=round(rows * per_row / total, 3), compute_dtype=dtype, table_dtype="f32",
                   optimizer_slots="f32 Adam m, v")
    return out


def bench_tfrecord(a, spec, hp, params, dev, rank):
    out = measure_tfrecord(a, spec, hp, params, dev)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")


def measure_tfrecord(a, spec, hp, params, dev):
    """Loader-fed end-to-end throughput on one GPU (the reference's tf.data chain is inside its
    training loop: PS:147-165, HVD:128-159): synthetic Criteo-shape TFRecord files (with their
    record indexes) → C++ loader (frames + CRCs; raw mode copies the Example payloads, the GPU
    parses them — ``--host_decode`` parses on the host instead) → pinned ring → HBM ring →
    multi-step graphs.  The files hold at most 512 batches; longer windows repeat them as epochs
    (the reference's ``repeat(num_epochs)``).  Warm-up trains W batches through the SAME ring and
    graph set, so the timed train_stream call rebuilds nothing: it starts a fresh loader (thread
    start, file mapping, first decode = the reported ``fill_ms``, time to the first graph launch)
    and ends when the last step has run."""
    import shutil
    import tempfile

    import torch

    from rocfm.data.synthetic import write_synthetic_tfrecord
    from rocfm.data.tfrecord import TFRecordDataset
    from rocfm.models.fused import FusedDeepFM

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("--input tfrecord measures one GPU (use the Estimator / rocfm.cli for multi-GPU runs)")
    B, F, S = a.batch_size, a.field_size, (a.steps_per_graph if a.steps_per_graph > 0 else 32)
    if a.warmup < 4 * S:  # both parities' graphs captured before the window (the first launch is eager)
        import copy

        a = copy.copy(a)
        a.warmup = 4 * S
    own = not a.data_dir
    d = a.data_dir or tempfile.mkdtemp(prefix="rocfm_bench_")
    os.makedirs(d, exist_ok=True)
    nbat = min(512, a.warmup + a.steps)  # batches in the file set (one epoch)
    nrec = nbat * B
    files, per = [], (nrec + 3) // 4
    t0 = time.perf_counter()
    for i in range(4):  # 4 files, like sharded S3 objects
        p = os.path.join(d, f"tr{i}.tfrecords")
        m = min(per, nrec - i * per)
        if m <= 0:
            break
        if not (os.path.exists(p) and a.data_dir):
            write_synthetic_tfrecord(p, m, a.feature_size, F, seed=a.seed + i)
        files.append(p)
    gen_s = time.perf_counter() - t0
    raw = not getattr(a, "host_decode", False)

    def groups(skip=0, limit=None, decode_raw=raw):
        epochs = -(-(skip + (limit or 0)) // nbat) + 1
        ds = TFRecordDataset(files, F, B, a.feature_size, num_threads=a.loader_threads, verify_crc=True,
                             hold=a.loader_hold, num_epochs=epochs)
        if decode_raw:
            return ds.raw_groups(S, hold=a.loader_hold, skip=skip, limit=limit)
        return ds.groups(S, hold=a.loader_hold, skip=skip, limit=limit)

    def loader_alone(decode_raw):
        t = time.perf_counter()
        nb = sum((g.n if decode_raw else int(g[0].shape[0])) for g in groups(0, a.steps, decode_raw))
        return nb * B / (time.perf_counter() - t)

    loader_eps = loader_alone(raw)
    host_eps = loader_alone(False) if raw else loader_eps

    eng = FusedDeepFM(spec, hp, B, dev, embedding_update=a.embedding_update, params=params, seed=a.seed,
                      compute_dtype=a.compute_dtype, table_dtype=a.table_dtype)
    H = a.loader_hold
    eng.train_stream(groups(0, a.warmup), S, hold=H)  # code objects + every graph of the ring
    stall = [0.0]

    def timed(it):
        it = iter(it)
        while True:
            t1 = time.perf_counter()
            x = next(it, None)
            stall[0] += time.perf_counter() - t1
            if x is None:
                return
            yield x

    eng.copy_timing = []  # per raw group: H2D copy + device parse on the copy stream
    eng.stall_timing = []  # per graph: main start / main end / side end (GPU-side gaps of the main stream)
    eng.host_copy_wait_s = 0.0  # host time blocked on copy completions (a ring slot's host memory recycled)
    marks = []  # (host time, event) after each graph launch

    def after(first, n):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((time.perf_counter(), ev, first + n))

    import gc

    gc.collect()
    gc.disable()  # a collector pass over the process's objects must not stall the launch loop
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = eng.train_stream(timed(groups(a.warmup, a.steps)), S, hold=H, after_steps=after)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        gc.enable()
    eng.check()
    if done != a.steps:
        raise RuntimeError(f"trained {done} steps, expected {a.steps}")
    # steady state: GPU time between the ends of the first and the last graph
    steady = None
    if len(marks) > 2:
        g0, g1 = marks[0], marks[-1]
        ms = g0[1].elapsed_time(g1[1])
        steady = (g1[2] - g0[2]) * B / (ms * 1e-3) if ms > 0 else None
    value = B * a.steps / dt
    ct = [(x[0].elapsed_time(x[1]), x[2], x[3], x[0].elapsed_time(x[4])) for x in eng.copy_timing]
    eng.copy_timing = None
    # GPU-side stall: the main stream's gaps between consecutive graphs (graph j may start only once
    # graph j-1 AND side graph j-1 — the sort of its batches, behind their H2D copy — are done, and the
    # host has submitted it); the part of each gap spent waiting for the side chain is its side stall
    stt, eng.stall_timing = eng.stall_timing, None
    gpu_stall = {}
    if len(stt) > 2:
        gap = side = busy = 0.0
        for j in range(1, len(stt)):
            s0, e0, d0 = stt[j - 1]
            s1, e1, _ = stt[j]
            g = e0.elapsed_time(s1)  # main end j-1 → main start j
            gap += max(0.0, g)
            side += min(max(0.0, g), max(0.0, e0.elapsed_time(d0)))
            busy += s1.elapsed_time(e1)
        span = stt[0][0].elapsed_time(stt[-1][1])
        gpu_stall = {"gpu_stall_fraction": round(gap / span, 4), "gpu_side_stall_fraction": round(side / span, 4),
                     "gpu_main_busy_fraction": round(busy / span, 4),
                     "host_copy_wait_s": round(getattr(eng, "host_copy_wait_s", 0.0), 4)}
    copy_ms = sum(c[0] for c in ct)
    h2d_ms = sum(c[3] for c in ct)
    out_copy = {"copy_stream_ms_per_group": round(copy_ms / max(len(ct), 1), 3),
                "copy_stream_h2d_ms_per_group": round(h2d_ms / max(len(ct), 1), 3),
                "copy_stream_parse_ms_per_group": round((copy_ms - h2d_ms) / max(len(ct), 1), 3),
                "copy_stream_h2d_GBps": round(sum(c[1] for c in ct) / max(h2d_ms, 1e-9) / 1e6, 2),
                "copy_stream_GBps": round(sum(c[1] for c in ct) / max(copy_ms, 1e-9) / 1e6, 2),
                "copy_stream_busy_fraction": round(copy_ms / (dt * 1e3), 3)} if ct else {}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "examples/sec", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "vs_eager_pytorch": round(value / EAGER_BASELINE[a.embedding_update], 3),
        "dtype": a.compute_dtype,
        "data": "synthetic Criteo-shape TFRecord files (39 fields, Zipf ids) through the C++ loader, random-init "
                "weights",
        "config": {"model": f"DeepFM Criteo-shape ({F} fields, {_human(a.feature_size)}-hash vocab, "
                            f"k={a.embedding_size}, mlp {a.deep_layers}, dropout keep {a.dropout}, {a.optimizer})",
                   "global_batch": B, "seq_len": F, "parallelism": "dp1", "engine": "fused",
                   "embedding_update": a.embedding_update, "input": "tfrecord", "steps_per_graph": S,
                   "loader_threads": a.loader_threads, "loader_hold": a.loader_hold,
                   "file_batches": nbat, "epochs": -(-(a.warmup + a.steps) // nbat)},
        "decode": "device" if raw else "host",
        "steady_examples_per_sec": round(steady, 1) if steady else None,
        "fill_ms": round((marks[0][0] - t0) * 1e3, 2) if marks else None,
        "loader_alone_examples_per_sec": round(loader_eps, 1),
        "host_decode_loader_alone_examples_per_sec": round(host_eps, 1),
        "input_stall_s": round(stall[0], 4),
        "input_stall_fraction": round(stall[0] / dt, 4),
        "data_gen_s": round(gen_s, 2),
        "world_size": 1, "backend": None,
    }
    out.update(out_copy)
    out.update(gpu_stall)
    if own:
        shutil.rmtree(d, ignore_errors=True)
    return out


if __name__ == "__main__":
    main()
