"""Estimator-style training engine (replaces tf.estimator.Estimator in PS:492-551 / HVD:402-493).

    est = Estimator(cfg)                  # builds the model, restores model_dir's latest checkpoint
    est.train(files, num_epochs)          # = DeepFM.train(input_fn(tr_files, …))
    est.evaluate(files)                   # = DeepFM.evaluate → {auc, auc_exact, loss, global_step}
    est.predict(files, pred_path)         # = DeepFM.predict → pred.txt ("%f\\n" per example, PS:531-533)
    est.export(servable_model_dir)        # = export_savedmodel (rank 0, PS:536-551)
    est.train_and_evaluate(tr, va)        # per-epoch train + all-rank eval (fixes Q7/Q8/Q13)

Engines: ``fused`` — the MI355X HIP path (rocfm.models.fused, one graph-replayed step per batch),
``torch`` — eager PyTorch (CPU, batch_norm beyond 4096 rows per GPU, or the GPU baseline); ``auto`` picks fused on a GPU
when the config allows it.  Multi-process runs (torchrun, one process per GPU) use data
parallelism (rocfm.parallel.dp); only rank 0 writes checkpoints/exports (HVD:402-415, 490).
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Callable, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import checkpoint as ckpt
from .config import Config
from .data.sharding import eval_shard, train_shard
from .data.tfrecord import TFRecordDataset
from .metrics import DeviceAUC, LossMean, TFStreamingAUC, exact_auc
from .models.deepfm import ModelSpec, init_params
from .ops import has_hip
from .optim import OptHParams
from .parallel.dist import RankInfo, rank_info_from_env
from .utils.fault import FaultInjector
from .utils.numerics import check_finite, check_ids, ids_check_enabled, numerics_check_enabled
from .utils.profiling import StepProfiler, StepTimer, trace_range
from .utils.watchdog import Watchdog

log = logging.getLogger("rocfm")


def _world() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


class Estimator:
    def __init__(self, cfg: Config, device: Optional[torch.device] = None, rank_info: Optional[RankInfo] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None, restore: bool = True):
        self.cfg = cfg.validate()
        self.info = rank_info or rank_info_from_env(cfg.worker_per_host or None)
        if device is None:
            device = torch.device("cuda", self.info.local_rank) if torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        # host threads next to the GPU (the loader's reader / worker threads and the pinned staging
        # buffers they first touch): the GPU's NUMA node, unless ROCFM_NUMA_BIND=0 (utils/numa.py,
        # profiles/r5_stream_queues.md)
        if self.device.type == "cuda" and os.environ.get("ROCFM_NUMA_BIND", "1") == "1":
            from .utils.numa import bind_to_gpu_node
            bind_to_gpu_node(self.device.index or 0)
        self.spec = ModelSpec.from_config(cfg)
        self.world = _world()
        self.hp = OptHParams(name=cfg.optimizer, lr=cfg.learning_rate)
        self.engine_name = self._pick_engine()
        if params is None and cfg.parallelism not in ("rowshard", "dp_owner", "async_ps"):
            params = init_params(self.spec, cfg.seed)
        P = params  # row-shard: None → every rank initialises only its own rows
        self.eng = self._build_engine(P)
        self._lr_scale = 1.0
        if self.world > 1 and cfg.lr_scaling == "linear":
            self._lr_scale = float(self.world)
            self.eng.set_lr_scale(self._lr_scale)  # HVD:171 learning_rate * hvd.size()
        self.model_dir = cfg.effective_model_dir
        self._last_save_t = time.time()
        self.metrics_fh = None
        if cfg.metrics_file and self.info.is_chief:
            os.makedirs(os.path.dirname(os.path.abspath(cfg.metrics_file)), exist_ok=True)
            self.metrics_fh = open(cfg.metrics_file, "a")
        self._tb = {}  # TensorBoard writers by subdirectory ("" = train, "eval"), chief only
        if restore and self.model_dir:
            self.restore()
        # steps already trained by the job this estimator resumes (fast-forward on restart, below)
        self._resume_step = self.global_step

    # ---- construction -------------------------------------------------------------------------
    def _pick_engine(self) -> str:
        e = self.cfg.engine
        if self.cfg.parallelism == "async_ps":  # the eager step against the parameter servers
            return "torch"
        if e == "auto":
            # batch_norm runs fused while the batch's row-kernel grid fits on the chip at once (its
            # moments are reduced with grid barriers): ≤ 4096 rows per GPU
            ok = (self.device.type == "cuda" and has_hip() and len(self.spec.layers) <= 6
                  and self.spec.embedding_size <= 63 and self.spec.field_size <= 64
                  and not (self.cfg.batch_norm and self.cfg.batch_size > 4096))
            return "fused" if ok else "torch"
        if e == "fused" and self.device.type != "cuda":
            raise ValueError("engine=fused needs a GPU")
        return e

    def _build_engine(self, P):
        cfg = self.cfg
        cap = cfg.exchange_capacity or None
        if cfg.parallelism == "async_ps":  # (RPC initialised by rocfm.parallel.async_ps.run_job)
            from .parallel.async_ps import AsyncPSWorker

            return AsyncPSWorker(self.spec, self.hp, cfg.num_ps, self.device, embedding_update=cfg.embedding_update,
                                 dropout_seed=cfg.seed + 7919 * self.info.rank)
        if cfg.parallelism in ("rowshard", "dp_owner"):
            from .parallel.emb_shard import FusedRowShard, TorchRowShard

            if self.engine_name == "fused":
                return FusedRowShard(self.spec, self.hp, cfg.batch_size, self.device, params=P,
                                     embedding_update=cfg.embedding_update, seed=cfg.seed,
                                     use_graph=cfg.use_hip_graph, capacity=cap, compute_dtype=cfg.compute_dtype, table_dtype=cfg.table_dtype,
                                     exchange=cfg.dp_exchange, staleness=cfg.ps_staleness,
                                     hot_rows=cfg.hot_rows, replicate_table=cfg.parallelism == "dp_owner")
            if cfg.ps_staleness or cfg.hot_rows or cfg.table_dtype != "f32":
                raise ValueError("ps_staleness / hot_rows / table_dtype=bf16 need the fused engine (a GPU)")
            return TorchRowShard(self.spec, self.hp, self.device, embedding_update=cfg.embedding_update, params=P,
                                 seed=cfg.seed)
        if self.engine_name == "fused":
            if self.world > 1 or cfg.parallelism in ("dp", "dense_dp"):
                from .parallel.dp import FusedDataParallel

                mode = "dense_dp" if cfg.parallelism == "dense_dp" else "dp"
                return FusedDataParallel(self.spec, self.hp, cfg.batch_size, self.device, params=P,
                                         embedding_update=cfg.embedding_update, mode=mode, seed=cfg.seed,
                                         use_graph=cfg.use_hip_graph, capacity=cap, compute_dtype=cfg.compute_dtype, table_dtype=cfg.table_dtype,
                                         exchange=cfg.dp_exchange)
            from .models.fused import FusedDeepFM

            return FusedDeepFM(self.spec, self.hp, cfg.batch_size, self.device, embedding_update=cfg.embedding_update,
                               seed=cfg.seed, params=P, use_graph=cfg.use_hip_graph, compute_dtype=cfg.compute_dtype, table_dtype=cfg.table_dtype)
        from .models.torch_engine import TorchDeepFM

        if cfg.table_dtype != "f32":
            raise ValueError("table_dtype=bf16 needs the fused engine (a GPU)")
        eng = TorchDeepFM(self.spec, self.hp, self.device, embedding_update=cfg.embedding_update, params=P,
                          seed=cfg.seed, dropout_seed=cfg.seed + 7919 * self.info.rank)
        if self.world > 1:
            from .parallel.dist import broadcast_tensors
            from .parallel.dp import attach_torch_dp

            broadcast_tensors(list(eng.P.values()))
            attach_torch_dp(eng, cfg.embedding_update)
        return eng

    # ---- data ---------------------------------------------------------------------------------
    def _dataset(self, files: Sequence[str], num_epochs: int, training: bool, drop_remainder: bool = True):
        cfg = self.cfg
        if training:
            count, index = train_shard(self.info, cfg.pipe_mode, cfg.enable_s3_shard, cfg.enable_data_multi_path)
        else:
            count, index = eval_shard(self.info)
        return TFRecordDataset(files, cfg.field_size, cfg.batch_size, cfg.feature_size, num_epochs=num_epochs,
                               shard_count=count, shard_index=index, drop_remainder=drop_remainder,
                               num_threads=max(1, min(cfg.num_threads, 16)), verify_crc=cfg.crc_check,
                               skip_bad=cfg.on_bad_record == "skip",
                               shuffle_buffer=(cfg.batch_size * 8 if (training and cfg.perform_shuffle) else 0),
                               seed=cfg.seed + self.info.rank, stream_mode=bool(cfg.pipe_mode),
                               shard_policy=cfg.shard_policy if training else "record",
                               hold=2)  # _device_batches syncs batch t's H2D copy while t+1 is current

    def _host_batches(self, ds: Iterable):
        chk = ids_check_enabled()
        for b in ds:
            if chk:
                check_ids(b[0], self.cfg.feature_size)
            yield b

    def _device_batches(self, ds: Iterable):
        """Host (pinned) batches → device tensors.  Batch t's H2D copy is waited for in the body
        of batch t+1, so the loader must keep t's pinned slot until batch t+2 is requested
        (``hold=2`` in _dataset); with hold=1 the slot was recycled by the decoders while its copy
        could still be queued behind the GPU's work (a rare corrupted batch)."""
        if getattr(ds, "hold", 2) < 2:
            raise ValueError("_device_batches needs a dataset with hold >= 2")
        prev_ev = None
        chk = ids_check_enabled()
        for ids, vals, labels in ds:
            if chk:
                check_ids(ids, self.cfg.feature_size)
            if prev_ev is not None:
                prev_ev.synchronize()
            if self.device.type == "cuda":
                d = (ids.to(self.device, non_blocking=True), vals.to(self.device, non_blocking=True),
                     labels.to(self.device, non_blocking=True))
                prev_ev = torch.cuda.Event()
                prev_ev.record()
            else:
                d = (ids.clone(), vals.clone(), labels.clone())
            yield d

    # ---- training ------------------------------------------------------------------------------
    @property
    def global_step(self) -> int:
        return self.eng.global_step()

    def train(self, files: Sequence[str], num_epochs: int = 1, max_steps: Optional[int] = None,
              hooks: Sequence[Callable] = (), skip_batches: int = 0) -> Dict[str, float]:
        """Train over ``num_epochs`` passes of ``files`` (this rank's shard).  ``skip_batches``
        fast-forwards the input stream (resume after a restart without re-training consumed data;
        the reference re-reads from the start, an Estimator limitation rocfm does not copy)."""
        cfg = self.cfg
        S = 16
        ds = self._dataset(files, num_epochs, training=True)
        # several ranks: every step is collective, so the ranks agree on a common number of
        # batches per epoch (the minimum of their shards'; the surplus of longer shards is dropped
        # each epoch, like drop_remainder)
        per_epoch = self._agreed_epoch_batches(ds)
        limit = None
        if per_epoch is not None:
            ds.kw["max_batches_per_epoch"] = per_epoch
            limit = max(0, per_epoch * num_epochs - skip_batches)
        if max_steps:
            limit = max_steps if limit is None else min(limit, max_steps)
        # fused engine + graphs: groups of S batches decoded into one pinned ring, moved by the
        # engine with one copy per group (copy stream → HBM ring) and trained S steps per graph
        # launch — on one GPU, and with several ranks (DP / row-shard graphs with the exchange
        # inline) whenever every rank streams an agreed number of batches and the exchanges are
        # capturable (p2p, or RCCL)
        stream = self.engine_name == "fused" and cfg.use_hip_graph and self.device.type == "cuda" \
            and hasattr(self.eng, "train_stream") and getattr(self.eng, "graph_collectives", True) \
            and (self.world == 1 or limit is not None)
        # device-side Example parsing: the loader hands the graphs' copy stream undecoded payloads
        # (raw_groups) and the GPU parses them (decode.hip); the host only frames, checks CRCs and
        # copies bytes.  Not for pipe mode, skip_bad or the decoded on-disk cache (host batches).
        raw = stream and cfg.device_decode and not cfg.pipe_mode and cfg.on_bad_record != "skip" \
            and not cfg.decoded_cache_dir and self._device_decode_fits()

        def groups_of(d, skip=0, lim=None):
            if raw:
                return d.raw_groups(S, hold=2, skip=skip, limit=lim)
            return self._host_batches(d.groups(S, hold=2, skip=skip, limit=lim))

        if stream:
            batches = groups_of(ds, skip_batches, limit)
        else:
            batches = self._device_batches(_skip(ds, skip_batches))
            if limit is not None:
                batches = _take(batches, limit)
            elif self.world > 1:
                batches = self._lockstep(batches)
        t0 = time.time()
        last_t, last_step = t0, self.global_step
        n0 = self.global_step
        loss = float("nan")
        timer = StepTimer()
        prof = StepProfiler(cfg.profile_steps, os.path.join(self.model_dir or ".", "profile")) \
            if cfg.profile_steps else None
        faults = FaultInjector(self.info.rank)
        wd = Watchdog(cfg.watchdog_s).start() if cfg.watchdog_s > 0 else None
        batches = _timed(batches, timer)

        def log_line(step, value):
            nonlocal last_t, last_step, loss
            loss = value
            if faults.corrupt_loss(step):
                loss = float("nan")
            if numerics_check_enabled():
                check_finite(loss, step)
            now = time.time()
            eps = (step - last_step) * cfg.batch_size * self.world / max(now - last_t, 1e-9)
            _, stall = timer.lap()
            last_t, last_step = now, step
            self._summary("", step, {"loss": loss, "global_step/sec": eps / (cfg.batch_size * self.world),
                                     "examples/sec": eps, "input_stall": stall})
            self._log({"event": "train", "global_step": step, "loss": loss, "examples_per_sec": eps,
                       "examples_per_sec_per_gpu": eps / self.world, "lr": self.hp.lr * self._lr_scale,
                       "input_stall": round(stall, 4)})

        def after_step(step=None, log=True):
            step = self.global_step if step is None else step
            if wd is not None:
                wd.beat()
            if prof is not None:
                prof.step(step)
            if log and cfg.log_steps and step % cfg.log_steps == 0:
                log_line(step, self.batch_loss())
            if cfg.save_checkpoints_steps and step % cfg.save_checkpoints_steps == 0:
                self.save()
            elif cfg.save_checkpoints_secs and self._time_to_save(step):
                self.save()
            for h in hooks:
                h(self, step)
            if faults:
                faults.after_step(step)

        # decoded-epoch HBM cache (several epochs of the same files, no shuffle; every rank its own
        # shard): epoch 1 streams from the loader into an HBM ring sized for the whole epoch,
        # epochs 2.. replay it from HBM (the reference's tf.data re-reads and re-parses every
        # epoch, PS:147-165).  Several ranks cache their agreed per-epoch batches.
        cache_nb = 0
        if stream and num_epochs > 1 and cfg.hbm_cache and not cfg.perform_shuffle and skip_batches == 0 \
                and not cfg.pipe_mode and not max_steps and (self.world == 1 or per_epoch is not None):
            ds1 = self._dataset(files, 1, training=True)
            if per_epoch is not None:
                ds1.kw["max_batches_per_epoch"] = per_epoch
            nb = ds1.num_batches()
            if nb and nb * cfg.batch_size * (8 * cfg.field_size + 4) <= cfg.hbm_cache_gb * (1 << 30):
                cache_nb = nb
                batches = _timed(groups_of(ds1), timer)
        # pre-decoded on-disk cache (rocfm.data.cache): the first pass over this rank's shard is
        # written through, every later pass (later epochs, restarted or repeated jobs) memory-maps it
        if stream and cfg.decoded_cache_dir and not cfg.perform_shuffle and not cfg.pipe_mode \
                and cfg.on_bad_record != "skip":
            from .data.cache import DecodedCache, cached_epochs

            dc = DecodedCache.for_dataset(self._dataset(files, 1, training=True), cfg.decoded_cache_dir)
            first = lambda sk, lim: self._dataset(files, 1, training=True).groups(S, hold=2, skip=sk, limit=lim)
            if cache_nb:  # the HBM cache replays epochs 2..: only the first pass comes from the loader / disk
                src = cached_epochs(dc, first, 1, S, hold=2)
            else:
                src = cached_epochs(dc, first, num_epochs, S, hold=2, skip=skip_batches, limit=limit)
            batches = _timed(self._host_batches(src), timer)
            self._log({"event": "decoded_cache", "path": dc.path, "complete": dc.complete()})
        try:
            with trace_range("train"):
                if stream:
                    # single GPU: batches staged into an HBM ring, S steps per graph launch.  Loss
                    # logging must not drain the queue of launched graphs: the loss after the graph
                    # that crosses a log_steps boundary is fetched asynchronously and logged (with
                    # that graph's last step) once ready.
                    pend = []

                    def flush(block):
                        while pend and (block or pend[0][1].query()):
                            st, ev, host = pend.pop(0)
                            ev.synchronize()
                            log_line(st, float(host[0]))

                    def after_graph(first, n):
                        for st in range(first + 1, first + n + 1):
                            after_step(st, log=False)
                        if cfg.log_steps and (first + n) // cfg.log_steps > first // cfg.log_steps:
                            pend.append((first + n, *self.eng.loss_async()))
                        flush(False)

                    self.eng.train_stream(batches, S, after_steps=after_graph, hold=2, ring_batches=cache_nb)
                    if cache_nb:
                        ids, vals, labels = self.eng.stream_ring()
                        for _ in range(num_epochs - 1):
                            g0 = self.global_step
                            self.eng.attach_pool(ids[:cache_nb], vals[:cache_nb], labels[:cache_nb],
                                                 start=(-g0) % cache_nb)
                            left = cache_nb
                            while left > 0:
                                n = min(S, left)
                                first = self.global_step
                                self.eng.train_steps(n, S)
                                after_graph(first, n)
                                left -= n
                        self._log({"event": "hbm_cache", "batches": cache_nb, "epochs_from_cache": num_epochs - 1})
                    flush(True)
                elif self.engine_name == "fused":
                    it = self.eng.train_on(batches) if not hasattr(self.eng, "eng") else self._dp_train_on(batches)
                    for _ in it:
                        after_step()
                else:
                    for ids, vals, labels in batches:
                        self.eng.train_step(ids, vals, labels)
                        after_step()
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                if hasattr(self.eng, "check"):  # sticky device error flags (exchange overflow, BN barrier)
                    self.eng.check()
        finally:
            if wd is not None:
                wd.stop()
            if prof is not None:
                prof.close()
        steps = self.global_step - n0
        dt = time.time() - t0
        out = {"global_step": self.global_step, "steps": steps,
               "examples_per_sec": steps * cfg.batch_size * self.world / max(dt, 1e-9)}
        if steps > 0:
            out["loss"] = self.batch_loss()
        if self.model_dir:
            self.save()
        self._log({"event": "train_end", **out})
        return out

    # ---- multi-rank step agreement -----------------------------------------------------------
    def _ctrl_group(self):
        """A gloo group for host-side control messages (never touches the GPU stream)."""
        if getattr(self, "_ctrl", None) is None:
            self._ctrl = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
        return self._ctrl

    def _device_decode_fits(self) -> bool:
        """The device Example parser's LDS stage fits this schema on this GPU (decode.hip
        decode_fits: ≤ 192 fields and the opt-in LDS limit); otherwise the host parses."""
        from .ops import hip

        H = hip()
        return H is not None and hasattr(H, "decode_fits") and bool(H.decode_fits(self.cfg.field_size))

    def _agreed_epoch_batches(self, ds) -> Optional[int]:
        """Every rank must run the same number of synchronous steps (each step is a collective).
        File mode: the minimum over ranks of the shard's batches per epoch (records counted from
        the files' indexes); the surplus batches of longer shards are dropped every epoch, like
        drop_remainder.  None at world 1, and in pipe mode / with skip_bad (lockstep instead)."""
        if self.world == 1:
            return None
        n = ds.batches_per_epoch() if self.cfg.on_bad_record != "skip" else None
        t = torch.tensor([n if n is not None else -1], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._ctrl_group())
        return int(t.item()) if int(t.item()) >= 0 else None

    def _time_to_save(self, step: int) -> bool:
        """Time-based checkpoint cadence (Estimator's save_checkpoints_secs).  Saving is
        collective (state gathers, barriers), so with several ranks the decision is rank 0's
        clock, broadcast on the host control group at an agreed step cadence
        (``ckpt_poll_steps``); every rank then saves at the same step.  Deciding on each rank's
        own clock let two ranks cross the interval on different steps and deadlock."""
        due = time.time() - self._last_save_t > self.cfg.save_checkpoints_secs
        if self.world == 1:
            return due
        poll = max(1, int(self.cfg.ckpt_poll_steps))
        if step % poll != 0:
            return False
        t = torch.tensor([1 if due else 0], dtype=torch.int64)
        dist.broadcast(t, src=0, group=self._ctrl_group())
        return bool(int(t.item()))

    def _lockstep(self, batches):
        """Stream mode (or skip_bad): agree per step, on the host control group, that every rank
        still has a batch."""
        it = iter(batches)
        while True:
            b = next(it, None)
            t = torch.tensor([0 if b is None else 1], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._ctrl_group())
            if int(t.item()) == 0:
                return
            yield b

    def _dp_train_on(self, batches):
        """FusedDataParallel: same one-batch-ahead ring protocol as FusedDeepFM.train_on."""
        it = iter(batches)
        cur = next(it, None)
        if cur is None:
            return
        self.eng.load_batch(*cur)
        nxt = next(it, None)
        while True:
            if nxt is not None:
                self.eng.push_batch(*nxt)
            self.eng.train_step()
            yield
            if nxt is None:
                break
            nxt = next(it, None)

    def batch_loss(self) -> float:
        """Loss of the last training batch incl. the full-table L2 terms (PS:275-279)."""
        return self.eng.batch_loss(include_l2=True)

    # ---- evaluation / prediction ------------------------------------------------------------
    @torch.no_grad()
    def _predict_stream(self, files, training_shard: bool = False, drop_remainder: bool = True):
        ds = self._dataset(files, 1, training=training_shard, drop_remainder=drop_remainder)
        batches = self._device_batches(ds)
        if getattr(self.eng, "collective_predict", False) and self.world > 1:
            # row-shard inference is collective: ranks with no batch left join with empty ones
            it = iter(batches)
            while True:
                b = next(it, None)
                t = torch.tensor([0 if b is None else 1], dtype=torch.int64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self._ctrl_group())
                if int(t.item()) == 0:
                    return
                if b is None:
                    F = self.cfg.field_size
                    b = (torch.zeros(0, F, dtype=torch.int32, device=self.device),
                         torch.zeros(0, F, device=self.device), torch.zeros(0, device=self.device))
                p, lr = self.eng.predict_batch(*b)
                if len(p):
                    yield p, lr, b[2]
            return
        for ids, vals, labels in batches:
            p, lr = self.eng.predict_batch(ids, vals, labels)
            yield p, lr, labels

    @torch.no_grad()
    def evaluate(self, files: Sequence[str], exact: bool = True) -> Dict[str, float]:
        """AUC (TF 200-threshold + exact) and mean loss over the eval files, sharded over all ranks."""
        on_gpu = self.device.type == "cuda" and has_hip()
        auc = DeviceAUC(self.device) if on_gpu else TFStreamingAUC()
        lm = LossMean()
        preds, labs = [], []
        with trace_range("evaluate"):
            for p, lr, labels in self._predict_stream(files):
                if on_gpu:  # histogram + loss sums on the device: no per-batch host sync
                    auc.update(labels, p, lr)
                else:
                    auc.update(labels, p)
                    lm.update(float(lr.double().mean()), len(p))
                if exact:
                    preds.append(p.float())
                    labs.append(labels.float().to(p.device))
        if on_gpu:
            lm.total, lm.count = auc.loss_total()
            auc = auc.streaming()
        preds = [torch.cat(preds).cpu()] if preds else []
        labs = [torch.cat(labs).cpu()] if labs else []
        l2 = self.eng.l2_value()
        state = auc.state()
        tot = np.array([lm.total, lm.count], np.float64)
        if self.world > 1:
            t = torch.from_numpy(np.concatenate([state.reshape(-1), tot]))
            t = t.to(self.device) if dist.get_backend() == "nccl" else t
            dist.all_reduce(t)
            t = t.cpu().numpy()
            state, tot = t[:-2].reshape(state.shape), t[-2:]
            auc.load_state(state)
        res = {"auc": auc.result(), "loss": float(tot[0] / max(tot[1], 1) + l2), "global_step": self.global_step,
               "examples": int(tot[1])}
        if exact:
            P = torch.cat(preds) if preds else torch.zeros(0)
            Y = torch.cat(labs) if labs else torch.zeros(0)
            if self.world > 1:
                P, Y = _gather_var(P), _gather_var(Y)
            res["auc_exact"] = exact_auc(Y, P) if len(P) else float("nan")
        self._summary("eval", self.global_step, {k: v for k, v in res.items() if k not in ("global_step", "examples")})
        self._log({"event": "eval", **res})
        return res

    @torch.no_grad()
    def predict(self, files: Sequence[str], pred_path: Optional[str] = None) -> torch.Tensor:
        """Probabilities for every (batched, drop_remainder) example; rank 0 writes ``pred.txt``."""
        out = [p.float().cpu() for p, _, _ in self._predict_stream(files)]
        probs = torch.cat(out) if out else torch.zeros(0)
        if self.world > 1:
            probs = _gather_var(probs)
        if pred_path and self.info.is_chief:
            with open(pred_path, "w") as f:
                for v in probs.tolist():
                    f.write("%f\n" % v)  # PS:531-533
        return probs

    def resume_point(self, files: Sequence[str], num_epochs: int):
        """(first epoch, batches to skip in it) for a job restored at ``_resume_step`` (file mode)."""
        done = self._resume_step
        if not done:
            return 0, 0
        per_epoch = self._dataset(files, 1, training=True).num_batches()
        if self.world > 1:
            # train() runs the MIN over ranks of the shard batch counts (_agreed_epoch_batches); the
            # resume split must use that same agreed count on every rank, or ranks with one
            # more batch per epoch skip differently and run different numbers of collective steps
            t = torch.tensor([per_epoch if per_epoch is not None else -1], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._ctrl_group())
            per_epoch = int(t.item()) if int(t.item()) >= 0 else None
        if not per_epoch:
            return 0, 0
        return min(done // per_epoch, num_epochs), done % per_epoch

    def train_and_evaluate(self, train_files, eval_files, num_epochs: Optional[int] = None):
        num_epochs = num_epochs or self.cfg.num_epochs
        results = []
        ep0, skip = self.resume_point(train_files, num_epochs)
        for ep in range(ep0, num_epochs):
            tr = self.train(train_files, 1, skip_batches=skip if ep == ep0 else 0)
            ev = self.evaluate(eval_files) if eval_files and self.cfg.eval_every_epoch else {}
            results.append({"epoch": ep, **tr, **{f"eval_{k}": v for k, v in ev.items()}})
        return results

    # ---- checkpoint / export ---------------------------------------------------------------------
    def state_dict(self):
        return self.eng.state_dict()

    def save(self) -> Optional[str]:
        with trace_range("checkpoint"):
            return self._save()

    def _save(self) -> Optional[str]:
        self._last_save_t = time.time()
        if not self.model_dir:
            return None
        sd = self.eng.state_dict()  # every rank participates (collectives / sync), rank 0 writes
        extra = {"config": {k: v for k, v in self.cfg.to_dict().items() if isinstance(v, (int, float, str, bool))}}
        step = int(sd["global_step"])
        if getattr(self.eng, "row_sharded", False) and self.world > 1:
            # one shard per rank (its rows + their global ids); rank 0 writes the manifest last
            rs = self.eng.row_sets()
            if not self.info.is_chief:
                ckpt.save_checkpoint(self.model_dir, sd, step, shard=(self.info.rank, self.world), row_sets=rs,
                                     write_index=False)
            dist.barrier(group=self._ctrl_group())
            path = None
            if self.info.is_chief:
                path = ckpt.save_checkpoint(self.model_dir, sd, step, self.cfg.keep_checkpoint_max,
                                            shard=(0, self.world), row_sets=rs, extra=extra,
                                            global_rows={k: self.cfg.feature_size for k in rs})
                self._log({"event": "checkpoint", "path": path})
            dist.barrier(group=self._ctrl_group())
            return path
        path = None
        if self.info.is_chief:
            path = ckpt.save_checkpoint(self.model_dir, sd, step, self.cfg.keep_checkpoint_max, extra=extra)
            self._log({"event": "checkpoint", "path": path})
        if self.world > 1:
            # replicas wait (GPU drained by state_dict) while rank 0 writes: no rank's exchange
            # kernel spins on a peer that is busy on the host
            dist.barrier(group=self._ctrl_group())
        return path

    def restore(self, prefix: Optional[str] = None) -> Optional[str]:
        prefix = prefix or ckpt.latest_checkpoint(self.model_dir)
        if not prefix:
            return None
        rows_for = self.eng.row_sets() if getattr(self.eng, "row_sharded", False) else None
        sd = ckpt.load_checkpoint(prefix, rows_for=rows_for)
        self.eng.load_state_dict(sd, strict=False)
        self._log({"event": "restore", "path": prefix, "global_step": self.global_step})
        return prefix

    def export(self, servable_model_dir: Optional[str] = None) -> Optional[str]:
        d = servable_model_dir or self.cfg.servable_model_dir
        if not d:
            return None
        cfgd = {"feature_size": self.cfg.feature_size, "field_size": self.cfg.field_size,
                "embedding_size": self.cfg.embedding_size, "deep_layers": self.cfg.deep_layers,
                "dropout": self.cfg.dropout, "batch_norm": self.cfg.batch_norm,
                "batch_norm_decay": self.cfg.batch_norm_decay, "loss_type": self.cfg.loss_type}
        if hasattr(self.eng, "iter_table_chunks"):
            # row-sharded tables: streamed, one gathered row range at a time (no rank holds a
            # whole table); the chief writes each range at its final offset
            V, K = self.cfg.feature_size, self.cfg.embedding_size
            w = ckpt.StreamedServable(d, self.eng.dense_parameters_tf(), {"fm_w": (V,), "fm_v": (V, K)}, cfgd) \
                if self.info.is_chief else None
            for a, fw, fv in self.eng.iter_table_chunks():  # collective
                if w is not None:
                    w.write_rows("fm_w", a, fw)
                    w.write_rows("fm_v", a, fv)
            if w is None:
                return None
            path = w.close()
            self._log({"event": "export", "path": path})
            return path
        params = self.eng.parameters_tf()
        if not self.info.is_chief:
            return None
        path = ckpt.export_servable(d, params, cfgd)
        self._log({"event": "export", "path": path})
        return path

    def close(self) -> None:
        """Release engine resources (captured graphs holding collectives) and the metrics file."""
        if hasattr(self.eng, "close"):
            self.eng.close()
        if self.metrics_fh:
            self.metrics_fh.close()
            self.metrics_fh = None
        for w in self._tb.values():
            w.close()
        self._tb = {}

    # ---- logging ------------------------------------------------------------------------------------
    def _summary(self, sub: str, step: int, values: dict) -> None:
        """Scalar summaries for TensorBoard (the Estimator's event files: model_dir, model_dir/eval)."""
        if not (self.cfg.tensorboard and self.info.is_chief and self.model_dir):
            return
        w = self._tb.get(sub)
        if w is None:
            from .utils.tensorboard import EventWriter

            w = self._tb[sub] = EventWriter(os.path.join(self.model_dir, sub) if sub else self.model_dir)
        w.scalars(int(step), values)

    def _log(self, rec: dict) -> None:
        if not self.info.is_chief:
            return
        log.info(json.dumps(rec))
        if self.metrics_fh:
            self.metrics_fh.write(json.dumps({"time": time.time(), **rec}) + "\n")
            self.metrics_fh.flush()


def _skip(it, n):
    """Drop the first ``n`` items (host batches: the loader recycles their slots at once)."""
    it = iter(it)
    for _ in range(n):
        if next(it, None) is None:
            break
    return it


def _timed(it, timer):
    """Yield from ``it`` while accounting the time spent waiting for each item (input stall)."""
    it = iter(it)
    while True:
        with timer.waiting():
            x = next(it, None)
        if x is None:
            return
        yield x


def _take(it, n):
    for i, x in enumerate(it):
        if i >= n:
            break
        yield x


def _gather_var(t: torch.Tensor) -> torch.Tensor:
    """all_gather of variable-length 1-D CPU tensors (rank-major)."""
    world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([t.numel()], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    m = int(max(int(x) for x in ns))
    pad = torch.zeros(m, dtype=t.dtype, device=dev)
    pad[: t.numel()] = t.to(dev)
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[: int(k)].cpu() for o, k in zip(outs, ns)])
