"""Asynchronous parameter server — the reference's PS-CPU job without a bound on staleness.

The reference's first job (``1-ps-cpu``; README:15-17, PS:461-521) is TF between-graph
replication: ``TF_CONFIG`` names ``ps`` and worker tasks, the Estimator places every variable on
the parameter servers, and every worker runs its own loop — read the variables it needs, compute
gradients on its batch, send them to the PS, which applies them on arrival.  Nothing synchronises
the workers: a worker's gradient is computed against whatever the PS held when it read, however
many other workers' updates landed since (unbounded staleness).  ``rocfm.parallel.emb_shard`` is
the GPU PS-equivalent with staleness 0 or 1; this module is the asynchronous one, over
``torch.distributed.rpc`` (TensorPipe), for CPU clusters like the reference's and for GPU workers
(the worker's step runs on its device; tensors travel through host memory).

Roles (``--parallelism async_ps --num_ps P``, one process per task, ``torchrun``):

* ranks ``0 .. P-1`` are parameter servers ``ps{p}``: ``fm_w`` / ``fm_v`` rows with
  ``id % P == p`` (local row ``id // P``) with their optimizer slots, and the MLP variables
  placed round-robin (TF's ``replica_device_setter`` placement) — every update is applied under
  the shard's lock (one apply at a time per shard; TF applies without locking by default);
* ranks ``P ..`` are workers ``worker{w}``: an :class:`rocfm.estimator.Estimator` whose engine
  is :class:`AsyncPSWorker` (same interface as the eager engine), reading its own ``1/W`` of the
  training files; worker 0 is the chief (restore, checkpoints, export, evaluation, PS:402-415).

Update semantics: the sparse engine's (``embedding_update=sparse``: the batch's unique rows,
lazy L2 on them, row-sparse optimizer, rocfm.models.torch_engine) applied on the PS with the PS's
current row values; the global step is the number of applies on ``ps0`` (every push reaches every
shard, so all shards count the same applies); Adam's bias correction uses it, as TF's
``beta1_power`` / ``beta2_power`` advance once per applied worker step.  As a TF worker's
``sess.run(train_op)`` returns once its own update is applied, a worker waits for its pushes
before its next pull (``max_inflight`` > 0 lets it run that many steps ahead of its own updates);
the staleness comes from the other workers.  With one worker the job is the single-process
sparse engine step for step (``tests/test_async_ps.py``).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from collections import OrderedDict, deque
from typing import Dict, List, Optional

import torch

from ..models.deepfm import ModelSpec, data_loss, forward, init_params, is_trainable, l2_terms, param_shapes
from ..optim import OptHParams, apply_dense, apply_rows, init_slots, slot_names

log = logging.getLogger("rocfm")

_SHARD = None  # this process's ParameterShard (PS ranks)
_READY = threading.Event()  # ps0: the chief has restored / initialised the variables


def ps_name(p: int) -> str:
    return f"ps{p}"


def worker_name(w: int) -> str:
    return f"worker{w}"


def dense_placement(spec: ModelSpec, n_ps: int) -> Dict[str, int]:
    """MLP / bias / batch-norm variables → PS index, round-robin in variable order."""
    names = [k for k in param_shapes(spec) if k not in ("fm_w", "fm_v")]
    return {k: i % n_ps for i, k in enumerate(names)}


class ParameterShard:
    """One PS task's variables: table rows ``id % n_ps == p`` and its round-robin MLP variables."""

    def __init__(self, spec: ModelSpec, hp: OptHParams, p: int, n_ps: int, seed: int):
        self.spec, self.hp, self.p, self.n_ps = spec, hp, p, n_ps
        full = init_params(spec, seed)  # the same initial values as every other engine
        self.place = dense_placement(spec, n_ps)
        self.P: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        self.P["fm_w"] = full["fm_w"][p::n_ps].clone()
        self.P["fm_v"] = full["fm_v"][p::n_ps].clone()
        for k, q in self.place.items():
            if q == p:
                self.P[k] = full[k].clone()
        self.slots = {k: init_slots(hp, v) for k, v in self.P.items() if is_trainable(k)}
        self.applies = 0
        self.lock = threading.Lock()

    def pull(self, rows: torch.Tensor, names: List[str]):
        with self.lock:
            return (self.P["fm_w"][rows].clone(), self.P["fm_v"][rows].clone(),
                    {k: self.P[k].clone() for k in names})

    def push(self, rows: torch.Tensor, gw: torch.Tensor, gv: torch.Tensor, dense: Dict[str, torch.Tensor],
             lr_scale: float) -> int:
        hp = self.hp
        if lr_scale != 1.0:
            hp = OptHParams(**self.hp.__dict__)
            hp.lr = self.hp.lr * lr_scale
        with self.lock:
            step = self.applies + 1
            if rows.numel():
                l2 = self.spec.l2_reg  # lazy L2 on the touched rows, with the PS's current values
                apply_rows(hp, self.P["fm_w"], rows, gw + l2 * self.P["fm_w"][rows], self.slots["fm_w"], step)
                apply_rows(hp, self.P["fm_v"], rows, gv + l2 * self.P["fm_v"][rows], self.slots["fm_v"], step)
            for k, g in dense.items():
                apply_dense(hp, self.P[k], g, self.slots[k], step)
            self.applies = step
            return step

    def state(self) -> dict:
        with self.lock:
            return {"P": {k: v.clone() for k, v in self.P.items()},
                    "slots": {k: [s.clone() for s in v] for k, v in self.slots.items()},
                    "applies": self.applies}

    def load(self, st: dict) -> None:
        with self.lock:
            for k, v in st["P"].items():
                self.P[k].copy_(v)
            for k, ss in st.get("slots", {}).items():
                for s, v in zip(self.slots[k], ss):
                    s.copy_(v)
            self.applies = int(st["applies"])


# ---- RPC entry points (run on the PS process, against its shard) --------------------------------
def _pull(rows, names):
    return _SHARD.pull(rows, names)


def _push(rows, gw, gv, dense, lr_scale):
    return _SHARD.push(rows, gw, gv, dense, lr_scale)


def _state():
    return _SHARD.state()


def _load(st):
    _SHARD.load(st)


def _applies():
    return _SHARD.applies


_DONE = [0]  # ps0: workers that finished training
_DONE_LOCK = threading.Lock()  # (RPC requests run on the agent's thread pool)


def _set_ready():
    _READY.set()


def _worker_done():
    with _DONE_LOCK:
        _DONE[0] += 1
        return _DONE[0]


def _done_count():
    return _DONE[0]


def _is_ready():
    return _READY.is_set()


_FAILED = [0]  # ps0: workers that raised (their peers stop waiting for them)


def _worker_failed():
    with _DONE_LOCK:
        _FAILED[0] += 1
        return _FAILED[0]


def _failed_count():
    return _FAILED[0]


def _wait_ps0(pred, what: str, timeout_s: float) -> None:
    """Poll ps0 until ``pred()`` (an RPC) holds; raise if a worker has reported a failure or after
    ``timeout_s`` — a dead peer must fail the job, not hang it (then rpc.shutdown hangs too)."""
    from torch.distributed import rpc

    deadline = time.time() + max(1.0, float(timeout_s))
    while not pred():
        if rpc.rpc_sync(ps_name(0), _failed_count) > 0:
            raise RuntimeError(f"async PS: a worker failed while this worker waited for {what}")
        if time.time() > deadline:
            raise TimeoutError(f"async PS: waited {timeout_s:.0f} s for {what} (dist_timeout_s)")
        time.sleep(0.05)


class AsyncPSWorker:
    """Worker-side engine: the eager sparse step against the parameter servers (duck-types
    rocfm.models.torch_engine.TorchDeepFM for the Estimator)."""

    def __init__(self, spec: ModelSpec, hp: OptHParams, n_ps: int, device="cpu", embedding_update: str = "sparse",
                 dropout_seed: int = 1234, max_inflight: int = 0):
        from torch.distributed import rpc

        if embedding_update != "sparse":
            raise ValueError("async_ps trains with embedding_update=sparse (a worker never holds the whole table)")
        if spec.batch_norm:
            raise ValueError("async_ps does not support batch_norm (moving statistics would need assign pushes)")
        self.rpc = rpc
        self.spec, self.hp, self.n_ps = spec, hp, int(n_ps)
        self.device = torch.device(device)
        self.embedding_update = embedding_update
        self.place = dense_placement(spec, self.n_ps)
        self.names_of = [[k for k, q in self.place.items() if q == p] for p in range(self.n_ps)]
        self.trainable = [k for k in self.place if is_trainable(k)]
        self.gen = torch.Generator(device=self.device).manual_seed(dropout_seed)
        self.lr_scale = 1.0
        self.t = 0  # this worker's steps
        self.max_inflight = max(0, int(max_inflight))
        self.inflight: "deque" = deque()

    # ---- helpers ------------------------------------------------------------------------------
    def _split(self, uniq: torch.Tensor):
        owner = torch.remainder(uniq, self.n_ps)
        return [(owner == p).nonzero().squeeze(1) for p in range(self.n_ps)], torch.div(uniq, self.n_ps,
                                                                                       rounding_mode="floor")

    def _pull(self, uniq: torch.Tensor):
        sels, local = self._split(uniq)
        futs = [self.rpc.rpc_async(ps_name(p), _pull, args=(local[sels[p]], self.names_of[p]))
                for p in range(self.n_ps)]
        rw = torch.empty(uniq.numel(), dtype=torch.float32)
        rv = torch.empty(uniq.numel(), self.spec.embedding_size, dtype=torch.float32)
        dense: Dict[str, torch.Tensor] = {}
        for p, f in enumerate(futs):
            w, v, d = f.wait()
            rw[sels[p]] = w
            rv[sels[p]] = v
            dense.update(d)
        dev = self.device
        return rw.to(dev), rv.to(dev), {k: v.to(dev) for k, v in dense.items()}, sels, local

    def _drain(self, keep: int) -> None:
        while len(self.inflight) > keep:
            self.inflight.popleft().wait()

    # ---- engine interface ---------------------------------------------------------------------
    def set_lr_scale(self, s: float) -> None:
        self.lr_scale = float(s)

    def train_step(self, ids: torch.Tensor, vals: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        labels = labels.to(self.device).float()
        uniq, inv = torch.unique(ids.reshape(-1), return_inverse=True)
        inv = inv.reshape(ids.shape)
        rw, rv, dense, sels, local = self._pull(uniq.cpu())
        rw.requires_grad_(True)
        rv.requires_grad_(True)
        params = {"fm_w": rw, "fm_v": rv}  # (rows are passed pre-gathered)
        for k, v in dense.items():
            params[k] = v.requires_grad_(True) if k in self.trainable else v
        y = forward(params, ids, vals, self.spec, train=True, gen=self.gen, rows_w=rw[inv], rows_v=rv[inv])
        loss = data_loss(y, labels, self.spec.loss_type)
        loss.backward()
        gw, gv = rw.grad.detach().cpu(), rv.grad.detach().cpu()
        for p in range(self.n_ps):
            sel = sels[p]
            dg = {k: params[k].grad.detach().cpu() for k in self.names_of[p] if k in self.trainable}
            self.inflight.append(self.rpc.rpc_async(ps_name(p), _push,
                                                    args=(local[sel], gw[sel], gv[sel], dg, self.lr_scale)))
        self._drain(self.max_inflight * self.n_ps)  # (0: this step's update is applied before the next pull)
        self.t += 1
        self._last_loss_t = loss.detach()
        return loss.detach()

    def flush(self) -> None:
        """Wait until every push of this worker has been applied."""
        self._drain(0)

    def batch_loss(self, include_l2: bool = True) -> float:
        if not hasattr(self, "_last_loss_t"):
            return float("nan")
        v = float(self._last_loss_t)
        return v + self.l2_value() if include_l2 else v

    @torch.no_grad()
    def predict_batch(self, ids, vals, labels=None):
        ids = ids.to(self.device).long()
        vals = vals.to(self.device).float()
        uniq, inv = torch.unique(ids.reshape(-1), return_inverse=True)
        rw, rv, dense, _, _ = self._pull(uniq.cpu())
        params = dict(dense)
        params["fm_w"], params["fm_v"] = rw, rv
        y = forward(params, ids, vals, self.spec, train=False, rows_w=rw[inv.reshape(ids.shape)],
                    rows_v=rv[inv.reshape(ids.shape)])
        p = torch.sigmoid(y)
        if labels is None:
            return p, torch.zeros_like(p)
        labels = labels.to(self.device).float()
        if self.spec.loss_type == "log_loss":
            lr = torch.clamp(y, min=0) - y * labels + torch.log1p(torch.exp(-y.abs()))
        else:
            lr = (p - labels) ** 2
        return p, lr

    def global_step(self) -> int:
        return int(self.rpc.rpc_sync(ps_name(0), _applies))

    def _gather(self):
        self.flush()
        sts = [self.rpc.rpc_sync(ps_name(p), _state) for p in range(self.n_ps)]
        V, K = self.spec.feature_size, self.spec.embedding_size
        full = init_params(self.spec, 0)  # shapes / names only; every value is overwritten
        slots = {k: init_slots(self.hp, v) for k, v in full.items() if is_trainable(k)}
        for p, st in enumerate(sts):
            for k in ("fm_w", "fm_v"):
                full[k][p::self.n_ps] = st["P"][k]
                for s, v in zip(slots[k], st["slots"].get(k, [])):
                    s[p::self.n_ps] = v
            for k in self.names_of[p]:
                full[k].copy_(st["P"][k])
                for s, v in zip(slots.get(k, []), st["slots"].get(k, [])):
                    s.copy_(v)
        assert full["fm_v"].shape == (V, K)
        return full, slots, int(sts[0]["applies"])

    def state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        full, slots, step = self._gather()
        sd: "OrderedDict[str, torch.Tensor]" = OrderedDict((k, v.clone()) for k, v in full.items())
        for si, sn in enumerate(slot_names(self.hp.name)):
            for k in slots:
                sd[f"{k}/{sn}"] = slots[k][si].clone()
        sd["global_step"] = torch.tensor(step, dtype=torch.int64)
        if self.hp.name == "Adam":
            sd["beta1_power"] = torch.tensor(self.hp.beta1 ** (step + 1), dtype=torch.float32)
            sd["beta2_power"] = torch.tensor(self.hp.beta2 ** (step + 1), dtype=torch.float32)
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        self.flush()
        step = int(sd["global_step"]) if "global_step" in sd else 0
        names = slot_names(self.hp.name)
        for p in range(self.n_ps):
            P, S = {}, {}
            for k in ["fm_w", "fm_v"] + self.names_of[p]:
                if k not in sd:
                    if strict:
                        raise KeyError(f"checkpoint is missing {k}")
                    continue
                v = sd[k]
                P[k] = v[p::self.n_ps].clone() if k in ("fm_w", "fm_v") else v.clone()
                if is_trainable(k):
                    ss = []
                    for sn in names:
                        key = f"{k}/{sn}"
                        if key not in sd:
                            if strict:
                                raise KeyError(f"checkpoint is missing {key}")
                            ss = None
                            break
                        s = sd[key]
                        ss.append(s[p::self.n_ps].clone() if k in ("fm_w", "fm_v") else s.clone())
                    if ss is not None:
                        S[k] = ss
            self.rpc.rpc_sync(ps_name(p), _load, args=({"P": P, "slots": S, "applies": step},))

    def parameters_tf(self) -> "OrderedDict[str, torch.Tensor]":
        full, _, _ = self._gather()
        return OrderedDict((k, v.clone()) for k, v in full.items())

    def l2_value(self) -> float:
        full, _, _ = self._gather()
        return float(l2_terms(full, self.spec.l2_reg))

    def close(self) -> None:
        self.flush()


# ---- the job ------------------------------------------------------------------------------------
def _rpc_init(name: str, rank: int, world: int, timeout_s: float) -> None:
    from torch.distributed import rpc

    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True":
        # no launcher store: rank 0 hosts the RPC rendezvous store next to MASTER_PORT; under
        # torchrun every rank joins the agent's store at MASTER_PORT (no process group uses it)
        port += int(os.environ.get("ROCFM_RPC_PORT_OFFSET", "1"))
    opts = rpc.TensorPipeRpcBackendOptions(init_method=f"tcp://{addr}:{port}", rpc_timeout=timeout_s,
                                           num_worker_threads=16)
    rpc.init_rpc(name, rank=rank, world_size=world, rpc_backend_options=opts)


def run_job(cfg, task_fn=None) -> dict:
    """Run this process's task of an async-PS job (ranks from RANK / WORLD_SIZE).

    PS ranks build their shard and serve until every worker has finished.  Worker ranks build an
    Estimator on an :class:`AsyncPSWorker` (``task_fn(est, worker_index, n_workers)`` runs the
    task; default: rocfm.cli's train / eval / infer / export flow) and return its result."""
    from torch.distributed import rpc

    from ..estimator import Estimator
    from .dist import RankInfo

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    n_ps = int(cfg.num_ps)
    if world <= n_ps:
        raise ValueError(f"async_ps needs more processes than parameter servers (world {world}, num_ps {n_ps})")
    spec = ModelSpec.from_config(cfg)
    hp = OptHParams(name=cfg.optimizer, lr=cfg.learning_rate)
    global _SHARD
    if rank < n_ps:
        _SHARD = ParameterShard(spec, hp, rank, n_ps, cfg.seed)
        _rpc_init(ps_name(rank), rank, world, cfg.dist_timeout_s)
        t0 = time.time()
        rpc.shutdown()  # graceful: returns once every worker has shut down
        out = {"role": ps_name(rank), "applies": _SHARD.applies, "served_s": round(time.time() - t0, 2)}
        _SHARD = None
        return out
    w, nw = rank - n_ps, world - n_ps
    _rpc_init(worker_name(w), rank, world, cfg.dist_timeout_s)
    info = RankInfo(rank=w, world=nw, local_rank=int(os.environ.get("LOCAL_RANK", "0")),
                    local_world=int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    device = torch.device("cuda", info.local_rank % max(torch.cuda.device_count(), 1)) \
        if torch.cuda.is_available() else torch.device("cpu")
    try:
        if w == 0:
            if cfg.clear_existing_model:
                from ..checkpoint import clear_model_dir

                clear_model_dir(cfg.effective_model_dir)
            est = Estimator(cfg, device=device, rank_info=info)  # restores model_dir into the PS
            rpc.rpc_sync(ps_name(0), _set_ready)
        else:
            _wait_ps0(lambda: rpc.rpc_sync(ps_name(0), _is_ready), "the chief's restore", cfg.dist_timeout_s)
            est = Estimator(cfg, device=device, rank_info=info, restore=False)
        out = (task_fn or _default_task)(est, w, nw)
        est.eng.flush()
        est.close()
        out["role"] = worker_name(w)
        return out
    except BaseException:
        try:  # tell ps0, so the chief / the other workers stop waiting for this one
            rpc.rpc_sync(ps_name(0), _worker_failed)
        except Exception:  # noqa: BLE001 — ps0 itself may be gone
            pass
        raise
    finally:
        rpc.shutdown()


def _default_task(est, w: int, nw: int) -> dict:
    """rocfm.cli's task flow for a worker: the chief evaluates, checkpoints and exports."""
    from ..data.tfrecord import discover_files
    from .dist import RankInfo

    cfg = est.cfg
    out: dict = {"task_type": cfg.task_type}
    tr_files = discover_files(cfg.training_data_dir, "tr", shuffle=True, seed=cfg.seed)
    va_files = discover_files(cfg.val_data_dir, "va")
    if cfg.task_type == "train":
        if not tr_files:
            raise FileNotFoundError(f"no tr*.tfrecords under {cfg.training_data_dir!r}")
        out["train"] = est.train(tr_files, cfg.num_epochs,
                                 max_steps=(cfg.max_steps // nw if cfg.max_steps else None))
        est.eng.flush()
        from torch.distributed import rpc

        rpc.rpc_sync(ps_name(0), _worker_done)
        if w == 0:  # the final checkpoint holds every worker's updates; evaluation reads all files
            _wait_ps0(lambda: rpc.rpc_sync(ps_name(0), _done_count) >= nw, "every worker to finish training",
                      cfg.dist_timeout_s)
            est.info = RankInfo(rank=0, world=1)
            if va_files:
                out["eval"] = est.evaluate(va_files)
            est.save()
            if cfg.servable_model_dir:
                out["export"] = est.export(cfg.servable_model_dir)
    elif w == 0 and cfg.task_type == "eval":
        est.info = RankInfo(rank=0, world=1)
        out["eval"] = est.evaluate(va_files)
    elif w == 0 and cfg.task_type == "export":
        out["export"] = est.export(cfg.servable_model_dir)
    return out
