"""Configuration / flag system.

One dataclass carries every flag the reference scripts define, under the same names, so a
SageMaker-style ``hyperparameters`` dict or the reference command lines work unchanged:

* PS script flags: ``1-ps-cpu/DeepFM-dist-ps-for-multipleCPU-multiInstance.py:36-107``
* Horovod script flags: ``2-hvd-gpu/DeepFM-hvd-tfrecord-vectorized-map.py:35-98``

Deliberate fixes over the reference:

* Q4  ``log_steps`` is live (logging cadence); ``loss_type`` supports ``log_loss`` and
  ``square_loss``.
* Q5  ``optimizer=GD`` is implemented (plain SGD).
* Q14 booleans parse strictly: ``--flag``, ``--noflag``, ``--flag=False``, ``--flag False``,
  ``--flag 0`` all work (SageMaker passes ``--enable_s3_shard False`` as two tokens).
* ``hosts``/``current_host`` default from ``SM_HOSTS``/``SM_CURRENT_HOST`` only when present
  (the reference crashes on ``json.loads(None)`` outside SageMaker, PS:80-84).

Flags added by this framework (not in the reference) are grouped at the bottom of the dataclass.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

_TRUE = {"1", "true", "t", "yes", "y", "on"}
_FALSE = {"0", "false", "f", "no", "n", "off", ""}


def str2bool(v: Any) -> bool:
    """Strict boolean parsing."""
    if isinstance(v, bool):
        return v
    if isinstance(v, (int, float)):
        return bool(v)
    s = str(v).strip().lower()
    if s in _TRUE:
        return True
    if s in _FALSE:
        return False
    raise ValueError(f"cannot parse boolean from {v!r}")


def _env_json_list(name: str, default: List[str]) -> List[str]:
    v = os.environ.get(name)
    if not v:
        return list(default)
    try:
        out = json.loads(v)
        return list(out) if isinstance(out, (list, tuple)) else [str(out)]
    except json.JSONDecodeError:
        return [v]


@dataclass
class Config:
    # ---- reference flags (PS:36-107 / HVD:35-98) ------------------------------------------
    dist_mode: int = 0  # PS:39 — dead in the reference; kept for CLI compatibility
    ps_hosts: str = ""  # PS:41 (dead)
    worker_hosts: str = ""  # PS:44 (dead)
    job_name: str = ""  # PS:47 (dead)
    task_index: int = 0  # PS:48 (dead)
    num_threads: int = 16  # PS:49 — used here as the data-loader thread count
    feature_size: int = 0  # PS:50 — vocabulary size V
    field_size: int = 0  # PS:51 — F
    embedding_size: int = 32  # PS:52 — K
    num_epochs: int = 10  # PS:53
    batch_size: int = 64  # PS:54 — per-worker batch
    log_steps: int = 1000  # PS:55 — live here (Q4)
    learning_rate: float = 0.0005  # PS:56
    l2_reg: float = 0.0001  # PS:57
    loss_type: str = "log_loss"  # PS:58 — log_loss | square_loss
    optimizer: str = "Adam"  # PS:59 — Adam | Adagrad | Momentum | ftrl | GD
    deep_layers: str = "256,128,64"  # PS:62
    dropout: str = "0.5,0.5,0.5"  # PS:63 — KEEP probabilities (PS:246, Q3)
    batch_norm: bool = False  # PS:64
    batch_norm_decay: float = 0.9  # PS:67
    training_data_dir: str = ""  # PS:70
    val_data_dir: str = ""  # PS:71
    model_dir: str = ""  # PS:73
    checkpoint_dir: str = ""  # HVD:59
    servable_model_dir: str = ""  # PS:74
    task_type: str = "train"  # PS:77 — train | eval | infer | export
    clear_existing_model: bool = False  # HVD:66
    hosts: List[str] = field(default_factory=lambda: _env_json_list("SM_HOSTS", ["localhost"]))  # PS:80
    current_host: str = field(default_factory=lambda: os.environ.get("SM_CURRENT_HOST", "localhost"))  # PS:85
    num_GPUs: int = field(default_factory=lambda: int(os.environ.get("SM_NUM_GPUS", "0") or 0))  # PS:90 (dead)
    num_CPUs: int = field(default_factory=lambda: int(os.environ.get("SM_NUM_CPUS", str(os.cpu_count() or 1)) or 1))
    pipe_mode: int = 0  # PS:96 — 0 file, 1 pipe/stream (FIFO or stdin)
    worker_per_host: int = 1  # HVD:80
    training_channel_name: str = ""  # PS:97
    evaluation_channel_name: str = ""  # PS:100
    enable_s3_shard: bool = False  # PS:103
    enable_data_multi_path: bool = False  # HVD:94
    perform_shuffle: bool = False  # input_fn arg (PS:113); live here as a buffer shuffle (Q6)

    # ---- rocfm flags ---------------------------------------------------------------------
    engine: str = "auto"  # auto | fused (HIP kernels) | torch (eager oracle; CPU or GPU)
    embedding_update: str = "sparse"  # sparse (lazy L2 + row optimizer) | exact (dense, faithful Q1)
    parallelism: str = "auto"  # auto | dp (replicated table) | rowshard (PS-equivalent) | dense_dp
    #                            | dp_owner (replicated table, owner-sharded embedding optimizer)
    #                            | async_ps (asynchronous parameter servers over RPC, PS:461-521)
    num_ps: int = 1  # async_ps: ranks 0 .. num_ps-1 are parameter servers, the rest workers
    lr_scaling: str = "linear"  # linear (lr × world, HVD:171) | none
    compute_dtype: str = "bf16"  # bf16 | fp8: MLP MFMA operands in the fused engine (fp8: the input
    #                              layer's forward GEMM on e4m3 with dynamic per-row/per-column scales)
    seed: int = 1234
    save_checkpoints_steps: int = 0  # 0 → only at end (plus save_checkpoints_secs)
    save_checkpoints_secs: int = 600  # Estimator default cadence
    hbm_cache: bool = True  # >1 epoch, no shuffle: every rank keeps its decoded first epoch in HBM and
    #                         trains later epochs from it (the reference re-reads + re-parses every epoch)
    device_decode: bool = True  # fused engine streaming: the loader copies undecoded Example payloads
    #                             and the GPU parses them (csrc/kernels/decode.hip); False = host parse
    hbm_cache_gb: float = 64.0  # budget for that cache (decoded epoch: B·(8F + 4) bytes per batch)
    # pre-decoded on-disk cache (rocfm.data.cache): each rank's first pass over its training shard is
    # written raw (int32 ids, f32 values / labels) under this directory and every later epoch — and
    # any later job on the same files, shard and batch size — memory-maps it instead of re-decoding
    # the TFRecords ("" = off; file mode without record shuffle only)
    decoded_cache_dir: str = ""
    ckpt_poll_steps: int = 200  # world > 1: steps between rank 0's broadcasts of the time-based save decision
    keep_checkpoint_max: int = 5
    eval_every_epoch: bool = True
    deterministic: bool = True
    use_hip_graph: bool = True
    profile_steps: str = ""  # "a:b" — wrap steps [a,b) with torch.profiler / roctx ranges
    metrics_file: str = ""  # JSONL metrics output
    tensorboard: bool = True  # chief writes TF event files: model_dir (train) and model_dir/eval (utils/tensorboard.py)
    # training-data sharding over ranks: "record" = Dataset.shard (every count-th record of the
    # concatenated file list, the reference's semantics — each rank reads only its own records
    # through the files' persistent record indexes, csrc/io/record_index.h);
    # "file" = each rank reads files[index::count] only (like SageMaker's ShardedByS3Key input,
    # README:87-92), so P ranks walk each byte once; needs at least `count` files
    shard_policy: str = "record"
    crc_check: bool = True  # verify TFRecord CRCs
    on_bad_record: str = "fail"  # fail | skip
    max_steps: int = 0  # 0 → run num_epochs
    dist_timeout_s: int = 600
    watchdog_s: int = 0  # >0: dump stacks and exit(3) when no step completes for this long (§5.3)
    exchange_capacity: int = 0  # rows per rank (dp) / per owner (rowshard) in the exchange buffers; 0 = B*F (safe)
    # rowshard: 0 = synchronous; 1 = bounded staleness (the reference's async PS, PS:461-521): a step's
    # rows are served during the previous step's owner update (Hogwild-style reads; not bitwise reproducible)
    ps_staleness: int = 0
    # rowshard: replicate the N most frequent ids (rank 0's first batches) on every rank; their
    # gradients ride the MLP all-reduce bucket (synchronous, same update as their owners would apply)
    hot_rows: int = 0
    table_dtype: str = "f32"  # fused engines: f32 | bf16 embedding-table storage (f32 slots, stochastic rounding)
    dp_exchange: str = "auto"  # dp / rowshard exchange transport: auto | p2p (IPC push over xGMI, one node) | rccl

    # ------------------------------------------------------------------------------------
    @property
    def layers(self) -> List[int]:
        return [int(x) for x in str(self.deep_layers).split(",") if str(x).strip()]

    @property
    def keep_probs(self) -> List[float]:
        return [float(x) for x in str(self.dropout).split(",") if str(x).strip()]

    @property
    def effective_model_dir(self) -> str:
        return self.model_dir or self.checkpoint_dir

    def validate(self) -> "Config":
        if self.field_size <= 0:
            raise ValueError("field_size must be > 0")
        if self.feature_size <= 0:
            raise ValueError("feature_size must be > 0")
        if self.embedding_size <= 0:
            raise ValueError("embedding_size must be > 0")
        if self.hot_rows < 0 or (self.hot_rows and self.parallelism != "rowshard"):
            raise ValueError("hot_rows (>= 0) applies to parallelism=rowshard")
        if self.table_dtype not in ("f32", "bf16"):
            raise ValueError("table_dtype must be f32 or bf16")
        if self.ps_staleness not in (0, 1):
            raise ValueError("ps_staleness must be 0 or 1")
        if self.ps_staleness and self.parallelism != "rowshard":
            raise ValueError("ps_staleness applies to parallelism=rowshard (the parameter-server equivalent)")
        if len(self.keep_probs) != len(self.layers):
            raise ValueError(
                f"len(dropout)={len(self.keep_probs)} must equal len(deep_layers)={len(self.layers)}")
        for p in self.keep_probs:
            if not (0.0 < p <= 1.0):
                raise ValueError(f"dropout values are keep probabilities in (0,1], got {p}")
        if self.optimizer not in ("Adam", "Adagrad", "Momentum", "ftrl", "GD"):
            raise ValueError(f"unknown optimizer {self.optimizer!r}")
        if self.loss_type not in ("log_loss", "square_loss"):
            raise ValueError(f"unknown loss_type {self.loss_type!r}")
        if self.shard_policy not in ("record", "file"):
            raise ValueError("shard_policy must be record or file")
        if self.dp_exchange not in ("auto", "p2p", "rccl"):
            raise ValueError(f"unknown dp_exchange {self.dp_exchange!r}")
        if self.task_type not in ("train", "eval", "infer", "export"):
            raise ValueError(f"unknown task_type {self.task_type!r}")
        if self.embedding_update not in ("sparse", "exact"):
            raise ValueError(f"unknown embedding_update {self.embedding_update!r}")
        if self.compute_dtype not in ("bf16", "fp8"):
            raise ValueError(f"compute_dtype must be bf16 or fp8, got {self.compute_dtype!r}")
        if self.num_ps < 1:
            raise ValueError("num_ps must be >= 1")
        if self.parallelism == "async_ps" and (self.embedding_update != "sparse" or self.batch_norm):
            raise ValueError("async_ps trains with embedding_update=sparse and without batch_norm")
        if self.parallelism not in ("auto", "dp", "dense_dp", "rowshard", "dp_owner", "async_ps"):
            raise ValueError(f"unknown parallelism {self.parallelism!r}")
        if self.engine not in ("auto", "fused", "torch"):
            raise ValueError(f"unknown engine {self.engine!r}")
        return self

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Config":
        c = cls()
        for k, v in d.items():
            c.set(k, v, strict=False)
        return c

    # ---- flag parsing ---------------------------------------------------------------------
    def set(self, name: str, value: Any, strict: bool = True) -> None:
        fields = {f.name: f for f in dataclasses.fields(self)}
        if name not in fields:
            if strict:
                raise KeyError(name)
            return  # unknown flags are tolerated like tf.app.flags does
        f = fields[name]
        cur = getattr(self, name)
        if isinstance(cur, bool):
            setattr(self, name, str2bool(value))
        elif isinstance(cur, int):
            setattr(self, name, int(float(value)) if not isinstance(value, int) else value)
        elif isinstance(cur, float):
            setattr(self, name, float(value))
        elif isinstance(cur, list):
            if isinstance(value, str):
                try:
                    value = json.loads(value)
                except json.JSONDecodeError:
                    value = [x for x in value.split(",") if x]
            setattr(self, name, list(value))
        else:
            setattr(self, name, str(value))


def parse_flags(argv: Sequence[str], base: Optional[Config] = None) -> Config:
    """Parse ``--flag value`` / ``--flag=value`` / ``--flag`` / ``--noflag`` tokens.

    ``--config file.yaml`` loads a YAML/JSON dict first (later flags override it).  Unknown flags
    are ignored, like ``tf.app.run`` (NB-PS:92 passes ``perform_shuffle`` which the PS script
    never defines).
    """
    cfg = base or Config()
    names = {f.name: f for f in dataclasses.fields(cfg)}
    toks = list(argv)
    i = 0
    while i < len(toks):
        t = toks[i]
        i += 1
        if not t.startswith("-"):
            continue
        t = t.lstrip("-")
        if "=" in t:
            k, v = t.split("=", 1)
        else:
            k, v = t, None
        if k == "config":
            if v is None:
                v = toks[i]
                i += 1
            _load_config_file(cfg, v)
            continue
        neg = False
        if k not in names and k.startswith("no") and k[2:] in names and isinstance(getattr(cfg, k[2:]), bool):
            k, neg = k[2:], True
        if k not in names:
            # unknown: swallow a value token if one follows
            if v is None and i < len(toks) and not toks[i].startswith("--"):
                i += 1
            continue
        is_bool = isinstance(getattr(cfg, k), bool)
        if v is None:
            if is_bool:
                if i < len(toks) and not toks[i].startswith("-"):
                    try:
                        v = str2bool(toks[i])
                        i += 1
                    except ValueError:
                        v = True
                else:
                    v = True
                if neg:
                    v = not v
            else:
                if i >= len(toks):
                    raise ValueError(f"flag --{k} needs a value")
                v = toks[i]
                i += 1
        cfg.set(k, v)
    return cfg


def _load_config_file(cfg: Config, path: str) -> None:
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml

        d = yaml.safe_load(text) or {}
    else:
        d = json.loads(text)
    for k, v in d.items():
        cfg.set(k, v, strict=False)
