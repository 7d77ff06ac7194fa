"""Command-line entry point — the reference training script's ``main`` (PS:389-551, HVD:331-493).

    python -m rocfm.cli --task_type train --training_data_dir data/ --val_data_dir data/ \\
        --model_dir /tmp/m --servable_model_dir /tmp/export --field_size 39 --feature_size 117581 \\
        --batch_size 1024 --deep_layers 128,64,32 --num_epochs 10 --log_steps 100

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m rocfm.cli …``
(one process per GPU; RCCL).  Every flag of the reference scripts is accepted (rocfm.config).

task_type:
  train   — train (+ per-epoch eval when val files exist), final checkpoint, export on rank 0 when
            servable_model_dir is set (the reference also exports after training, Q10)
  eval    — evaluate the latest checkpoint on ``va*`` files
  infer   — predict ``te*`` files, write ``<val_data_dir>/pred.txt`` ("%f\\n" per example)
  export  — export the latest checkpoint as a servable bundle
"""
from __future__ import annotations

import json
import logging
import os
import sys
from typing import List, Optional

from .config import Config, parse_flags


def _remaining_steps(max_steps: int, global_step: int) -> Optional[int]:
    """Steps left to reach the global-step target ``max_steps`` (None = no limit)."""
    return max(0, max_steps - global_step) if max_steps else None


def run(cfg: Config) -> dict:
    import torch

    from .checkpoint import clear_model_dir
    from .data.tfrecord import discover_files
    from .estimator import Estimator
    from .parallel.dist import init_distributed

    if cfg.parallelism == "async_ps":  # PS / worker roles over RPC, no process group
        from .parallel.async_ps import run_job

        return run_job(cfg)
    info = init_distributed("cuda" if torch.cuda.is_available() else "cpu", cfg.dist_timeout_s)
    if cfg.clear_existing_model and info.is_chief:
        clear_model_dir(cfg.effective_model_dir)  # HVD:372-378
    if info.world > 1:
        import torch.distributed as dist

        dist.barrier()
    if info.is_chief:  # PS:398-414: print every flag
        logging.getLogger("rocfm").info("flags %s", json.dumps(cfg.to_dict(), default=str))
    est = Estimator(cfg)
    out: dict = {"task_type": cfg.task_type}
    if cfg.pipe_mode and cfg.task_type == "train":
        # SageMaker Pipe mode: one FIFO per channel and epoch, channels bound by SM_CHANNELS or the
        # channel-name flags; one training pass over the epochs' streams, then evaluation on the
        # evaluation channel (HVD:443-456; PS:505-521)
        from .data.sharding import pipe_mode_sources

        tr_fifos, va_fifos = pipe_mode_sources(cfg.num_epochs, info.local_rank, cfg.training_channel_name,
                                               cfg.evaluation_channel_name)
        out["channels"] = {"train": tr_fifos, "eval": va_fifos}
        # max_steps is a global-step target, as in file mode: a restarted job resumes toward it
        max_steps = _remaining_steps(cfg.max_steps, est.global_step)
        if max_steps is not None and max_steps <= 0:
            out["train"] = {"global_step": est.global_step, "steps": 0}
        else:
            out["train"] = est.train(tr_fifos, 1, max_steps=max_steps)
        if va_fifos:
            out["eval"] = est.evaluate(va_fifos)
        if cfg.servable_model_dir:
            out["export"] = est.export(cfg.servable_model_dir)
        est.close()
        return out
    tr_files = discover_files(cfg.training_data_dir, "tr", shuffle=True, seed=cfg.seed)
    va_files = discover_files(cfg.val_data_dir, "va")
    te_files = discover_files(cfg.val_data_dir, "te")
    if cfg.task_type == "train":
        if not tr_files:
            raise FileNotFoundError(f"no tr*.tfrecords under {cfg.training_data_dir!r}")
        if va_files and cfg.eval_every_epoch:
            out["epochs"] = est.train_and_evaluate(tr_files, va_files, cfg.num_epochs)
        else:
            ep0, skip = est.resume_point(tr_files, cfg.num_epochs)  # restarted job: fast-forward
            max_steps = _remaining_steps(cfg.max_steps, est.global_step)
            if max_steps is not None and max_steps <= 0:
                out["train"] = {"global_step": est.global_step, "steps": 0}
            else:
                out["train"] = est.train(tr_files, cfg.num_epochs - ep0, max_steps=max_steps, skip_batches=skip)
        if cfg.servable_model_dir:
            out["export"] = est.export(cfg.servable_model_dir)
    elif cfg.task_type == "eval":
        out["eval"] = est.evaluate(va_files)
    elif cfg.task_type == "infer":
        path = os.path.join(cfg.val_data_dir, "pred.txt")
        probs = est.predict(te_files, path)
        out["infer"] = {"pred_path": path, "n": int(len(probs))}
    elif cfg.task_type == "export":
        out["export"] = est.export(cfg.servable_model_dir)
    est.close()
    return out


def main(argv: Optional[List[str]] = None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    cfg = parse_flags(sys.argv[1:] if argv is None else argv)
    res = run(cfg)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res, default=str))
    return 0


if __name__ == "__main__":
    sys.exit(main())
