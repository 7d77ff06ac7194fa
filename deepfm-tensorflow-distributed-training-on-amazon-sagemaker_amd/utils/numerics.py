"""Numerics / input guards.

* ``ROCFM_CHECK_IDS=1`` — every batch's ids are checked against ``[0, feature_size)`` before they
  reach a kernel (the fused kernels index the table without bounds checks).
* ``check_finite(loss, step)`` — raise on a NaN/Inf loss at a log point (the Estimator calls it
  whenever it logs; ``ROCFM_CHECK_NUMERICS=0`` disables it).
"""
from __future__ import annotations

import math
import os

import torch


def ids_check_enabled() -> bool:
    return os.environ.get("ROCFM_CHECK_IDS", "0") not in ("", "0")


def check_ids(ids: torch.Tensor, feature_size: int) -> None:
    if ids.numel() == 0:
        return
    lo, hi = int(ids.min()), int(ids.max())
    if lo < 0 or hi >= feature_size:
        raise ValueError(f"feature id out of range: min {lo}, max {hi}, feature_size {feature_size}")


def numerics_check_enabled() -> bool:
    return os.environ.get("ROCFM_CHECK_NUMERICS", "1") not in ("", "0")


class NonFiniteLoss(FloatingPointError):
    pass


def check_finite(loss: float, step: int) -> None:
    if not math.isfinite(loss):
        raise NonFiniteLoss(f"non-finite loss {loss} at global step {step}")
