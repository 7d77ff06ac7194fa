"""Optimizers with TF-1.x update formulas (dense and lazy row-sparse)."""
from .tf_optim import OPTIMIZERS, OPT_ID, OptHParams, adam_lr_t, apply_dense, apply_rows, init_slots, slot_names  # noqa: F401
