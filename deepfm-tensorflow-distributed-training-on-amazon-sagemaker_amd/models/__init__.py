"""DeepFM model: spec/parameters (deepfm), eager engine (torch_engine), fused HIP engine (fused)."""
from .deepfm import ModelSpec, init_params, param_shapes  # noqa: F401
