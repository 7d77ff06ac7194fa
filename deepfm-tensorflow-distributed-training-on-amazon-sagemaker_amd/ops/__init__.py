"""Native-op loading and the pure-PyTorch reference implementations of every HIP kernel."""
from ._ext import has_hip, has_io, hip, io, require_hip, require_io  # noqa: F401
