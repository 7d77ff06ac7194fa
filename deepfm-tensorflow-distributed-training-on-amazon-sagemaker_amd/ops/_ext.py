"""Locate the in-tree native modules built by ``build.py``.

``_rocfm_hip`` holds every HIP kernel; ``_rocfm_io`` the host runtime.  On a machine with a GPU
the fused engine refuses to run without ``_rocfm_hip`` (no silent eager fallback): ``require_hip``
raises with the build command to run.
"""
from __future__ import annotations

import importlib
import os

_PKG = __name__.rsplit(".", 2)[0]
_hip_mod = None
_io_mod = None
_hip_err = None
_io_err = None


def _load(name):
    return importlib.import_module(f"{_PKG}.{name}")


def hip():
    global _hip_mod, _hip_err
    if _hip_mod is None and _hip_err is None:
        try:
            import torch  # noqa: F401  (load torch's libamdhip64 first; same SONAME)

            _hip_mod = _load("_rocfm_hip")
        except ImportError as e:  # pragma: no cover - exercised on broken installs only
            _hip_err = e
    return _hip_mod


def has_hip() -> bool:
    return hip() is not None


def require_hip():
    m = hip()
    if m is None:
        raise RuntimeError(
            "rocfm HIP extension (_rocfm_hip) is not built or failed to load "
            f"({_hip_err}); run `python build.py` in {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}/..")
    return m


def io():
    global _io_mod, _io_err
    if _io_mod is None and _io_err is None:
        try:
            _io_mod = _load("_rocfm_io")
        except ImportError as e:  # pragma: no cover
            _io_err = e
    return _io_mod


def has_io() -> bool:
    return io() is not None


def require_io():
    m = io()
    if m is None:
        raise RuntimeError(f"rocfm host runtime (_rocfm_io) is not built ({_io_err}); run `python build.py`")
    return m
