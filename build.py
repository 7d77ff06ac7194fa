#!/usr/bin/env python3
"""Build the rocfm native extensions in-tree (gfx950 only).

Two Python extension modules are produced next to the package sources:

* ``rocfm/_rocfm_hip``  – every HIP kernel (csrc/kernels/*.hip, hipcc --offload-arch=gfx950)
  plus pybind11 launch bindings (csrc/hip_module.cpp).  No torch headers: ops take raw device
  pointers + the current HIP stream, so the module compiles in seconds and its launches are
  captured by torch.cuda.CUDAGraph.
* ``rocfm/_rocfm_io``   – the host-only C++ runtime (TFRecord reader/writer, CRC32C,
  fixed-schema Example decoder, multi-threaded prefetching batch loader, libsvm converter).
  Built with g++ so it works on CPU-only machines too.

Usage: ``python build.py [--force] [-j N]``.  Incremental: an object is rebuilt only when its source or
one of the headers it includes (transitively) changed (content hash).
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import re
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "deepfm-tensorflow-distributed-training-on-amazon-sagemaker_amd")
BUILD = os.path.join(ROOT, "build", "obj")
CSRC = os.path.join(ROOT, "csrc")
ARCH = os.environ.get("ROCFM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _py_includes():
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(src, seen=None):
    """The quoted headers a source includes, transitively (resolved next to the includer, then
    under csrc/): an object is rebuilt only when one of ITS headers changed."""
    seen = set() if seen is None else seen
    try:
        text = open(src, encoding="utf-8", errors="replace").read()
    except OSError:
        return seen
    for name in _INC.findall(text):
        for cand in (os.path.join(os.path.dirname(src), name), os.path.join(CSRC, name)):
            cand = os.path.normpath(cand)
            if os.path.exists(cand):
                if cand not in seen:
                    seen.add(cand)
                    _deps(cand, seen)
                break
    return seen


def _digest(src):
    """Content hash of a source and every header it includes (mtimes alone miss a header that a
    checkout restored with an older time — an object built against another struct layout)."""
    h = hashlib.sha1()
    for f in [src] + sorted(_deps(src)):
        with open(f, "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def _stale(obj, src):
    stamp = obj + ".sha1"
    if not os.path.exists(obj) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(src)


def _stamp(obj, src):
    with open(obj + ".sha1", "w") as f:
        f.write(_digest(src))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n$ " + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return r.stderr


def hip_objects(force, jobs):
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + [os.path.join(CSRC, "hip_module.cpp")]
    os.makedirs(BUILD, exist_ok=True)
    base = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-I", CSRC,
            "-Wno-unused-result", "-munsafe-fp-atomics"]
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(BUILD, "hip_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, s):
            extra = []
            if s.endswith(".cpp"):
                extra = ["-x", "hip"] + sum((["-I", p] for p in _py_includes()), [])
            todo.append(base + extra + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max(1, jobs)) as ex:
        for err in ex.map(_run, todo):
            if err and "warning" in err:
                sys.stderr.write(err)
    for cmd in todo:
        _stamp(cmd[-1], cmd[cmd.index("-c") + 1])
    return objs


def io_objects(force, jobs):
    srcs = sorted(glob.glob(os.path.join(CSRC, "io", "*.cpp")))
    os.makedirs(BUILD, exist_ok=True)
    base = [CXX, "-O3", "-fPIC", "-std=c++17", "-msse4.2", "-pthread", "-I", CSRC]
    base += sum((["-I", p] for p in _py_includes()), [])
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(BUILD, "io_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, s):
            todo.append(base + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max(1, jobs)) as ex:
        list(ex.map(_run, todo))
    for cmd in todo:
        _stamp(cmd[-1], cmd[cmd.index("-c") + 1])
    return objs


def link(objs, out, hip):
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(o) for o in objs):
        return out
    if hip:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
    else:
        cmd = [CXX, "-shared", "-fPIC", "-pthread", "-o", out] + objs
    _run(cmd)
    return out


def build(force=False, jobs=None, hip=True, io=True):
    jobs = jobs or min(16, os.cpu_count() or 4)
    outs = []
    if io and glob.glob(os.path.join(CSRC, "io", "*.cpp")):
        outs.append(link(io_objects(force, jobs), os.path.join(PKG, "_rocfm_io" + EXT), hip=False))
    if hip:
        outs.append(link(hip_objects(force, jobs), os.path.join(PKG, "_rocfm_hip" + EXT), hip=True))
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--no-hip", action="store_true")
    a = ap.parse_args()
    for o in build(a.force, a.j, hip=not a.no_hip):
        print("built", os.path.relpath(o, ROOT))
