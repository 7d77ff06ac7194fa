"""Checkpoints and servable export (the Estimator's model_dir / export_savedmodel).

Layout of ``model_dir`` (same roles as TF's):

    checkpoint                          text index: model_checkpoint_path + all_model_checkpoint_paths
    model.ckpt-<step>.index.json        manifest: TF variable names → shape/dtype/shard + row ranges
    model.ckpt-<step>.shard-<r>-of-<n>.safetensors
                                        tensors (safetensors: loading executes nothing)

Variable names follow the reference: ``fm_bias``, ``fm_w``, ``fm_v``, ``Deep-part/mlp{i}/weights``,
``…/biases``, ``Deep-part/deep_out/…``, ``Deep-part/bn_{i}/…``, optimizer slots ``<var>/Adam``,
``<var>/Adam_1`` (or ``/Adagrad``, ``/Momentum``, ``/Ftrl``, ``/Ftrl_1``), ``global_step``,
``beta1_power``, ``beta2_power``.  Row-sharded tables (rocfm.parallel.emb_shard) write one shard
per rank with its row set recorded in the manifest, so a checkpoint written by N ranks restores
on M ranks (reshard) or on a single process.  Writes are atomic (temp file + rename; the index is
updated last) and only the chief writes replicated state (HVD:402-415).  ``keep_checkpoint_max``
old checkpoints are kept (Estimator default 5).

``export_servable`` writes ``<servable_model_dir>/<unix-ts>/`` with the trainable weights, the
model config and the serving signature of PS:262-272 / 536-551 (inputs feat_ids int64[None,F],
feat_vals float32[None,F]; output prob).
"""
from __future__ import annotations

import json
import math
import struct
import os
import re
import shutil
import tempfile
import time
from typing import Dict, List, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file

INDEX = "checkpoint"


def _atomic_write_text(path: str, text: str) -> None:
    d = os.path.dirname(path) or "."
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp-")
    with os.fdopen(fd, "w") as f:
        f.write(text)
    os.replace(tmp, path)


def _sanitize(name: str) -> str:
    return name  # safetensors keys may contain '/' and '-'


def list_checkpoints(model_dir: str) -> List[str]:
    p = os.path.join(model_dir, INDEX)
    if not os.path.exists(p):
        return []
    out = []
    for line in open(p):
        m = re.match(r'all_model_checkpoint_paths:\s*"(.*)"', line.strip())
        if m:
            out.append(m.group(1))
    return out


def latest_checkpoint(model_dir: str) -> Optional[str]:
    p = os.path.join(model_dir or "", INDEX)
    if not model_dir or not os.path.exists(p):
        return None
    for line in open(p):
        m = re.match(r'model_checkpoint_path:\s*"(.*)"', line.strip())
        if m:
            prefix = os.path.join(model_dir, m.group(1))
            if os.path.exists(prefix + ".index.json"):
                return prefix
    return None


def save_checkpoint(model_dir: str, state: Dict[str, torch.Tensor], step: int, keep_max: int = 5,
                    shard: Tuple[int, int] = (0, 1), row_sets: Optional[Dict[str, torch.Tensor]] = None,
                    extra: Optional[dict] = None, write_index: bool = True,
                    global_rows: Optional[Dict[str, int]] = None) -> str:
    """Write shard ``shard=(r, n)`` of checkpoint ``step``; the rank with r == 0 writes the manifest.

    ``row_sets``: for row-sharded variables, the global row ids held by this shard (1-D int64);
    ``global_rows``: their full row counts (default: 1 + the largest row id of this shard's set).
    """
    os.makedirs(model_dir, exist_ok=True)
    r, n = shard
    prefix = f"model.ckpt-{step}"
    data = f"{prefix}.shard-{r:05d}-of-{n:05d}.safetensors"
    tensors = {_sanitize(k): v.detach().contiguous().cpu() for k, v in state.items()}
    if row_sets:
        for k, rows in row_sets.items():
            tensors[f"__rows__/{k}"] = rows.detach().to(torch.int64).cpu().clone()
    fd, tmp = tempfile.mkstemp(dir=model_dir, prefix=".tmp-", suffix=".safetensors")
    os.close(fd)
    save_file(tensors, tmp)
    os.replace(tmp, os.path.join(model_dir, data))
    if r == 0 and write_index:
        def gshape(k, v):
            if row_sets and k in row_sets:
                rows = (global_rows or {}).get(k, int(row_sets[k].max()) + 1 if row_sets[k].numel() else 0)
                return [int(rows)] + list(v.shape[1:])
            return list(v.shape)

        manifest = {
            "step": int(step),
            "num_shards": int(n),
            "variables": {k: {"shape": gshape(k, v), "dtype": str(v.dtype).replace("torch.", ""),
                              "row_sharded": bool(row_sets and k in row_sets)} for k, v in state.items()},
            "created": time.time(),
        }
        if extra:
            manifest["extra"] = extra
        _atomic_write_text(os.path.join(model_dir, prefix + ".index.json"), json.dumps(manifest, indent=1))
        paths = [p for p in list_checkpoints(model_dir) if p != prefix] + [prefix]
        drop, keep = (paths[:-keep_max], paths[-keep_max:]) if keep_max > 0 else ([], paths)
        text = f'model_checkpoint_path: "{prefix}"\n' + "".join(f'all_model_checkpoint_paths: "{p}"\n' for p in keep)
        _atomic_write_text(os.path.join(model_dir, INDEX), text)
        for old in drop:
            for f in os.listdir(model_dir):
                if f.startswith(old + ".") and (f.endswith(".safetensors") or f.endswith(".json")):
                    try:
                        os.remove(os.path.join(model_dir, f))
                    except FileNotFoundError:
                        pass
    return os.path.join(model_dir, prefix)


def load_checkpoint(prefix: str, rows_for: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
    """Load a checkpoint (all shards).  Row-sharded variables are reassembled into full tables, or —
    with ``rows_for={name: global_row_ids}`` — only those rows are returned (resharding)."""
    with open(prefix + ".index.json") as f:
        man = json.load(f)
    n = man["num_shards"]
    shards = [load_file(f"{prefix}.shard-{r:05d}-of-{n:05d}.safetensors") for r in range(n)]
    out: Dict[str, torch.Tensor] = {}
    for name, meta in man["variables"].items():
        if not meta["row_sharded"]:
            for s in shards:
                if name in s:
                    out[name] = s[name]
                    break
            continue
        shape = meta["shape"]
        full_rows = shape[0] if len(shape) else 0
        dtype = getattr(torch, meta["dtype"])
        if rows_for is not None and name in rows_for:
            want = rows_for[name].to(torch.int64)
            res = torch.zeros((len(want),) + tuple(shape[1:]), dtype=dtype)
            pos = torch.full((full_rows,), -1, dtype=torch.int64)
            pos[want] = torch.arange(len(want))
            for s in shards:
                if name in s:
                    rows = s[f"__rows__/{name}"]
                    sel = pos[rows]
                    m = sel >= 0
                    res[sel[m]] = s[name][m]
            out[name] = res
        else:
            res = torch.zeros(tuple(shape), dtype=dtype)
            for s in shards:
                if name in s:
                    res[s[f"__rows__/{name}"]] = s[name]
            out[name] = res
    return out


def checkpoint_step(prefix: str) -> int:
    with open(prefix + ".index.json") as f:
        return int(json.load(f)["step"])


# --------------------------------------------------------------------------------------------
# servable export
# --------------------------------------------------------------------------------------------
SIGNATURE = {
    "serving_default": {
        "inputs": {"feat_ids": {"dtype": "int64", "shape": [None, "field_size"]},
                   "feat_vals": {"dtype": "float32", "shape": [None, "field_size"]}},
        "outputs": {"prob": {"dtype": "float32", "shape": [None]}},
    }
}


def export_servable(servable_model_dir: str, params: Dict[str, torch.Tensor], model_config: dict) -> str:
    """Write a self-contained inference bundle; returns its directory (``<dir>/<unix-ts>``)."""
    ts = str(int(time.time()))
    out = os.path.join(servable_model_dir, ts)
    while os.path.exists(out):
        ts = str(int(ts) + 1)
        out = os.path.join(servable_model_dir, ts)
    tmp = out + ".tmp"
    os.makedirs(os.path.join(tmp, "variables"), exist_ok=True)
    save_file({k: v.detach().contiguous().cpu().float() for k, v in params.items()},
              os.path.join(tmp, "variables", "variables.safetensors"))
    sig = json.loads(json.dumps(SIGNATURE))
    F = model_config.get("field_size")
    for inp in sig["serving_default"]["inputs"].values():
        inp["shape"] = [None, F]
    with open(os.path.join(tmp, "model.json"), "w") as f:
        json.dump({"format": "rocfm-servable-v1", "model": "DeepFM", "config": model_config, "signatures": sig},
                  f, indent=1)
    os.replace(tmp, out)
    return out


class StreamedServable:
    """The same bundle as ``export_servable``, written incrementally: the dense variables at once,
    the [V, ...] tables chunk by chunk at their final offsets (the row-sharded engine gathers one
    row range at a time, so no rank ever holds a whole 1B-row table).  The safetensors header is
    written first — the shapes are known — and the file is renamed into place on ``close``."""

    def __init__(self, servable_model_dir: str, dense: Dict[str, torch.Tensor], table_shapes: Dict[str, tuple],
                 model_config: dict):
        ts = str(int(time.time()))
        out = os.path.join(servable_model_dir, ts)
        while os.path.exists(out):
            ts = str(int(ts) + 1)
            out = os.path.join(servable_model_dir, ts)
        self.out, self.tmp = out, out + ".tmp"
        self.config = model_config
        os.makedirs(os.path.join(self.tmp, "variables"), exist_ok=True)
        dense = {k: v.detach().contiguous().cpu().float() for k, v in dense.items()}
        header, off = {}, 0
        for k, v in dense.items():
            n = v.numel() * 4
            header[k] = {"dtype": "F32", "shape": list(v.shape), "data_offsets": [off, off + n]}
            off += n
        self.table_off = {}
        for k, shp in table_shapes.items():
            n = int(math.prod(shp)) * 4
            header[k] = {"dtype": "F32", "shape": list(shp), "data_offsets": [off, off + n]}
            self.table_off[k] = (off, int(math.prod(shp[1:])) if len(shp) > 1 else 1)
            off += n
        hb = json.dumps(header, separators=(",", ":")).encode()
        hb += b" " * ((8 - len(hb) % 8) % 8)  # 8-byte aligned data start
        self.data0 = 8 + len(hb)
        self.path = os.path.join(self.tmp, "variables", "variables.safetensors")
        self.fh = open(self.path, "wb")
        self.fh.write(struct.pack("<Q", len(hb)) + hb)
        for v in dense.values():
            self.fh.write(v.numpy().tobytes())
        self.fh.truncate(self.data0 + off)

    def write_rows(self, name: str, row0: int, rows: torch.Tensor) -> None:
        off, per = self.table_off[name]
        self.fh.seek(self.data0 + off + row0 * per * 4)
        self.fh.write(rows.detach().contiguous().cpu().float().numpy().tobytes())

    def close(self) -> str:
        self.fh.close()
        sig = json.loads(json.dumps(SIGNATURE))
        F = self.config.get("field_size")
        for inp in sig["serving_default"]["inputs"].values():
            inp["shape"] = [None, F]
        with open(os.path.join(self.tmp, "model.json"), "w") as f:
            json.dump({"format": "rocfm-servable-v1", "model": "DeepFM", "config": self.config, "signatures": sig},
                      f, indent=1)
        os.replace(self.tmp, self.out)
        return self.out


def load_servable(path: str):
    """(model_config, params) of an exported bundle (a directory, or its parent → newest)."""
    if os.path.exists(os.path.join(path, "model.json")):
        d = path
    else:
        subs = sorted((s for s in os.listdir(path) if s.isdigit()), key=int)
        if not subs:
            raise FileNotFoundError(f"no servable under {path}")
        d = os.path.join(path, subs[-1])
    with open(os.path.join(d, "model.json")) as f:
        meta = json.load(f)
    params = load_file(os.path.join(d, "variables", "variables.safetensors"))
    return meta, params


def clear_model_dir(model_dir: str) -> None:
    """``clear_existing_model`` (HVD:372-378)."""
    if model_dir and os.path.isdir(model_dir):
        shutil.rmtree(model_dir)
