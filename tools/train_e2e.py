#!/usr/bin/env python3
"""End-to-end training throughput: synthetic Criteo-shape TFRecord files → C++ loader → Estimator
(fused engine) on one GPU.  Reports examples/sec of the real input pipeline + training loop and
the loader alone."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rocfm.config import parse_flags
from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.data.tfrecord import TFRecordDataset
from rocfm.estimator import Estimator


def main():
    n = int(os.environ.get("N", "1000000"))
    d = os.environ.get("DATA", "/tmp/e2e_data")
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    for i in range(4):
        p = os.path.join(d, f"tr{i}.tfrecords")
        if not os.path.exists(p):
            write_synthetic_tfrecord(p, n // 4, 1_000_000, seed=i)
    print(f"data: {n} records in {time.time() - t0:.1f}s", flush=True)
    files = sorted(os.path.join(d, f) for f in os.listdir(d) if f.startswith("tr"))
    for threads in (4, 8, 12):
        ds = TFRecordDataset(files, 39, 1024, 1_000_000, num_threads=threads, verify_crc=True)
        t = time.time()
        k = sum(int(b[0].shape[0]) for b in ds)
        dt = time.time() - t
        t = time.time()
        kg = sum(int(g[0].shape[0]) * 1024 for g in ds.groups(16))
        dtg = time.time() - t
        print(f"loader alone, {threads} threads: {k / dt / 1e6:.2f} M ex/s per batch, "
              f"{kg / dtg / 1e6:.2f} M ex/s in groups of 16", flush=True)
    argv = ["--feature_size", "1000000", "--field_size", "39", "--embedding_size", "10", "--deep_layers",
            "128,64,32", "--dropout", "0.5,0.5,0.5", "--batch_size", "1024", "--training_data_dir", d,
            "--val_data_dir", d, "--model_dir", "", "--log_steps", "200", "--engine", "fused",
            "--num_threads", os.environ.get("THREADS", "8"), "--save_checkpoints_secs", "0"]
    est = Estimator(parse_flags(argv))
    est.train(files, num_epochs=1, max_steps=50)  # warm-up (graphs, code objects)
    for epochs in (1, 2):
        t = time.time()
        out = est.train(files, num_epochs=epochs)
        dt = time.time() - t
        print(f"estimator train (fused, loader fed, {epochs} epoch(s)): {out['steps']} steps, "
              f"{out['steps'] * 1024 / dt / 1e6:.2f} M ex/s, loss {out.get('loss', float('nan')):.4f}", flush=True)


if __name__ == "__main__":
    main()
