"""Loader-alone breakdown on the current host: pinned-ring allocation, time to the first group,
steady-state rate, for short (bench secondary window) and long runs.

    python tools/loader_breakdown.py [--batches 272,2064] [--threads 8,16] [--dir DIR]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocfm.data.synthetic import write_synthetic_tfrecord  # noqa: E402
from rocfm.data.tfrecord import TFRecordDataset  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="272,2064")
    ap.add_argument("--threads", default="8,16")
    ap.add_argument("--dir", default="")
    ap.add_argument("--group", type=int, default=16)
    a = ap.parse_args()
    B, F, V = 1024, 39, 1_000_000
    d = a.dir or tempfile.mkdtemp(prefix="rocfm_ldb_")
    os.makedirs(d, exist_ok=True)
    out = {"cpus": os.cpu_count(), "sched_cpus": len(os.sched_getaffinity(0)), "pinned": torch.cuda.is_available()}
    for nb in [int(x) for x in a.batches.split(",")]:
        nrec, files = nb * B, []
        per = (nrec + 3) // 4
        for i in range(4):
            p = os.path.join(d, f"b{nb}_{i}.tfrecords")
            if not os.path.exists(p):
                write_synthetic_tfrecord(p, per, V, F, seed=1234 + i)
            files.append(p)
        for th in [int(x) for x in a.threads.split(",")]:
            for rep in range(3):
                ds = TFRecordDataset(files, F, B, V, num_threads=th, verify_crc=True, hold=2)
                t0 = time.perf_counter()
                it = ds.groups(a.group, hold=2)
                first = None
                n = 0
                for g in it:
                    if first is None:
                        first = time.perf_counter() - t0
                    n += int(g[0].shape[0])
                dt = time.perf_counter() - t0
                rest = (n - a.group) * B / max(dt - first, 1e-9)
                r = dict(batches=n, threads=th, rep=rep, total_ms=round(dt * 1e3, 2), first_group_ms=round(first * 1e3, 2),
                         rate_m=round(n * B / dt / 1e6, 2), after_first_m=round(rest / 1e6, 2))
                print(json.dumps(r), flush=True)
    t = time.perf_counter()
    x = torch.empty(64, B, F, dtype=torch.int32, pin_memory=torch.cuda.is_available())
    out["pinned_alloc_ms_fresh_shape"] = round((time.perf_counter() - t) * 1e3, 2)
    del x
    print(json.dumps(out))


if __name__ == "__main__":
    main()
