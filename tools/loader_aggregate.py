#!/usr/bin/env python3
"""Aggregate decode rate of P concurrent TFRecord loader processes, one per rank shard.

An 8-GPU job runs one process per GPU, each decoding its own shard of the training files with the
C++ loader (rocfm.data.tfrecord, csrc/io).  This measures what P such processes decode together on
this host, next to the per-process rate and the rate of reading the same batches from the
pre-decoded on-disk cache (rocfm.data.cache) and of the raw mode that leaves the Example parsing to
the GPU (csrc/kernels/decode.hip), so the loader's margin over P GPUs can be read off:

    python tools/loader_aggregate.py --procs 1,2,4,8 --threads 4 --records 400000 [--json out.json]

Synthetic Criteo-shape files (39 fields, Zipf ids) are written to a temporary directory first
(not timed).  Every process is started at once and decodes ``groups(16)`` of its shard
(record-index sharding, as the Estimator's training input); the aggregate is all processes'
examples over the slowest process's wall time.
"""
import argparse
import json
import multiprocessing as mp
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(files, rank, procs, threads, B, F, V, mode, cache_dir, q, bar, policy):
    import torch

    torch.set_num_threads(1)
    from rocfm.data.tfrecord import TFRecordDataset

    ds = TFRecordDataset(files, F, B, V, shard_count=procs, shard_index=rank, num_threads=threads,
                         verify_crc=True, pin_memory=False, hold=2, shard_policy=policy)
    if mode == "cache":
        from rocfm.data.cache import DecodedCache

        cache = DecodedCache.for_dataset(ds, cache_dir)
        if not cache.complete():
            for _ in cache.write_through(ds.groups(16, hold=2)):
                pass
        src = cache.groups(16, pin_memory=False)
    elif mode == "raw":  # undecoded payloads for the GPU parser (the fused engine's streaming input)
        src = ds.raw_groups(16, hold=2)
    else:
        src = ds.groups(16, hold=2)
    bar.wait()  # every process starts its timed pass together (cache mode: after its first pass)
    t0 = time.perf_counter()
    n = 0
    for g in src:
        if mode == "raw":
            n += g.n
            continue
        n += int(g[0].shape[0]) if g[0].dim() == 3 else 1
    q.put((rank, n * B, time.perf_counter() - t0))


def run(files, procs, threads, B, F, V, mode, cache_dir, policy):
    ctx = mp.get_context("spawn")
    q, bar = ctx.Queue(), ctx.Barrier(procs)
    ps = [ctx.Process(target=_worker, args=(files, r, procs, threads, B, F, V, mode, cache_dir, q, bar, policy))
          for r in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=1200) for _ in ps]
    for p in ps:
        p.join()
    ex = sum(r[1] for r in res)
    wall = max(r[2] for r in res)
    return {"mode": mode, "shard_policy": policy, "procs": procs, "threads_per_proc": threads, "examples": ex,
            "aggregate_examples_per_sec": round(ex / wall, 1),
            "per_proc_examples_per_sec": [round(r[1] / r[2], 1) for r in sorted(res)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,4,8")
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--records", type=int, default=400_000)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--batch_size", type=int, default=1024)
    ap.add_argument("--feature_size", type=int, default=1_000_000)
    ap.add_argument("--modes", default="raw,tfrecord,cache",
                    help="raw (frames + CRCs + payload copy; the GPU parses), tfrecord (host parse), cache")
    ap.add_argument("--shard_policy", default="record,file", help="record (Dataset.shard) and/or file")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from rocfm.data.synthetic import write_synthetic_tfrecord

    d = tempfile.mkdtemp(prefix="rocfm_loadagg_")
    try:
        per = a.records // a.files
        files = []
        for i in range(a.files):
            p = os.path.join(d, f"tr{i}.tfrecords")
            write_synthetic_tfrecord(p, per, a.feature_size, 39, seed=100 + i)
            files.append(p)
        out = {"host_cpus": os.cpu_count(), "records": per * a.files, "results": []}
        for mode in a.modes.split(","):
            for pol in a.shard_policy.split(","):
                if mode == "cache" and pol == "file":
                    continue  # the cache reads only its own shard either way
                for P in (int(x) for x in a.procs.split(",")):
                    cache_dir = os.path.join(d, f"cache_{P}")
                    r = run(files, P, a.threads, a.batch_size, 39, a.feature_size, mode, cache_dir, pol)
                    out["results"].append(r)
                    print(json.dumps(r), flush=True)
        if a.json:
            with open(a.json, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
