"""libsvm → TFRecord converter (the reference's tools/libsvm_to_tfrecord.py, TOOL:22-76).

Each input line ``label id:val id:val …`` becomes one ``tf.train.Example`` with features
``label`` (float_list, 1 value), ``ids`` (int64_list) and ``values`` (float_list) — the schema the
training scripts parse (PS:117-126).  Conversion runs in the native multi-threaded converter
(csrc/io/loader.cpp ``convert_libsvm``: mmap input, per-thread line ranges, masked-CRC32C framing).

Unlike the reference (hard-coded paths, one output file) it takes paths on the command line and can
split the output into contiguous shards named like ``tr-00000-of-00004.tfrecords`` — one per
SageMaker ``ShardedByS3Key`` object or per training rank (README:67-108).

    python -m rocfm.tools.libsvm_to_tfrecord train.libsvm tr.tfrecords [--shards 8] [--threads 16]
    python -m rocfm.tools.libsvm_to_tfrecord a.libsvm b.libsvm --output_dir out/ --prefix tr
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List


def shard_paths(output: str, shards: int) -> List[str]:
    """``x.tfrecords`` → [``x-00000-of-0000N.tfrecords``, …] (or [output] for one shard)."""
    if shards <= 1:
        return [output]
    stem, ext = os.path.splitext(output)
    ext = ext or ".tfrecords"
    return [f"{stem}-{k:05d}-of-{shards:05d}{ext}" for k in range(shards)]


def convert(input_path: str, output: str, shards: int = 1, threads: int = 8) -> dict:
    from ..ops import io

    m = io()
    if m is None:
        raise RuntimeError("rocfm._rocfm_io is not built (python build.py)")
    outs = shard_paths(output, shards)
    for o in outs:
        os.makedirs(os.path.dirname(os.path.abspath(o)), exist_ok=True)
    t0 = time.time()
    n = m.convert_libsvm_sharded(input_path, outs, threads)
    for o in outs:  # persistent record indexes next to the shards (ranks jump to their records)
        m.build_index(o, True)
    return {"input": input_path, "outputs": outs, "records": int(n), "seconds": round(time.time() - t0, 3)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("inputs", nargs="+", help="libsvm file(s); with one input the last positional may be the output")
    ap.add_argument("--output_dir", default="", help="write <prefix>[-k-of-N].tfrecords per input here")
    ap.add_argument("--prefix", default="", help="output name prefix with --output_dir (default: the input's stem)")
    ap.add_argument("--shards", type=int, default=1, help="contiguous output shards per input")
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args(argv)
    if a.output_dir:
        jobs = []
        for i, src in enumerate(a.inputs):
            stem = a.prefix or os.path.splitext(os.path.basename(src))[0]
            if a.prefix and len(a.inputs) > 1:
                stem = f"{a.prefix}{i}"
            jobs.append((src, os.path.join(a.output_dir, stem + ".tfrecords")))
    else:
        if len(a.inputs) != 2:
            ap.error("give INPUT OUTPUT, or inputs with --output_dir")
        jobs = [(a.inputs[0], a.inputs[1])]
    for src, dst in jobs:
        print(json.dumps(convert(src, dst, a.shards, a.threads)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
