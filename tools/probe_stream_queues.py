"""Probe: does the throughput of the multi-step graphs depend on how many streams the process
created before the engine?  (HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues; a side /
copy stream that lands on the main stream's queue serialises the side chain behind the steps.)

    python tools/probe_stream_queues.py K [tf|pool]

creates K torch.cuda.Stream objects first, then measures the bench's pool-fed window (K=0..7
from separate processes) or a short TFRecord-fed window.  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    k = int(sys.argv[1])
    mode = sys.argv[2] if len(sys.argv) > 2 else "pool"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    keep = [torch.cuda.Stream(device=dev) for _ in range(k)]
    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    spec = ModelSpec(1_000_000, 39, 10, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=5e-4)
    out = {"k": k, "mode": mode}
    if mode == "pool":
        gen = SyntheticCriteo(1_000_000, 39, seed=1)
        g = torch.Generator(device=dev).manual_seed(1)
        pb = [gen.batch(1024, dev, g) for _ in range(32)]
        e = FusedDeepFM(spec, hp, 1024, dev, params=init_params(spec, 1))
        e.attach_pool(*(torch.stack([x[i] for x in pb]) for i in range(3)))
        e.train_steps(64, 64)
        e.precapture(640, 64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.train_steps(640, 64)
        torch.cuda.synchronize()
        out["us_per_step"] = round((time.perf_counter() - t0) / 640 * 1e6, 2)
    else:
        import argparse

        import bench

        a = argparse.Namespace(batch_size=1024, field_size=39, feature_size=1_000_000, steps=1024, warmup=128,
                               steps_per_graph=32, data_dir="", loader_threads=8, host_decode=False, loader_hold=2,
                               embedding_update="sparse", compute_dtype="bf16", table_dtype="f32", seed=1234,
                               embedding_size=10, deep_layers="128,64,32", dropout="0.5,0.5,0.5", optimizer="Adam",
                               json_out="")
        r = bench.measure_tfrecord(a, spec, hp, init_params(spec, 1), dev)
        out.update({x: r[x] for x in ("value", "ms_per_step", "steady_examples_per_sec", "input_stall_fraction")})
    out["streams"] = [s.cuda_stream for s in keep][:2]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
