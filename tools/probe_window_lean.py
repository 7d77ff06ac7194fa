"""Probe: the driver-shaped 20-step window (one multi-step graph pair) timed like bench.py (host
clock from before the launch to after a device synchronize), with the ROCFM_LEAN_LAUNCH variants
interleaved in one process: 0 (events created per launch, a wait on the previous side graph, a
trailing side-chain join), 1 (preallocated events, no wait on a side graph already complete),
3 (1 + lazy trailing join).  Usage (GPU): python tools/probe_window_lean.py [k=10|32]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.data.synthetic import SyntheticCriteo  # noqa: E402
from rocfm.models.deepfm import ModelSpec, init_params  # noqa: E402
from rocfm.models.fused import FusedDeepFM  # noqa: E402
from rocfm.optim import OptHParams  # noqa: E402


def main():
    dev = torch.device("cuda")
    S = int(os.environ.get("S", "20"))
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    V = 1_000_000 if k == 10 else 117_581
    spec = ModelSpec(V, 39, k, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
    eng = FusedDeepFM(spec, OptHParams("Adam", 5e-4), 1024, dev, params=init_params(spec, 1234))
    gen = SyntheticCriteo(V, 39, seed=1234)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = [gen.batch(1024, dev, g) for _ in range(32)]
    eng.attach_pool(*(torch.stack([x[i] for x in pool]) for i in range(3)))
    eng.train_steps(5, S)
    res = {0: [], 1: [], 3: []}
    for rnd in range(8):
        for v in (0, 1, 3):
            eng._lean_launch = v
            eng.precapture(S, S)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.train_steps(S, S)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            eng._join_side_chain()
            res[v].append(round(1e6 * dt / S, 2))
        print(f"round {rnd}: " + " ".join(f"v{v}={res[v][-1]}" for v in res), file=sys.stderr, flush=True)
    eng.check()
    print(json.dumps({"k": k, "S": S, "us_per_step": {str(v): x for v, x in res.items()},
                      "median": {str(v): statistics.median(x[1:]) for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
