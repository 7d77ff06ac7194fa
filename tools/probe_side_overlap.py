"""Probe: what the overlapped side chain (fetch + sort + plan of the next graph's batches) costs
the main chain.  GPU time of the main graph per step (events around its replay) with the side
graph overlapped (default) vs serialised behind the main graph (ROCFM_SIDE_AFTER_MAIN), windows
interleaved in one process.  Usage (GPU): python tools/probe_side_overlap.py [k=10|32] [S]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.data.synthetic import SyntheticCriteo  # noqa: E402
from rocfm.models.deepfm import ModelSpec, init_params  # noqa: E402
from rocfm.models.fused import FusedDeepFM  # noqa: E402
from rocfm.optim import OptHParams  # noqa: E402


def main():
    dev = torch.device("cuda")
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    V = 1_000_000 if k == 10 else 117_581
    spec = ModelSpec(V, 39, k, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
    eng = FusedDeepFM(spec, OptHParams("Adam", 5e-4), 1024, dev, params=init_params(spec, 1234))
    gen = SyntheticCriteo(V, 39, seed=1234)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = [gen.batch(1024, dev, g) for _ in range(32)]
    eng.attach_pool(*(torch.stack([x[i] for x in pool]) for i in range(3)))
    eng.train_steps(5, S)
    res = {"overlap": [], "serial": []}
    side_end = []  # overlapped: side graph end after its main graph's start, µs (graphs 2..4)
    for rnd in range(6):
        for name in res:
            eng._side_after_main = name == "serial"
            eng.precapture(4 * S, S)
            torch.cuda.synchronize()
            eng.stall_timing = []
            eng.train_steps(4 * S, S)
            torch.cuda.synchronize()
            st, eng.stall_timing = eng.stall_timing, None
            # main graph GPU time per step, graphs 2..4 (the first may follow an idle gap)
            per = [s0.elapsed_time(m1) * 1e3 / S for s0, m1, _ in st[1:]]
            res[name].append(round(statistics.mean(per), 2))
            if name == "overlap":
                side_end.append(round(statistics.mean(s0.elapsed_time(sd) * 1e3 for s0, _, sd in st[1:]), 1))
        print(f"round {rnd}: " + " ".join(f"{n}={v[-1]}" for n, v in res.items()), file=sys.stderr, flush=True)
    eng._side_after_main = False
    eng.check()
    print(json.dumps({"k": k, "S": S, "main_graph_us_per_step": res,
                      "median": {n: statistics.median(v[1:]) for n, v in res.items()},
                      "side_end_after_main_start_us": statistics.median(side_end[1:]),
                      "main_graph_us": round(statistics.median(res["overlap"][1:]) * S, 1)}), flush=True)


if __name__ == "__main__":
    main()
