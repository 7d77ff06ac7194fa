"""Probe: where the driver-shaped 20-step window's extra per-step time goes (one graph of 20 steps vs
the 200-step window's steady state): host time of the main / side graph replays, time from the
window's start to the first kernel, and the GPU span of the main graph.  Usage (GPU):
python tools/probe_graph_launch.py"""
import os
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
    spec = ModelSpec(1_000_000, 39, 10, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
    eng = FusedDeepFM(spec, OptHParams("Adam", 5e-4), 1024, dev, params=init_params(spec, 1234))
    gen = SyntheticCriteo(1_000_000, 39, seed=1234)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = [gen.batch(1024, dev, g) for _ in range(32)]
    eng.attach_pool(*(torch.stack([x[i] for x in pool]) for i in range(3)))
    eng.train_steps(5, S)
    for _ in range(4):
        eng.precapture(S, S)
        torch.cuda.synchronize()
        main = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(main)
        eng.stall_timing = []
        eng.train_steps(S, S)
        t1 = time.perf_counter()
        e1.record(main)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        st = eng.stall_timing
        eng.stall_timing = None
        s0, m1, sd = st[0]
        print(f"S={S}: window {1e6 * (t2 - t0):.1f} us ({1e6 * (t2 - t0) / S:.2f} us/step); host launch calls "
              f"{1e6 * (t1 - t0):.1f} us; GPU: window start -> main graph start {e0.elapsed_time(s0) * 1e3:.1f} us, "
              f"main graph {s0.elapsed_time(m1) * 1e3:.1f} us ({s0.elapsed_time(m1) * 1e3 / S:.2f} us/step), "
              f"side graph ends {s0.elapsed_time(sd) * 1e3:.1f} us after the main graph's start; "
              f"main end -> window end {m1.elapsed_time(e1) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
