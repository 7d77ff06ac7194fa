"""Probe: does a short timed window depend on how long the GPU was idle before it?

Pool-fed headline engine; 20-step windows (the driver's shape) measured
  (1) right after a 5-step warm-up in a fresh process (the driver's bench),
  (2) right after ~300 ms of back-to-back GPU work,
  (3) after 2 s of host-only idling,
  (4) after a 2 s idle and then 300 ms of GPU work again.
Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    from rocfm.data.synthetic import SyntheticCriteo
    from rocfm.models.deepfm import ModelSpec, init_params
    from rocfm.models.fused import FusedDeepFM
    from rocfm.optim import OptHParams

    spec = ModelSpec(1_000_000, 39, 10, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
    gen = SyntheticCriteo(1_000_000, 39, seed=1)
    g = torch.Generator(device=dev).manual_seed(1)
    pb = [gen.batch(1024, dev, g) for _ in range(32)]
    e = FusedDeepFM(spec, OptHParams(name="Adam", lr=5e-4), 1024, dev, params=init_params(spec, 1))
    e.attach_pool(*(torch.stack([x[i] for x in pb]) for i in range(3)))
    S = 20

    def window():
        e.precapture(20, S)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.train_steps(20, S)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / 20 * 1e6, 2)

    def busy(ms):
        a = torch.randn(4096, 4096, device=dev)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < ms:
            for _ in range(10):
                a = a @ a
                a = a / a.norm()
            torch.cuda.synchronize()

    e.train_steps(5, S)
    out = {"cold": window()}
    out["cold_again"] = window()
    busy(300)
    out["after_busy"] = window()
    out["after_busy_again"] = window()
    time.sleep(2.0)
    out["after_idle_2s"] = window()
    busy(300)
    out["after_idle_then_busy"] = window()
    e.train_steps(2000, S)  # 2,000 steps back to back, then a window
    out["after_2000_steps"] = window()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
