#!/usr/bin/env python3
"""Critical-path experiments for the single-GPU fused step (graph-replayed, 8 steps per graph):
which chain bounds the step — main (rows → emb_update ‖ wgrad) or side (fetch → sort)?"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rocfm.data.synthetic import SyntheticCriteo
from rocfm.models.deepfm import ModelSpec, init_params
from rocfm.models.fused import FusedDeepFM
from rocfm.optim import OptHParams


def build(B=1024):
    spec = ModelSpec(1_000_000, 39, 10, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4)
    eng = FusedDeepFM(spec, OptHParams(name="Adam", lr=5e-4), B, torch.device("cuda"), params=init_params(spec, 1))
    gen = SyntheticCriteo(1_000_000, 39, seed=1)
    g = torch.Generator(device="cuda").manual_seed(1)
    pool = [gen.batch(B, "cuda", g) for _ in range(16)]
    eng.attach_pool(torch.stack([x[0] for x in pool]), torch.stack([x[1] for x in pool]),
                    torch.stack([x[2] for x in pool]))
    eng.train_steps(4)
    torch.cuda.synchronize()
    return eng


def timeit(fn, iters=50):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    e = build()
    S = 8
    main_s = lambda: torch.cuda.current_stream()
    res = {}
    res["pipelined"] = timeit(lambda: e._enqueue_pipelined(S)) / S
    res["step_join"] = timeit(lambda: [e._enqueue_step(k % 2) for k in range(S)]) / S

    def main_only():
        for k in range(S):
            aux = e._enqueue_rows_then_fork_wgrad(k % 2)
            e._enqueue_emb_update(k % 2)
            e._join(aux)
    res["main_only"] = timeit(main_only) / S

    def rows_only():
        for k in range(S):
            e.H.deepfm_rows(e.rows_params[k % 2], main_s().cuda_stream)
    res["rows_only"] = timeit(rows_only) / S

    def rows_emb():
        for k in range(S):
            e.H.deepfm_rows(e.rows_params[k % 2], main_s().cuda_stream)
            e._enqueue_emb_update(k % 2)
    res["rows+emb_serial"] = timeit(rows_emb) / S

    def emb_only():
        for k in range(S):
            e._enqueue_emb_update(k % 2)
    res["emb_only"] = timeit(emb_only) / S

    def wgrad_only():
        for k in range(S):
            e.H.mlp_wgrad(e.wgrad_params[k % 2], main_s().cuda_stream)
    res["wgrad_only"] = timeit(wgrad_only) / S

    def side_only():
        for k in range(S):
            e.H.fetch_batch(e.fetch_params[k % 2], main_s().cuda_stream)
            e._sort(1 - k % 2, main_s())
    res["fetch+sort"] = timeit(side_only) / S

    def sort_only():
        for k in range(S):
            e._sort(1 - k % 2, main_s())
    res["sort_only"] = timeit(sort_only) / S

    def empty_kernels():
        for k in range(S):
            e.H.fetch_batch(e.fetch_params[k % 2], main_s().cuda_stream)
    res["fetch_only"] = timeit(empty_kernels) / S
    def serial_main():
        for k in range(S):
            e.H.deepfm_rows(e.rows_params[k % 2], main_s().cuda_stream)
            e.H.mlp_wgrad(e.wgrad_params[k % 2], main_s().cuda_stream)
            e._enqueue_emb_update(k % 2)
    res["V1 serial main"] = timeit(serial_main) / S

    def serial_main_emb_first():
        for k in range(S):
            e.H.deepfm_rows(e.rows_params[k % 2], main_s().cuda_stream)
            e._enqueue_emb_update(k % 2)
            e.H.mlp_wgrad(e.wgrad_params[k % 2], main_s().cuda_stream)
    res["V1b rows,emb,wgrad"] = timeit(serial_main_emb_first) / S

    def v2():
        main = main_s()
        side = e.sort_stream
        prev = None
        for k in range(S):
            p = k % 2
            side.wait_stream(main)
            with torch.cuda.stream(side):
                e.H.fetch_batch(e.fetch_params[p], side.cuda_stream)
                evf = torch.cuda.Event(); evf.record(side)
                e._sort(1 - p, side)
                evs = torch.cuda.Event(); evs.record(side)
            if prev is not None:
                main.wait_event(prev[0])
            e.H.deepfm_rows(e.rows_params[p], main.cuda_stream)
            e.H.mlp_wgrad(e.wgrad_params[p], main.cuda_stream)
            if prev is not None:
                main.wait_event(prev[1])
            e._enqueue_emb_update(p)
            prev = (evf, evs)
        main.wait_stream(side)
    res["V2 serial+pipelined side"] = timeit(v2) / S

    def v3():
        main = main_s()
        for k in range(S):
            p = k % 2
            side = e._fork_next(p)
            e.H.deepfm_rows(e.rows_params[p], main.cuda_stream)
            e.H.mlp_wgrad(e.wgrad_params[p], main.cuda_stream)
            e._enqueue_emb_update(p)
            e._join(side)
    res["V3 serial+side joined/step"] = timeit(v3) / S

    def v4():
        main = main_s()
        side = e.sort_stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for k in range(S):
                e._sort(1 - k % 2, side)
        for k in range(S):
            p = k % 2
            e.H.deepfm_rows(e.rows_params[p], main.cuda_stream)
            e.H.mlp_wgrad(e.wgrad_params[p], main.cuda_stream)
            e._enqueue_emb_update(p)
        main.wait_stream(side)
    res["V4 serial + 1 side/graph"] = timeit(v4) / S

    def v5():
        main = main_s()
        for k in range(S):
            ev = torch.cuda.Event(); ev.record(main)
            side = e.sort_stream
            side.wait_event(ev)
            with torch.cuda.stream(side):
                e.H.fetch_batch(e.fetch_params[k % 2], side.cuda_stream)
            main.wait_stream(side)
            e.H.deepfm_rows(e.rows_params[k % 2], main.cuda_stream)
    res["V5 rows + 1 fork/join per step"] = timeit(v5) / S

    for k, v in res.items():
        print(f"{k:18s} {v:7.1f} us/step", flush=True)


if __name__ == "__main__":
    main()
