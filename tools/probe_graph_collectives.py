#!/usr/bin/env python3
"""Probe: can RCCL collectives (all_gather / all_to_all / all_reduce) be captured in a HIP graph
through torch.distributed and replayed correctly?  Run under torchrun (any nproc)."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    W, r = dist.get_world_size(), dist.get_rank()
    n = 1 << 16
    x = torch.full((n,), float(r + 1), device=dev)
    ag = torch.empty(W * n, device=dev)
    a2a_in = torch.arange(W * 8, dtype=torch.float32, device=dev) + 100 * r
    a2a_out = torch.empty_like(a2a_in)
    ar = torch.empty(n, device=dev)
    # eager warm-up (communicator init must not happen during capture)
    dist.all_gather_into_tensor(ag, x)
    dist.all_to_all_single(a2a_out, a2a_in)
    ar.copy_(x)
    dist.all_reduce(ar)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            y = x * 2
            dist.all_gather_into_tensor(ag, y)
            dist.all_to_all_single(a2a_out, a2a_in)
            ar.copy_(y)
            dist.all_reduce(ar)
    torch.cuda.synchronize()
    x.fill_(float(r + 2))
    ag.zero_()
    ar.zero_()
    g.replay()
    torch.cuda.synchronize()
    exp_ag = torch.cat([torch.full((n,), 2.0 * (q + 2), device=dev) for q in range(W)])
    ok = torch.equal(ag, exp_ag) and torch.allclose(ar, torch.full((n,), float(sum(2 * (q + 2) for q in range(W))), device=dev))
    exp_a2a = torch.cat([torch.arange(r * 8, r * 8 + 8, dtype=torch.float32, device=dev) + 100 * q for q in range(W)])
    ok = ok and torch.equal(a2a_out, exp_a2a)
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 200 * 1e6
    print(f"rank {r}/{W}: graph-captured collectives {'OK' if ok else 'MISMATCH'}; replay {dt:.1f} us", flush=True)
    mode = os.environ.get("PROBE_EXIT", "plain")
    if mode in ("delgraph", "delgraph_nodestroy"):
        del g
        torch.cuda.synchronize()
        print("graph deleted", flush=True)
    if mode != "nobarrier":
        dist.barrier(device_ids=[local])
        print("barrier done", flush=True)
    if mode != "delgraph_nodestroy":
        dist.destroy_process_group()
        print("destroyed", flush=True)
    sys.stdout.flush()
    os._exit(0 if ok else 1)


if __name__ == "__main__":
    main()
