"""One-shot push exchange over IPC-mapped peer buffers (csrc/kernels/p2p.hip, rocfm.parallel.p2p).

Two processes share one GPU (gloo only carries the IPC handles), so the mapping, the flag
protocol, graph replay and the bounded waits are exercised; xGMI bandwidth is not (one GPU).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)


def _exchange_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from rocfm.parallel.p2p import P2PExchange, selftest

    dev = torch.device("cuda", 0)
    n = 70_000  # floats per destination (not a multiple of the chunk size)
    ex = P2PExchange(world * n, dev)
    res = {"selftest": selftest(ex, n)}
    # all-gather through a captured graph: the graph re-reads src and advances the device counter
    src = torch.zeros(n, device=dev)
    p = ex.params(src.data_ptr(), n)
    out = torch.zeros(world * ex.slot, device=dev)
    g = torch.cuda.CUDAGraph()
    ex.push(p)  # warm
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            ex.push(p)
    ok = True
    for it in range(5):
        src.copy_(torch.arange(n, device=dev, dtype=torch.float32) + 100000.0 * rank + it)
        g.replay()
        ex.copy_out(out)
        torch.cuda.synchronize()
        for r in range(world):
            want = torch.arange(n, device=dev, dtype=torch.float32) + 100000.0 * r + it
            ok = ok and torch.equal(out[r * ex.slot: r * ex.slot + n], want)
    res["graph_allgather"] = ok
    # equal-split all-to-all: destination d gets src[d*n:(d+1)*n]
    a2a = torch.arange(world * n, device=dev, dtype=torch.float32) + 1e6 * rank
    p2 = ex.params(a2a.data_ptr(), n, src_stride_floats=n)
    ex.push(p2)
    ex.copy_out(out)
    torch.cuda.synchronize()
    ok = True
    for r in range(world):
        want = torch.arange(rank * n, (rank + 1) * n, device=dev, dtype=torch.float32) + 1e6 * r
        ok = ok and torch.equal(out[r * ex.slot: r * ex.slot + n], want)
    res["alltoall"] = ok
    # timing of the eager push (one GPU: both ranks' kernels share it; indicative only)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier()
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    res["us_per_push"] = e0.elapsed_time(e1) * 1e3 / 20
    res["error"] = ex.errored()
    ex.close()
    torch.save(res, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_p2p_allgather_alltoall_graph(tmp_path):
    out = str(tmp_path / "p2p")
    mp.start_processes(_exchange_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    for r in range(2):
        res = torch.load(out + f".{r}", weights_only=True)
        print(f"rank {r}: {res}")
        assert res["selftest"] and res["graph_allgather"] and res["alltoall"] and not res["error"], res


def _timeout_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from rocfm.parallel.p2p import P2PExchange

    dev = torch.device("cuda", 0)
    ex = P2PExchange(1024, dev, spin_limit=1 << 14)  # ≈1 ms waits
    src = torch.ones(1024, device=dev)
    if rank == 0:  # rank 1 never pushes: rank 0's waits must time out, not hang
        ex.push(ex.params(src.data_ptr(), 1024))
    torch.cuda.synchronize()
    res = {"error": ex.errored()}
    ex.close()
    torch.save(res, out_path + f".{rank}")
    dist.destroy_process_group()


def test_p2p_missing_peer_times_out(tmp_path):
    out = str(tmp_path / "p2pto")
    mp.start_processes(_timeout_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    assert torch.load(out + ".0", weights_only=True)["error"]
    assert not torch.load(out + ".1", weights_only=True)["error"]
