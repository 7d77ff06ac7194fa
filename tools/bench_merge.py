"""Microbenchmark of the multi-rank row merge (merge.hip) at world sizes 1-8 on ONE GPU.

W rank exports are synthesised from W synthetic Criteo-shape batches (unique ids of each batch,
ascending — the sorted DP export), laid out like the gathered receive buffer; the two merges are
timed on them with HIP events: the search mode (one launch, binary search in the other lists), the
same search started inside each key's bucket of a directory (search+dir, what DP runs at 2-4
ranks), the map mode (scatter into W×V position maps, then apply) and the range mode.  Both write a dense gradient table
(mode 1) so repeated launches leave the inputs unchanged.

    python tools/bench_merge.py [--V 1000000] [--B 1024] [--iters 200] [--worlds 1,2,4,8] [--sdir_buckets N]
                                [--memory cached,uncached] [--cap N]

``--memory uncached`` places the gathered lists (keys, counts, rows, directories) in a
hipDeviceMallocUncached buffer — the memory type of the engine's p2p receive slots (p2p.py), which
the merge reads on the node — instead of cached torch tensors.  ``--cap N`` sizes the lists' slots
at N rows (the production default is batch_size · field_size) to show whether a merge's cost
follows the slot capacity or the live row counts.

It also times the owner-sharded DP merge (parallelism=dp_owner, owner_merge below).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rocfm.data.synthetic import SyntheticCriteo  # noqa: E402
from rocfm.ops import require_hip  # noqa: E402


def range_buckets(W: int, cap: int) -> int:
    """Buckets of the range merge: ≈192 gathered entries per workgroup, at least 64."""
    from rocfm.parallel.dp import range_merge_buckets

    return range_merge_buckets(W, cap)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=1_000_000)
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--F", type=int, default=39)
    ap.add_argument("--Kp", type=int, default=12)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--hash", action="store_true")
    ap.add_argument("--sdir_buckets", type=int, default=0, help="search+dir bucket count (0: dp's default)")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--memory", default="cached", help="cached and/or uncached (the p2p receive slots' type)")
    ap.add_argument("--cap", type=int, default=0, help="slot capacity in rows (0: the largest list)")
    ap.add_argument("--skip_owner", action="store_true")
    a = ap.parse_args()
    H = require_hip()
    dev = torch.device("cuda")
    gen = SyntheticCriteo(a.V, a.F, seed=1)
    g = torch.Generator(device=dev).manual_seed(1)
    # --hash: keys are a bijective multiplicative hash of the ids (id · odd mod 2^bits), spreading
    # the Zipf-clustered ids uniformly over the key space (what the range merge's buckets need)
    bits = max(1, (a.V - 1).bit_length())
    for W in [int(x) for x in a.worlds.split(",")]:
        lists = [gen.batch(a.B, dev, g)[0].flatten().to(torch.int64) for _ in range(W)]
        if a.hash:
            lists = [(x * 0x9E3779B1) & ((1 << bits) - 1) for x in lists]
        lists = [torch.unique(x) for x in lists]
        Vk = (1 << bits) if a.hash else a.V
        cap = (max(max(len(x) for x in lists), a.cap) + 3) // 4 * 4
        keys = torch.full((W, cap), 0xFFFFFFFF, dtype=torch.int64)
        for r, x in enumerate(lists):
            keys[r, : len(x)] = x.cpu()
        keys32 = torch.from_numpy(keys.numpy().astype(np.uint32).view(np.int32)).to(dev)  # pads = 0xFFFFFFFF
        counts = torch.tensor([len(x) for x in lists], dtype=torch.int32, device=dev)
        rows = torch.randn(W, cap, a.Kp, device=dev)
        dg = torch.zeros(Vk, a.Kp, device=dev)
        touched = torch.zeros(Vk, dtype=torch.int32, device=dev)
        step = torch.zeros(1, dtype=torch.int64, device=dev)
        pos = torch.full((W * Vk,), -1, dtype=torch.int32, device=dev)
        rep = torch.full((Vk,), W, dtype=torch.int32, device=dev)
        p = H.MergeParams()
        p.keys, p.key_stride = keys32.data_ptr(), cap
        p.rows, p.row_stride = rows.data_ptr(), cap * a.Kp
        p.counts, p.count_stride = counts.data_ptr(), 1
        p.W, p.cap, p.Kp, p.K1 = W, cap, a.Kp, a.Kp - 1
        p.key_div, p.Vmap = 1, Vk
        p.pos, p.rep = pos.data_ptr(), rep.data_ptr()
        p.mode, p.dense_grad, p.touched, p.step = 1, dg.data_ptr(), touched.data_ptr(), step.data_ptr()
        p.emb = dg.data_ptr()  # merge_apply loads the table row in every mode (any valid [V][Kp] f32)
        p.grad_scale = 1.0 / W
        # range mode: bucket directories of the sorted lists (what the sorted DP export writes)
        nb = range_buckets(W, cap)
        div = (Vk + nb - 1) // nb
        bounds = torch.arange(nb + 1, dtype=torch.int64) * div
        dirs = torch.zeros(W, nb + 1, dtype=torch.int32)
        for r, x in enumerate(lists):
            dirs[r] = torch.searchsorted(x.cpu(), bounds).to(torch.int32)
        dirs = dirs.to(dev)
        # search+dir: the search merge's own directory (the bucket count of dp.search_dir_buckets)
        snb = a.sdir_buckets or max(64, min(8192, Vk // 16))
        sdiv = (Vk + snb - 1) // snb
        sb = torch.arange(snb + 1, dtype=torch.int64) * sdiv
        sdirs = torch.stack([torch.searchsorted(x.cpu(), sb).to(torch.int32) for x in lists]).to(dev)
        s = torch.cuda.current_stream().cuda_stream
        names = ("search", "search+dir", "maps", "range")
        for mem in a.memory.split(","):
            src = (keys32, counts, rows, dirs, sdirs)
            raw = None
            if mem == "uncached":  # one uncached allocation holding every list, like a receive buffer
                sizes = [t.numel() for t in src]
                raw = H.p2p_malloc(4 * (sum(sizes) + 64), 0)
                views, off = [], 0
                for t, n in zip(src, sizes):
                    v = _uncached_view(raw + 4 * off, t.shape, t.dtype, dev)
                    v.copy_(t)
                    views.append(v)
                    off += (n + 3) // 4 * 4
                src = tuple(views)
            k_, c_, r_, d_, sd_ = src
            p.keys, p.rows, p.counts = k_.data_ptr(), r_.data_ptr(), c_.data_ptr()
            dir_of = {"range": (d_.data_ptr(), nb + 1, nb, div), "search+dir": (sd_.data_ptr(), snb + 1, snb, sdiv)}
            plan = plan_for(H, W, cap, k_, c_, Vk, dev, s)
            if W > 1:  # the side chain's per-step share when a 16-step graph builds its plans at once
                print(f"W={W} {mem}: plan build {plan_for(H, W, cap, k_, c_, Vk, dev, s, S=16)[1]:.2f} us per step "
                      f"at S = 16 ({plan[1]:.2f} at S = 1)")
            _time_merges(H, a, p, W, cap, nb, snb, names, dir_of, s, dg, mem, sum(len(x) for x in lists), plan)
            torch.cuda.synchronize()
            if raw is not None:
                del src, k_, c_, r_, d_, sd_
                H.p2p_free(raw)
        if not a.hash and not a.skip_owner:  # (hashed keys exceed the owner table's rows)
            owner_merge(H, a, W, lists, dev)


def _uncached_view(ptr, shape, dtype, dev):
    class _Raw:
        pass

    raw = _Raw()
    n = int(np.prod(shape))
    raw.__cuda_array_interface__ = {"shape": (n,), "typestr": {torch.float32: "<f4", torch.int32: "<i4"}[dtype],
                                    "data": (ptr, False), "version": 3, "strides": None}
    return torch.as_tensor(raw, device=dev).view(*shape)


def plan_for(H, W, cap, keys32, counts, Vk, dev, s, S=1):
    """The plan-ahead merge's side-chain product for these W lists (merge_plan.hip plan_build, S
    steps of the same lists, as one multi-step graph builds them): union ids + every id's position
    in every list.  Returns (PlanStep of step 0, build µs PER STEP, kept buffers)."""
    n = W * cap
    i32 = dict(dtype=torch.int32, device=dev)
    bufs = {k: torch.zeros(S * n, **i32) for k in ("pkeys", "sk", "sv", "rows")}
    pos = torch.zeros(S * n * W, **i32)
    cnt = torch.zeros(max(4, S), **i32)
    tiles = torch.zeros(H.plan_tile_ints(S, W, cap), **i32)
    bits = max(1, int(Vk).bit_length())  # the pad key Vk sorts after every id
    temp = torch.zeros(max(16, H.plan_sort_temp_bytes(S, W, cap, bits)), dtype=torch.uint8, device=dev)
    pp = H.PlanParams()
    pp.S, pp.W, pp.cap = S, W, cap
    pp.gkeys, pp.gcounts = keys32.data_ptr(), counts.data_ptr()
    pp.gk_stride, pp.gc_stride, pp.gkey_step, pp.gcount_step = cap, 1, 0, 0
    pp.pad_key = Vk
    pp.pkeys, pp.skeys_sorted, pp.svals_sorted = bufs["pkeys"].data_ptr(), bufs["sk"].data_ptr(), bufs["sv"].data_ptr()
    pp.tile_counts, pp.plan_rows, pp.plan_pos, pp.plan_count = (tiles.data_ptr(), bufs["rows"].data_ptr(),
                                                                pos.data_ptr(), cnt.data_ptr())
    for _ in range(3):
        H.plan_build(pp, temp.data_ptr(), temp.numel(), bits, s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        H.plan_build(pp, temp.data_ptr(), temp.numel(), bits, s)
    e1.record()
    torch.cuda.synchronize()
    ps = H.PlanStep()
    ps.rows, ps.pos, ps.count = bufs["rows"].data_ptr(), pos.data_ptr(), cnt.data_ptr()
    return ps, e0.elapsed_time(e1) * 1000 / 20 / S, (bufs, pos, cnt, tiles, temp)  # (keeps the buffers alive)


def _time_merges(H, a, p, W, cap, nb, snb, names, dir_of, s, dg, mem, live, plan=None):
    res = {}
    if plan is not None:
        names = names + ("plan",)
    for name in names:
        p.dirs, p.dir_stride, p.nb, p.bucket_div = dir_of.get(name, (0, 0, 0, 1))

        def run():
            if name in ("search", "search+dir"):
                H.merge_search_apply(p, None, s)
            elif name == "range":
                H.merge_range_apply(p, None, s)
            elif name == "plan":
                H.merge_plan_apply(p, plan[0], None, s)
            else:
                H.merge_scatter(p, s)
                H.merge_apply(p, s)
        for _ in range(10):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1000 / a.iters
    print(f"W={W} {mem} cap={cap} live rows={live} buckets={nb}: search {res['search']:.2f} us, "
          f"search+dir ({snb} buckets) {res['search+dir']:.2f} us, "
          f"maps {res['maps']:.2f} us, range {res['range']:.2f} us"
          + (f", plan apply {res['plan']:.2f} us (critical path; plan build {plan[1]:.2f} us on the side chain)"
             if plan is not None else ""), flush=True)
    # the merges write the same dense gradient rows
    outs = []
    for name in names:
        p.dirs, p.dir_stride, p.nb, p.bucket_div = dir_of.get(name, (0, 0, 0, 1))
        dg.zero_()
        if name in ("search", "search+dir"):
            H.merge_search_apply(p, None, s)
        elif name == "range":
            H.merge_range_apply(p, None, s)
        elif name == "plan":
            H.merge_plan_apply(p, plan[0], None, s)
        else:
            H.merge_scatter(p, s)
            H.merge_apply(p, s)
        torch.cuda.synchronize()
        outs.append(dg.clone())
    assert all(torch.equal(outs[0], o) for o in outs[1:]), W


def owner_merge(H, a, W, lists, dev):
    """parallelism=dp_owner: the same W batches, but owner 0 merges only the rows it owns (id % W
    == 0) — W source lists of ≈1/W of each export, as local rows id // W — and applies the row
    optimizer (mode 0, Adam) with a broadcast list of the updated rows (X5); then every replica
    scatters the W owners' lists (row_scatter).  Timed like the merges above."""
    Vs = (a.V + W - 1) // W
    own = [torch.unique(x[x % W == 0] // W) for x in lists]
    cap = (max(max(len(x) for x in own), 1) + 3) // 4 * 4
    keys = torch.full((W, cap), 0xFFFFFFFF, dtype=torch.int64)
    for r, x in enumerate(own):
        keys[r, : len(x)] = x.cpu()
    keys32 = torch.from_numpy(keys.numpy().astype(np.uint32).view(np.int32)).to(dev)
    counts = torch.tensor([len(x) for x in own], dtype=torch.int32, device=dev)
    rows = torch.randn(W, cap, a.Kp, device=dev) * 1e-3
    emb = torch.randn(Vs, a.Kp, device=dev) * 1e-2
    s0, s1 = torch.zeros_like(emb), torch.zeros_like(emb)
    step = torch.ones(1, dtype=torch.int64, device=dev)
    lrt = torch.full((1,), 1e-3, device=dev)
    capB = W * cap
    bc = torch.zeros(4 + capB * (1 + a.Kp), device=dev)
    p = H.MergeParams()
    p.keys, p.key_stride = keys32.data_ptr(), cap
    p.rows, p.row_stride = rows.data_ptr(), cap * a.Kp
    p.counts, p.count_stride = counts.data_ptr(), 1
    p.W, p.cap, p.Kp, p.K1 = W, cap, a.Kp, a.Kp - 1
    p.key_div, p.Vmap = 1, Vs
    pos = torch.full((W * Vs,), -1, dtype=torch.int32, device=dev)
    rep = torch.full((Vs,), W, dtype=torch.int32, device=dev)
    p.pos, p.rep = pos.data_ptr(), rep.data_ptr()
    p.emb, p.s0, p.s1, p.step, p.mode = emb.data_ptr(), s0.data_ptr(), s1.data_ptr(), step.data_ptr(), 0
    o = H.OptParams()
    o.type, o.lr, o.beta1, o.beta2, o.eps, o.lrt = 0, 1e-3, 0.9, 0.999, 1e-8, lrt.data_ptr()  # Adam
    p.opt, p.l2, p.grad_scale = o, 1e-4, 1.0 / W
    p.bc_count, p.bc_keys, p.bc_rows = bc.data_ptr(), bc[4:].data_ptr(), bc[4 + capB:].data_ptr()
    p.bc_cap, p.bc_mul, p.bc_add = capB, W, 0
    s = torch.cuda.current_stream().cuda_stream
    uniq = sum(len(x) for x in [torch.unique(torch.cat(own))])
    # every replica's X5 receive side: W owners' lists of ≈ the union's 1/W each
    recv = torch.zeros(W, 4 + capB * (1 + a.Kp), device=dev)
    table = torch.zeros(a.V, a.Kp, device=dev)
    for r in range(W):
        recv[r, 0] = torch.tensor([uniq], dtype=torch.int32).view(torch.float32)[0]
        recv[r, 4:4 + uniq] = (torch.arange(uniq, device=dev, dtype=torch.int32) * W + r).view(torch.float32)
    sp = H.RowScatterParams()
    sp.recv, sp.slot_stride, sp.W, sp.cap, sp.Kp = recv.data_ptr(), recv.shape[1], W, capB, a.Kp
    sp.table, sp.rows = table.data_ptr(), a.V
    res = {}
    for name in ("search", "maps", "scatter"):
        def run():
            bc[:1].zero_()
            if name == "search":
                p.use_maps = 0
                H.merge_search_apply(p, None, s)
            elif name == "maps":
                p.use_maps = 1
                H.merge_scatter(p, s)
                H.merge_search_apply(p, None, s)
            else:
                H.row_scatter(sp, s)
        for _ in range(10):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) * 1000 / a.iters
    bc[:1].zero_()
    p.use_maps = 0
    H.merge_search_apply(p, None, s)
    torch.cuda.synchronize()
    n_up = int(bc[:1].view(torch.int32).item())
    assert n_up == uniq, (n_up, uniq)  # one broadcast row per distinct owned id
    print(f"  dp_owner W={W}: owner lists cap={cap} entries={int(counts.sum())} updated rows={uniq}: "
          f"search+opt {res['search']:.2f} us, maps+opt {res['maps']:.2f} us, row_scatter (W lists) "
          f"{res['scatter']:.2f} us")


if __name__ == "__main__":
    main()
