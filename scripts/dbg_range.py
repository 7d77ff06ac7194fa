# Debug: rows where the range merge differs from the search merge (bucket, rank membership)
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rocfm.ops import require_hip
from rocfm.parallel.dp import range_merge_buckets

H = require_hip()
dev = torch.device("cuda")
for (W, crowd), MODE in [((w, c), m) for m in (1, 0) for w, c in ((2, False), (2, True), (3, True))]:
    V, Kp = 2_000_000, 12
    g = torch.Generator().manual_seed(W)
    lists = []
    for r in range(W):
        parts = [torch.randint(0, V, (3000 + 500 * r,), generator=g)]
        if crowd:
            parts.append(torch.arange(0, 2000))
        lists.append(torch.unique(torch.cat(parts)))
    cap = (max(len(x) for x in lists) + 3) // 4 * 4
    keys = torch.full((W, cap), -1, dtype=torch.int32)
    for r, x in enumerate(lists):
        keys[r, : len(x)] = x.to(torch.int32)
    keys = keys.to(dev)
    counts = torch.tensor([len(x) for x in lists], dtype=torch.int32, device=dev)
    rows = torch.randn(W, cap, Kp, generator=g).to(dev)
    nb = range_merge_buckets(W, cap)
    div = (V + nb - 1) // nb
    dirs = torch.stack([torch.searchsorted(x, torch.arange(nb + 1) * div).to(torch.int32) for x in lists]).to(dev)
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    outs = []
    for rng in (False, True):
        dg = torch.zeros(V, Kp, device=dev)
        touched = torch.zeros(V, dtype=torch.int32, device=dev)
        emb = torch.randn(V, Kp, generator=torch.Generator().manual_seed(1)).to(dev)
        s0, s1 = torch.zeros_like(emb), torch.zeros_like(emb)
        p = H.MergeParams()
        p.keys, p.key_stride, p.rows, p.row_stride = keys.data_ptr(), cap, rows.data_ptr(), cap * Kp
        p.counts, p.count_stride = counts.data_ptr(), 1
        p.W, p.cap, p.Kp, p.K1, p.key_div, p.Vmap = W, cap, Kp, Kp - 1, 1, V
        p.emb, p.s0, p.s1, p.l2 = emb.data_ptr(), s0.data_ptr(), s1.data_ptr(), 1e-3
        p.grad_scale = 1.0 / W
        o = H.OptParams()
        o.type, o.lr, o.beta1, o.beta2, o.eps = 0, 1e-3, 0.9, 0.999, 1e-8
        lrt = torch.full((1,), 1e-3, device=dev)
        o.lrt = lrt.data_ptr()
        p.opt = o
        p.step, p.mode = step.data_ptr(), MODE
        p.dense_grad, p.touched = dg.data_ptr(), touched.data_ptr()
        p.dirs, p.dir_stride, p.nb, p.bucket_div = dirs.data_ptr(), nb + 1, nb, div
        s = torch.cuda.current_stream().cuda_stream
        (H.merge_range_apply if rng else H.merge_search_apply)(p, None, s)
        torch.cuda.synchronize()
        outs.append(dg.cpu() if MODE == 1 else emb.cpu())
    d = (outs[0] - outs[1]).abs().sum(1)
    bad = torch.nonzero(d).flatten()
    print(f"mode={MODE} W={W} crowd={crowd} nb={nb} div={div} cap_lds={H.merge_range_lds_entries(Kp)} "
          f"bucket0 entries={int((dirs[:, 1] - dirs[:, 0]).sum())} bad rows={len(bad)}")
    for row in bad[:8].tolist():
        mem = [int((lists[r] == row).any()) for r in range(W)]
        print(f"  row {row} bucket {row // div} in ranks {mem} search {outs[0][row, :3].tolist()} range {outs[1][row, :3].tolist()}")
