"""Pure-PyTorch/numpy references of the HIP kernels.

Every HIP kernel has an oracle here with the *same* numerics contract (where the kernel rounds to
bf16, the oracle rounds at the same point), so kernel tests compare against a plain fp32
PyTorch computation of the same op:

* ``philox4x32_10`` / ``dropout_masks`` — bit-exact replica of ``dropout_bits`` in csrc/common.h
* ``fused_step_reference`` — deepfm_rows.hip + mlp_wgrad.hip (forward, head, backward, dW/db)
* ``emb_grad_reference`` — sort + emb_update.hip aggregation (Σ per unique id)
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 on uint64 numpy arrays holding 32-bit values (vectorised)."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint64) & MASK32 for x in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & 0xFFFFFFFF)
    k1 = np.uint64(k1 & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK32, lo1, (hi0 ^ c3 ^ k1) & MASK32, lo0
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return c0, c1, c2, c3


def dropout_masks(seed: int, layer: int, step: int, rows: int, cols: int, keep: float) -> torch.Tensor:
    """Keep mask [rows, cols] (bool) exactly as deepfm_rows.hip draws it."""
    assert rows % 4 == 0
    rg = np.repeat(np.arange(rows // 4, dtype=np.uint64), cols)
    cc = np.tile(np.arange(cols, dtype=np.uint64), rows // 4)
    x, y, z, w = philox4x32_10(rg, cc, np.uint64(layer), np.uint64(step & 0xFFFFFFFF), seed & 0xFFFFFFFF,
                               (seed >> 32) & 0xFFFFFFFF)
    lanes = np.stack([x, y, z, w], axis=1).reshape(rows // 4, cols, 4)  # [rg, col, lane]
    u = (lanes >> np.uint64(8)).astype(np.float64) / 16777216.0
    keepm = (u.astype(np.float32) < np.float32(keep))
    return torch.from_numpy(np.ascontiguousarray(keepm.transpose(0, 2, 1).reshape(rows, cols)))


def bf16(x: torch.Tensor) -> torch.Tensor:
    """Round to bf16 (RNE) and back to f32."""
    return x.to(torch.bfloat16).to(torch.float32)


def fused_step_reference(emb: torch.Tensor, layers: List[Dict[str, torch.Tensor]], w_out: torch.Tensor,
                         b_out: float, fm_bias: float, ids: torch.Tensor, vals: torch.Tensor,
                         labels: torch.Tensor, K: int, keeps: List[float], masks: Optional[List[torch.Tensor]],
                         inv_scale: float, train: bool = True, loss_type: int = 0, fp8: bool = False,
                         bn: Optional[List[Dict[str, torch.Tensor]]] = None, bn_eps: float = 1e-3):
    """Forward + backward with the fused kernels' numerics, on unpadded shapes.

    ``emb`` [V, Kp] (cols 0..K-1 fm_v, col K fm_w); ``layers[l]`` = {W [in,out] f32, b [out]}.
    ``bn[l]`` = {gamma, beta, mean, var} enables batch norm after each ReLU (batch moments when
    training, the given moving moments otherwise); its outputs include the batch moments and the
    γ / β gradients.  Returns dict with prob, loss_rows, g, contrib [B*F, K+1], dW/db per layer,
    dw_out, d_bout.
    """
    B, F = ids.shape
    rows = emb[ids.long()]  # [B,F,Kp]
    V = rows[..., :K]
    w = rows[..., K]
    x = vals
    e = V * x.unsqueeze(-1)
    S = e.sum(1)
    y_lin = fm_bias + (w * x).sum(1) + 0.5 * (S * S - (e * e).sum(1)).sum(1)
    h = [bf16(e.reshape(B, F * K))]
    bn_state = []
    for li, L in enumerate(layers):
        if fp8 and li == 0:
            z = fp8_row_tensor_matmul(h[-1], L["W"]) + L["b"]
        else:
            z = h[-1] @ bf16(L["W"]) + L["b"]
        a = torch.relu(z)
        if bn is not None:
            if train:
                mean, var = a.mean(0), a.var(0, unbiased=False)
            else:
                mean, var = bn[li]["mean"], bn[li]["var"]
            rstd = torch.rsqrt(var + bn_eps)
            xh = (a - mean) * rstd
            bn_state.append((a, xh, rstd, mean, var))
            a = xh * bn[li]["gamma"] + bn[li]["beta"]
        if train and keeps[li] < 1.0:
            a = torch.where(masks[li], a / keeps[li], torch.zeros_like(a))
        h.append(bf16(a))
    y = y_lin + h[-1] @ w_out + b_out
    p = torch.sigmoid(y)
    if loss_type == 0:
        loss = torch.clamp(y, min=0) - y * labels + torch.log1p(torch.exp(-y.abs()))
        g = (p - labels) * inv_scale
    else:
        loss = (p - labels) ** 2
        g = 2 * (p - labels) * p * (1 - p) * inv_scale
    out = {"prob": p, "loss_rows": loss, "g": g, "y": y}
    if not train:
        return out
    nl = len(layers)
    dz = [None] * (nl + 1)
    dgamma, dbeta = [None] * nl, [None] * nl

    def undrop(l, d):  # gradient through layer l's dropout
        if keeps[l] < 1.0:
            return torch.where(masks[l], d / keeps[l], torch.zeros_like(d))
        return d

    def bn_back(l, dy):  # dy: gradient w.r.t. layer l's BN output → bf16 dz of its pre-activation
        r, xh, rstd, _, _ = bn_state[l]
        dgamma[l], dbeta[l] = (dy * xh).sum(0), dy.sum(0)
        dr = bn[l]["gamma"] * rstd * (dy - dy.mean(0) - xh * (dy * xh).mean(0))
        return bf16(torch.where(r > 0, dr, torch.zeros_like(dr)))

    if bn is not None:
        dz[nl] = bn_back(nl - 1, undrop(nl - 1, g[:, None] * w_out[None, :]))
    else:
        dz[nl] = bf16(torch.where(h[nl] > 0, g[:, None] * w_out[None, :] / keeps[nl - 1], torch.zeros_like(h[nl])))
    dh0 = None
    for a in range(nl, 0, -1):
        if fp8 and a == 1:  # the input layer's dgrad on fp8 MFMA (dz per row, W0ᵀ per tensor)
            dh = fp8_row_tensor_matmul(dz[a], layers[0]["W"].t())
        else:
            dh = dz[a] @ bf16(layers[a - 1]["W"]).t()
        if a - 1 >= 1:
            if bn is not None:
                dz[a - 1] = bn_back(a - 2, undrop(a - 2, dh))
            else:
                dz[a - 1] = bf16(torch.where(h[a - 1] > 0, dh / keeps[a - 2], torch.zeros_like(dh)))
        else:
            dh0 = dh
    de = g[:, None, None] * (S[:, None, :] - e) + dh0.reshape(B, F, K)
    contrib = torch.cat([x.unsqueeze(-1) * de, (g[:, None] * x).unsqueeze(-1)], dim=-1).reshape(B * F, K + 1)
    out["contrib"] = contrib
    out["dW"] = [h[a].t() @ dz[a + 1] for a in range(nl)]
    out["db"] = [dz[a + 1].sum(0) for a in range(nl)]
    out["dw_out"] = h[nl].t() @ g
    out["d_bout"] = g.sum()
    out["h"] = h
    out["dz"] = dz
    if bn is not None:
        out["dgamma"], out["dbeta"] = dgamma, dbeta
        out["bn_mean"] = [st[3] for st in bn_state]
        out["bn_var"] = [st[4] for st in bn_state]
    return out


FP8_MAX = 448.0  # largest finite float8 e4m3fn


def fp8_row_tensor_matmul(A: torch.Tensor, W: torch.Tensor, w_amax: Optional[float] = None) -> torch.Tensor:
    """A·W on fp8-e4m3 operands: A quantised per row, W (the f32 master weights) with ONE scale
    448 / w_amax (default: max |W|, what a host refresh uses; training refreshes use the previous
    weights' max, deepfm_rows.h Fp8W0) — the fused kernel's pre-quantised input-layer GEMMs."""
    sa = FP8_MAX / A.abs().amax(1, keepdim=True).clamp_min(1e-30)
    am = float(W.abs().max()) if w_amax is None else float(w_amax)
    sb = FP8_MAX / max(am, 1e-30)
    Aq = (A * sa).to(torch.float8_e4m3fn).float()
    Wq = (W * sb).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float()
    return (Aq @ Wq) * ((1.0 / sa) * (1.0 / sb))


def emb_grad_reference(ids: torch.Tensor, contrib: torch.Tensor):
    """Σ of per-lookup gradient rows per unique id → (unique ids, summed rows)."""
    flat = ids.reshape(-1).long()
    uniq, inv = torch.unique(flat, return_inverse=True)
    acc = torch.zeros(len(uniq), contrib.shape[1], dtype=contrib.dtype)
    acc.index_add_(0, inv, contrib)
    return uniq, acc


def shard_route_reference(ids: np.ndarray, W: int, Vs: int, cap: int):
    """Oracle of shard.hip's routing: (send_ids [W,cap] with -1 padding, local_idx [n], counts [W]).

    Owner of id i is i % W; an owner's requests are its unique ids in ascending local-row order;
    lookup l reads received row o*cap + j of its id's owner o.
    """
    ids = np.asarray(ids, dtype=np.int64).reshape(-1)
    send = np.full((W, cap), -1, dtype=np.int64)
    local = np.zeros(len(ids), dtype=np.int64)
    counts = np.zeros(W, dtype=np.int64)
    for o in range(W):
        mine = np.unique(ids[ids % W == o])  # ascending id == ascending local row
        counts[o] = len(mine)
        send[o, : min(len(mine), cap)] = mine[:cap]
        pos = {int(v): j for j, v in enumerate(mine)}
        for l in np.nonzero(ids % W == o)[0]:
            local[l] = o * cap + min(pos[int(ids[l])], cap - 1)
    return send, local, counts


def emb_plan_reference(keys: np.ndarray, nw: int, beta: int = 4, lsplit: int = 128):
    """Sequential replica of emb_plan.hip for ONE batch's sorted keys.

    Returns ``(items [nw, 4], slots [nw, 4])``: item k = (es, ee, lead slot, tail slot) — empty items
    are (0, 0, -1, -1) — and slot s = (key, first non-head window, last window, pieces) for every
    split run, numbered in run order.  Cuts are the run heads and, inside runs longer than
    ``lsplit``, the 64-entry window boundaries; cut c of run r goes to item
    floor((c + beta·r) / Q), Q = ceil((n + beta·U) / nw)."""
    keys = np.asarray(keys)
    n = int(keys.size)
    heads = np.flatnonzero(np.r_[True, keys[1:] != keys[:-1]]) if n else np.zeros(0, np.int64)
    U = int(heads.size)
    runs = np.r_[heads, n]
    Q = max(1, (n + beta * U + nw - 1) // nw)
    items = np.zeros((nw, 4), np.int64)
    items[:, 2:] = -1
    slots = np.zeros((nw, 4), np.int64)
    cuts = []  # (position, run, is_head)
    for r in range(U):
        s, e = int(runs[r]), int(runs[r + 1])
        cuts.append((s, r, True))
        if e - s > lsplit:
            c = (s & ~63) + 64
            while c < e:
                cuts.append((c, r, False))
                c += 64
    prev_item, nslot = -1, 0
    cur_slot = {}  # run → slot
    for j, (c, r, is_head) in enumerate(cuts):
        it = (c + beta * r) // Q
        if it != prev_item:
            items[it, 0] = c
            if prev_item >= 0:
                items[prev_item, 1] = c
            if not is_head:  # the run is split here
                if r not in cur_slot:
                    cur_slot[r] = nslot
                    s0 = int(runs[r])
                    slots[nslot] = (int(keys[s0]), c >> 6, (int(runs[r + 1]) - 1) >> 6, 1)
                    items[(s0 + beta * r) // Q, 3] = nslot
                    nslot += 1
                sl = cur_slot[r]
                items[it, 2] = sl
                slots[sl, 3] += 1
            prev_item = it
    if prev_item >= 0:
        items[prev_item, 1] = n
    return items, slots
