"""Diagnostic: per-phase durations of the fused kernels from in-kernel s_memrealtime stamps.

Stamps are recorded by thread 0 of every workgroup (100 MHz real-time counter).  Prints the mean /
max over workgroups of each phase's duration (µs) and of the whole kernel, for a few eager steps.
Not a performance measurement of the real kernels (stamps add a little work).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.data.synthetic import SyntheticCriteo  # noqa: E402
from rocfm.models.deepfm import ModelSpec, init_params  # noqa: E402
from rocfm.models.fused import FusedDeepFM  # noqa: E402
from rocfm.optim import OptHParams  # noqa: E402


def report(name, st, idx, labels):
    st = st[:, idx].double()
    valid = (st > 0).all(1)
    st = st[valid]
    d = (st[:, 1:] - st[:, :-1]) * 0.01  # ticks of 10 ns → µs
    tot = (st[:, -1] - st[:, 0]) * 0.01
    span = (st[:, -1].max() - st[:, 0].min()) * 0.01
    print(f"== {name}: {int(valid.sum())} workgroups, kernel span {span:.2f} us, per-WG total mean {tot.mean():.2f} max {tot.max():.2f}")
    off = ((st[:, 0] - st[:, 0].min()) * 0.01).sort().values
    if off.numel():
        q = lambda f: float(off[min(off.numel() - 1, int(f * off.numel()))])  # noqa: E731
        print(f"   entry offsets p50 {q(.5):.2f} p90 {q(.9):.2f} p99 {q(.99):.2f} max {float(off[-1]):.2f}; "
              f"workgroups entering > 2 us late: {int((off > 2).sum())}")
    for i in range(d.shape[1]):
        print(f"   {labels[i]:<28} mean {d[:, i].mean():7.2f}  max {d[:, i].max():7.2f}")


def main():
    # MULTI=1: stamps from the multi-step graph path (step_tail's fused wgrad + embedding roles);
    # default: the per-step path (separate mlp_wgrad / emb_rows_update launches)
    B = int(os.environ.get("B", "1024"))
    V = int(os.environ.get("V", "1000000"))
    K = int(os.environ.get("K", "10"))
    generic = os.environ.get("GENERIC", "0") == "1"  # runtime-shape row kernel (the only one with stamps
    #                                                   besides the 39x10 128-64-32 training kernel)
    dev = torch.device("cuda")
    layers = [int(x) for x in os.environ.get("LAYERS", "128,64,32").split(",")]
    spec = ModelSpec(V, 39, K, layers, [0.5] * len(layers), l2_reg=1e-4)
    multi = os.environ.get("MULTI", "0") == "1"  # the multi-step graph path (fused step_tail)
    eng = FusedDeepFM(spec, OptHParams("Adam", 5e-4), B, dev, params=init_params(spec, 1), use_graph=multi,
                      force_generic_kernels=generic, compute_dtype=os.environ.get("DTYPE", "bf16"))
    gen = SyntheticCriteo(V, 39, seed=1)
    g = torch.Generator(device=dev).manual_seed(1)
    pool = [gen.batch(B, dev, g) for _ in range(8)]
    eng.attach_pool(torch.stack([x[0] for x in pool]), torch.stack([x[1] for x in pool]),
                    torch.stack([x[2] for x in pool]))
    for _ in range(6):
        eng.train_step()
    torch.cuda.synchronize()
    nrows = eng.Bp // 4  # ≥ the row kernel's workgroups (4..16 examples each)
    s_rows = torch.zeros(nrows * 16, dtype=torch.int64, device=dev)
    s_wg = torch.zeros(4096 * 16, dtype=torch.int64, device=dev)
    s_emb = torch.zeros(max((eng.n_lookup + 255) // 256, 1024) * 16, dtype=torch.int64, device=dev)  # ≥ per-WG slots
    for p in range(2):
        eng.rows_params[p].stamps = s_rows.data_ptr()
        eng.wgrad_params[p].stamps = s_wg.data_ptr()
        eng.emb_params[p].stamps = s_emb.data_ptr()
    abl = int(os.environ.get("ABLATE", "0"))
    sync = torch.zeros(4, dtype=torch.int32, device=dev)  # ABLATE bit 3: the grid barrier's counters
    for p in range(2):
        eng.rows_params[p].ablate = abl
        if abl & 8:
            eng.rows_params[p].bn_sync, eng.rows_params[p].bn_error = sync.data_ptr(), sync[2:].data_ptr()
    if multi:
        eng.train_steps(8, 4)  # builds the multi-step parameter blocks
        for q in range(2):
            for k in range(eng.mS):
                rows, wp, _, ep, _ = eng.m_params[q][k]
                rows.stamps, wp.stamps, ep.stamps = s_rows.data_ptr(), s_wg.data_ptr(), s_emb.data_ptr()
                rows.ablate = abl
                if abl & 8:
                    rows.bn_sync, rows.bn_error = sync.data_ptr(), sync[2:].data_ptr()
        eng._m_graphs = {}  # recapture with the stamp pointers
    for _ in range(3):
        s_rows.zero_(); s_wg.zero_(); s_emb.zero_()
        if multi:
            eng.train_steps(4, 4)
        else:
            eng.train_step()
        torch.cuda.synchronize()
    print("ablate", abl)
    report("deepfm_rows", s_rows.view(-1, 16).cpu(), [0, 1, 2, 3, 4, 5, 9, 10, 11, 12],
           ["0 ids/vals stage", "A gather+e+h0", "B FM + h0T store", "C layer0 fwd", "C layer1 fwd",
            "C layer2 fwd", "D head + dz_L", "E backward (3 GEMMs)", "F FM bwd + contrib"])
    if abl & 8:
        report("deepfm_rows grid barrier (diagnostic)", s_rows.view(-1, 16).cpu(), [13, 14], ["grid barrier"])
        print("   barrier timeouts:", int(sync[2].item()))
    wg = s_wg.view(-1, 16).cpu()
    report("mlp_wgrad (tile WGs)", wg[wg[:, 1] > 0], [0, 1, 2], ["MFMA + LDS reduce", "epilogue (opt+bf16)"])
    # the fused tail's workgroups from entry to exit (stamps 15 / 14, both roles; multi-step path)
    em = s_emb.view(-1, 16).cpu()
    ent = torch.cat([em[em[:, 15] > 0, 15], wg[wg[:, 15] > 0, 15]]).double()
    ext = torch.cat([em[em[:, 14] > 0, 14], wg[wg[:, 14] > 0, 14]]).double()
    if ent.numel() and ext.numel():
        t0 = ent.min()
        off = ((ent - t0) * 0.01).sort().values
        ex = ((ext - t0) * 0.01).sort().values
        q = lambda v, f: float(v[min(v.numel() - 1, int(f * v.numel()))])  # noqa: E731
        print(f"== step tail (all {ent.numel()} workgroups): first entry → last exit {float(ex[-1]):.2f} us; entry "
              f"offsets p50 {q(off, .5):.2f} p90 {q(off, .9):.2f} max {float(off[-1]):.2f}; exits p50 {q(ex, .5):.2f} "
              f"p90 {q(ex, .9):.2f} max {float(ex[-1]):.2f}")
        # the last exits by role (emb: its workgroup index; wgrad: its index among the wgrad workgroups)
        ne = int((em[:, 15] > 0).sum())
        rows_ = [("emb", i, float(em[i, 15] - t0) * 0.01, float(em[i, 14] - t0) * 0.01)
                 for i in range(em.shape[0]) if em[i, 15] > 0]
        rows_ += [("wgrad", i, float(wg[i, 15] - t0) * 0.01, float(wg[i, 14] - t0) * 0.01)
                  for i in range(wg.shape[0]) if wg[i, 15] > 0]
        rows_.sort(key=lambda r: -r[3])
        print("   last exits: " + "; ".join(f"{r} {i} (entry {a:.2f}, exit {b:.2f})" for r, i, a, b in rows_[:6])
              + f"  [{ne} emb workgroups]")
    if getattr(eng, "m_eplan", False) and multi:  # the planned embedding role (emb_plan_body.h)
        st = s_emb.view(-1, 16).cpu()
        report("emb_plan (planned items)", st, [0, 1, 2, 3],
               ["keys+rows+scan+pieces", "publish + complete runs", "split-run combine"])
        # the last step's plan: entries and run heads per item, and the slowest items
        q = eng._mq ^ 1  # parity of the last graph
        k = eng.mS - 1
        nw = eng.m_plan_nw
        it = eng.m_pitems[q, k * nw * 4:(k + 1) * nw * 4].view(nw, 4).cpu().long()
        sk = eng.m_sk[q, k * eng.n_lookup:(k + 1) * eng.n_lookup].cpu().long()
        heads = torch.ones_like(sk, dtype=torch.bool)
        heads[1:] = sk[1:] != sk[:-1]
        ent = (it[:, 1] - it[:, 0]).clamp(min=0)
        hd = torch.tensor([int(heads[a:b].sum()) if b > a else 0 for a, b in it[:, :2].tolist()])
        live = ent > 0
        print(f"   items: {int(live.sum())} of {nw}; entries per item min {int(ent[live].min())} mean "
              f"{float(ent[live].float().mean()):.0f} max {int(ent[live].max())}; heads min {int(hd[live].min())} "
              f"mean {float(hd[live].float().mean()):.0f} max {int(hd[live].max())}; split-run slots "
              f"{int((it[:, 3] >= 0).sum())}")
        stf = st.double()
        tot = (stf[:nw, 3] - stf[:nw, 0]) * 0.01
        order = torch.argsort(tot, descending=True)[:6]
        # where each tail workgroup ran (stamp 13: XCC << 32 | HW_ID; CU = HW_ID bits 8-15)
        wgs = wg[wg[:, 15] > 0]
        hw = torch.cat([st[:nw, 13], wgs[:, 13]]).long()
        place = [(int(h) >> 32, (int(h) >> 8) & 0xff) for h in hw.tolist()]
        cnt = {}
        for pl in place:
            cnt[pl] = cnt.get(pl, 0) + 1
        shared = {pl for pl, c in cnt.items() if c > 1}
        per_xcc = [sum(1 for x, _ in place if x == k) for k in range(8)]
        print(f"   placement: {len(cnt)} distinct CUs for {len(place)} tail workgroups; CUs holding 2+: {len(shared)}; "
              f"workgroups per XCC {per_xcc}")
        t0 = float(torch.cat([st[:nw, 15], wgs[:, 15]]).double().min())
        for w in order.tolist():
            ph = [(stf[w, j + 1] - stf[w, j]) * 0.01 for j in range(3)]
            print(f"   slow item {w:3d}: total {tot[w]:.2f} us (entry +{(stf[w, 15] - t0) * 0.01:.2f}, phases "
                  f"{ph[0]:.2f} / {ph[1]:.2f} / {ph[2]:.2f}), entries {int(ent[w])}, heads {int(hd[w])}, "
                  f"lead {int(it[w, 2])}, tail {int(it[w, 3])}, xcc {place[w][0]} cu {place[w][1]:#04x}"
                  f"{' SHARED' if place[w] in shared else ''}")
        xt = [[float(tot[w]) for w in range(nw) if ent[w] > 0 and place[w][0] == k] for k in range(8)]
        print("   item total by XCC (mean / max): " + ", ".join(
            f"{k}: {sum(v) / len(v):.2f}/{max(v):.2f}" for k, v in enumerate(xt) if v))
        return
    report("emb_rows_update", s_emb.view(-1, 16).cpu(), [0, 1, 2, 3, 4],
           ["keys+rows+scan+heads", "end search", "continuation", "optimizer items"])
    # the slowest embedding workgroups of the last step, with their chunk's run-head count
    p = (eng._i - 1) % 2
    sk = eng.skeys[p].cpu().long()
    heads = torch.ones_like(sk, dtype=torch.bool)
    heads[1:] = sk[1:] != sk[:-1]
    chunk = eng.H.tail_chunk() if eng.Kp <= 48 else 256  # step_tail's / emb_update's entries per workgroup
    st = s_emb.view(-1, 16).cpu().double()
    nwg = (sk.numel() + chunk - 1) // chunk
    tot = (st[:nwg, 4] - st[:nwg, 0]) * 0.01
    opt = (st[:nwg, 4] - st[:nwg, 3]) * 0.01
    order = torch.argsort(tot, descending=True)[:6]
    for w in order.tolist():
        h = int(heads[w * chunk:(w + 1) * chunk].sum())
        print(f"   slow emb WG {w:3d}: total {tot[w]:.2f} us, optimizer items {opt[w]:.2f} us, run heads {h}")
    hs = [int(heads[w * chunk:(w + 1) * chunk].sum()) for w in range(nwg)]
    print(f"   run heads per chunk: min {min(hs)} mean {sum(hs) / len(hs):.0f} max {max(hs)}")


if __name__ == "__main__":
    main()
