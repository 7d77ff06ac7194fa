"""Debug: the side chain's per-chunk run-head keys (m_hk) against the heads of the sorted keys."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.models.deepfm import ModelSpec, init_params  # noqa: E402
from rocfm.models.fused import FusedDeepFM  # noqa: E402
from rocfm.optim import OptHParams  # noqa: E402

spec = ModelSpec(feature_size=3000, field_size=39, embedding_size=10, layers=[64, 32], keep_probs=[0.7, 0.8], l2_reg=1e-3)
hp = OptHParams(name="Adam", lr=2e-3)
B = 128
g = torch.Generator().manual_seed(9)
ids = torch.randint(0, 3000, (5, B, 39), generator=g, dtype=torch.int32).cuda()
vals = torch.rand(5, B, 39, generator=g).cuda()
labels = (torch.rand(5, B, generator=g) < 0.5).float().cuda()
a = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True)
a.attach_pool(ids, vals, labels)
a.train_steps(16, 8)
torch.cuda.synchronize()
n, ch, nch = a.n_lookup, a.m_chunk, a.m_nch
print("n", n, "chunk", ch, "nch", nch, "S", a.mS, "composite", a.m_composite, "plain", a.m_plain)
bad = 0
for q in range(2):
    for k in range(a.mS):
        sk = a.m_sk[q, k * n:(k + 1) * n].cpu().numpy().view("uint32")
        hk = a.m_hk[q, k * nch * ch:(k + 1) * nch * ch].cpu().numpy().view("uint32")
        for c in range(nch):
            seg = sk[c * ch:min((c + 1) * ch, n)]
            i0 = c * ch
            heads = [seg[j] for j in range(len(seg)) if (i0 + j == 0 or sk[i0 + j] != sk[i0 + j - 1])]
            got = list(hk[c * ch:c * ch + len(heads)])
            if [int(x) for x in heads] != [int(x) for x in got]:
                bad += 1
                if bad < 4:
                    print("mismatch q", q, "k", k, "c", c, heads[:6], got[:6])
print("bad chunks", bad)
ep = a.m_params[0][0][3]
print("ep.hkeys", ep.hkeys, "rows", ep.rows, "mode", ep.mode, "sorted", ep.sorted_contrib, "id_offset", ep.id_offset,
      "id_stride", ep.id_stride, "n_dev", ep.n_dev)
