"""Debug: streamed wide-vocabulary training vs per-step (seg_sort paths)."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rocfm.data import tfrecord as T
from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.models.deepfm import ModelSpec
from rocfm.models.fused import FusedDeepFM
from rocfm.optim import OptHParams

V = int(os.environ.get("V", "100000000")); S = int(os.environ.get("S", "16"))
B, F = 256, 39
n = S + 9
d = tempfile.mkdtemp()
f = os.path.join(d, "tr.tfrecords")
write_synthetic_tfrecord(f, B * n, V, F, seed=4)
spec = ModelSpec(V, F, 10, [128, 64, 32], [0.5, 0.5, 0.5], l2_reg=1e-4)
hp = OptHParams(name="Adam", lr=1e-3)
dev = torch.device("cuda")
host = [tuple(x.clone() for x in g) for g in T.TFRecordDataset([f], F, B, V, num_threads=2).groups(8, hold=2)]
ids = torch.cat([g[0] for g in host]).to(dev); vals = torch.cat([g[1] for g in host]).to(dev)
labels = torch.cat([g[2] for g in host]).to(dev)
touched = torch.unique(ids.reshape(-1)).long()
print("ids max", int(ids.max()), "touched", touched.numel())
res = {}
for mode in os.environ.get("MODES", "raw,host,pool,step").split(","):
    e = FusedDeepFM(spec, hp, B, dev, params=None, seed=7, use_graph=(mode != "step"))
    e0 = e.emb[touched].clone()
    if mode in ("raw", "host"):
        ds = T.TFRecordDataset([f], F, B, V, num_threads=2)
        got = e.train_stream(ds.raw_groups(S, hold=2) if mode == "raw" else ds.groups(S, hold=2), S, hold=2)
        ring = e.stream_ring()
        print(mode, "trained", got, "composite", e.m_composite, "plain", e.m_plain, "idbits", e.m_idbits,
              "halt", e.halt_word.tolist(), "ring ids == host:", torch.equal(ring[0][:n], ids))
    elif mode == "pool":
        e.attach_pool(ids, vals, labels); e.train_steps(n, S)
        print(mode, "composite", e.m_composite, "plain", e.m_plain)
    else:
        e.attach_pool(ids, vals, labels)
        for _ in range(n): e.train_step()
    torch.cuda.synchronize(); e.check()
    res[mode] = (e.emb[touched].cpu(), e.dense.cpu())
    print(mode, "moved rows", int((e.emb[touched] != e0).any(1).sum()), "of", touched.numel(),
          "steps", e.global_step())
    del e; torch.cuda.empty_cache()
ks = list(res)
for k in ks[1:]:
    print(ks[0], "vs", k, "emb equal", torch.equal(res[ks[0]][0], res[k][0]), "dense equal",
          torch.equal(res[ks[0]][1], res[k][1]))
