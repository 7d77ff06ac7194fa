"""Debug: device-parsed ring contents at a 1B-row vocabulary."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rocfm.data import tfrecord as T
from rocfm.data.synthetic import write_synthetic_tfrecord
from rocfm.models.deepfm import ModelSpec
from rocfm.models.fused import FusedDeepFM
from rocfm.ops.decode import decode_on_device
from rocfm.optim import OptHParams

V = int(os.environ.get("V", "1000000000")); S = 64
B, F, n = 256, 39, 73
d = tempfile.mkdtemp(); f = os.path.join(d, "tr.tfrecords")
write_synthetic_tfrecord(f, B * n, V, F, seed=4)
dev = torch.device("cuda")
host = [tuple(x.clone() for x in g) for g in T.TFRecordDataset([f], F, B, V, num_threads=2).groups(8, hold=2)]
ids = torch.cat([g[0] for g in host])
# 1. the parser alone
ok = True
for g in T.TFRecordDataset([f], F, B, V, num_threads=2).raw_groups(S, hold=2):
    di, dv, dl, err = decode_on_device(g.bytes, g.offs, g.n, B, F, dev, V)
    hi = g.decode_host(F, V)[0]
    ok &= torch.equal(di.cpu(), hi)
    print("parser alone: group n", g.n, "equal", torch.equal(di.cpu(), hi), "err", err.tolist(), flush=True)
spec = ModelSpec(V, F, 10, [128, 64, 32], [0.5] * 3, l2_reg=1e-4)
e = FusedDeepFM(spec, OptHParams(name="Adam", lr=1e-3), B, dev, params=None, seed=7)
print("engine built; mem GB", torch.cuda.memory_allocated() / 1e9, flush=True)
for g in T.TFRecordDataset([f], F, B, V, num_threads=2).raw_groups(S, hold=2):
    di, dv, dl, err = decode_on_device(g.bytes, g.offs, g.n, B, F, dev, V)
    print("parser beside the engine: equal", torch.equal(di.cpu(), g.decode_host(F, V)[0]), "err", err.tolist(), flush=True)
got = e.train_stream(T.TFRecordDataset([f], F, B, V, num_threads=2).raw_groups(S, hold=2), S, hold=2)
torch.cuda.synchronize()
ring = e.stream_ring()
r = ring[0][:n].cpu()
print("trained", got, "halt", e.halt_word.tolist(), "raw_dev err", e._raw_dev[3].tolist() if e._raw_dev else None)
print("ring nonzero ids", int((r != 0).sum()), "of", r.numel(), "batches equal:",
      [int(torch.equal(r[i], ids[i])) for i in range(n)])
print("R", ring[0].shape[0], "start", getattr(e, "_start_batch", None))
