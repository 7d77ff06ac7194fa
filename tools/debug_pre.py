"""Debug: multi-step graphs vs per-step launches — where do the parameters differ?"""
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
ids = (torch.rand(5, B, 39, generator=g) ** 3 * 3000).int().cuda()
vals = torch.rand(5, B, 39, generator=g).cuda()
labels = (torch.rand(5, B, generator=g) < 0.5).float().cuda()
for steps in (1, 2, 8, 9, 16):
    a = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=True)
    b = FusedDeepFM(spec, hp, B, "cuda", params=init_params(spec, 4), use_graph=False)
    a.attach_pool(ids, vals, labels)
    b.attach_pool(ids, vals, labels)
    a.train_steps(steps, 8)
    for _ in range(steps):
        b.train_step()
    torch.cuda.synchronize()
    de = (a.emb - b.emb).abs()
    rows = (de.amax(1) > 0).nonzero().flatten()
    print(f"steps {steps}: emb rows differing {rows.numel()} (max {de.max().item():.3g}) first {rows[:8].tolist()}; "
          f"dense max {(a.dense - b.dense).abs().max().item():.3g}; m {(a.emb_slots[0] - b.emb_slots[0]).abs().max().item():.3g} "
          f"v {(a.emb_slots[1] - b.emb_slots[1]).abs().max().item():.3g}")
    if rows.numel():
        r = rows[0].item()
        print("   row", r, "a", a.emb[r, :4].tolist(), "b", b.emb[r, :4].tolist(), "cols differing",
              (de[r] > 0).nonzero().flatten().tolist())
