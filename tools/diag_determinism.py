"""Diagnostic: train the same batches twice through 16-step graphs and twice through per-step
launches; print which runs' weights differ (bitwise) and by how much."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rocfm.models.deepfm import ModelSpec, init_params  # noqa: E402
from rocfm.models.fused import FusedDeepFM  # noqa: E402
from rocfm.optim import OptHParams  # noqa: E402


def main():
    dev = torch.device("cuda")
    spec = ModelSpec(feature_size=20000, field_size=39, embedding_size=int(os.environ.get("K", "10")),
                     layers=[128, 64, 32], keep_probs=[0.5, 0.5, 0.5], l2_reg=1e-4)
    hp = OptHParams(name="Adam", lr=1e-3)
    B = 256
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 20000, (8, B, 39), generator=g, dtype=torch.int32)
    ids[:, :, :13] = torch.arange(1, 14, dtype=torch.int32)
    vals = torch.rand(8, B, 39, generator=g)
    labels = (torch.rand(8, B, generator=g) < 0.3).float()
    out = {}
    runs = [(16, 0), (16, 1), (1, 0), (1, 1)]
    for S, rep in runs:
        eng = FusedDeepFM(spec, hp, B, dev, params=init_params(spec, 1), seed=3)
        eng.attach_pool(ids.to(dev), vals.to(dev), labels.to(dev))
        eng.train_steps(int(os.environ.get("STEPS", "40")), S)
        torch.cuda.synchronize()
        out[(S, rep)] = {k: v.detach().cpu().clone() for k, v in eng.parameters_tf().items()}
    keys = list(out)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            a, b = out[keys[i]], out[keys[j]]
            diffs = [(k, float((a[k] - b[k]).abs().max())) for k in a if not torch.equal(a[k], b[k])]
            print(keys[i], keys[j], "equal" if not diffs else diffs[:4], flush=True)


if __name__ == "__main__":
    main()
