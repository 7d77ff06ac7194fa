"""Inference on an exported servable (the SavedModel ``serving_default`` signature, PS:262-272).

    pred = Predictor("/opt/ml/model")            # newest <unix-ts> bundle under the directory
    prob = pred.predict(feat_ids, feat_vals)     # int64/int32 [N,F], float32 [N,F] → float32 [N]

On a GPU with the HIP extension the fused inference kernel (deepfm_rows.hip, train=0) is used;
otherwise the eager PyTorch forward.  ``python -m rocfm.serving <bundle> <te.tfrecords> [out]``
writes one probability per line ("%f").
"""
from __future__ import annotations

import sys
from typing import Optional

import torch

from .checkpoint import load_servable
from .models.deepfm import ModelSpec, forward


class Predictor:
    def __init__(self, path: str, device: Optional[str] = None, engine: str = "auto", batch_size: int = 4096):
        meta, params = load_servable(path)
        c = meta["config"]
        self.spec = ModelSpec(feature_size=int(c["feature_size"]), field_size=int(c["field_size"]),
                              embedding_size=int(c["embedding_size"]),
                              layers=[int(x) for x in str(c["deep_layers"]).split(",")],
                              keep_probs=[float(x) for x in str(c["dropout"]).split(",")],
                              batch_norm=bool(c.get("batch_norm", False)),
                              batch_norm_decay=float(c.get("batch_norm_decay", 0.9)),
                              loss_type=c.get("loss_type", "log_loss"))
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.params = {k: v.to(self.device) for k, v in params.items()}
        self.fused = None
        if engine in ("auto", "fused") and self.device.type == "cuda":
            from .ops import has_hip

            if has_hip():
                from .models.fused import FusedDeepFM
                from .optim import OptHParams

                self.fused = FusedDeepFM(self.spec, OptHParams(name="GD", lr=0.0), batch_size, self.device,
                                         params={k: v.cpu() for k, v in params.items()}, use_graph=False)
        if engine == "fused" and self.fused is None:
            raise RuntimeError("fused inference needs a GPU and the HIP extension")

    @torch.no_grad()
    def predict(self, feat_ids, feat_vals) -> torch.Tensor:
        ids = torch.as_tensor(feat_ids).to(self.device)
        vals = torch.as_tensor(feat_vals, dtype=torch.float32).to(self.device)
        if ids.dim() != 2 or ids.shape[1] != self.spec.field_size or vals.shape != ids.shape:
            raise ValueError(f"expected feat_ids/feat_vals of shape [N, {self.spec.field_size}]")
        if self.fused is not None:
            p, _ = self.fused.predict_batch(ids.to(torch.int32), vals)
            return p.float().cpu()
        y = forward(self.params, ids.long(), vals, self.spec, train=False)
        return torch.sigmoid(y).float().cpu()


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print("usage: python -m rocfm.serving <servable_dir> <file.tfrecords> [out.txt]")
        return 2
    from .data.tfrecord import decode_file

    pred = Predictor(argv[0])
    _, ids, vals = decode_file(argv[1], pred.spec.field_size, pred.spec.feature_size)
    p = pred.predict(ids, vals)
    out = open(argv[2], "w") if len(argv) > 2 else sys.stdout
    for v in p.tolist():
        out.write("%f\n" % v)
    return 0


if __name__ == "__main__":
    sys.exit(main())
