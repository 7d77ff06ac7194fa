"""Device-side Example parsing (csrc/kernels/decode.hip) outside the training engine.

``decode_on_device`` parses undecoded batches (``TFRecordDataset.raw_groups`` items, or any
payload bytes + offsets) into device tensors; the engine's ``train_stream`` launches the same
kernel straight into its batch ring.  Used by tests and by tools that want decoded batches on the
GPU without training.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch

from . import require_hip

PARSE_STATUS = {0: "ok", 1: "malformed Example protobuf", 2: "missing feature",
                3: "wrong feature length (FixedLenFeature expects field_size values)",
                4: "id out of range [0, feature_size)", 5: "bad record offsets"}


def pack_payloads(payloads: Sequence[bytes], B: int) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Payloads (n·B of them, batch-major) → (bytes [n, cap] uint8, offs [n, B+1] int32, n) in the
    loader's raw layout (cap = the longest batch rounded up to 16 B)."""
    if len(payloads) % B:
        raise ValueError("payload count must be a multiple of B")
    n = len(payloads) // B
    sizes = [sum(len(p) for p in payloads[k * B:(k + 1) * B]) for k in range(n)]
    cap = max(16, (max(sizes) + 15) // 16 * 16)
    raw = torch.zeros(n, cap, dtype=torch.uint8)
    offs = torch.zeros(n, B + 1, dtype=torch.int32)
    for k in range(n):
        buf = b"".join(payloads[k * B:(k + 1) * B])
        raw[k, :len(buf)] = torch.frombuffer(bytearray(buf), dtype=torch.uint8) if buf else raw[k, :0]
        o = 0
        for r in range(B):
            offs[k, r] = o
            o += len(payloads[k * B + r])
        offs[k, B] = o
    return raw, offs, n


def decode_on_device(raw: torch.Tensor, offs: torch.Tensor, n: int, B: int, F: int, device, max_id: int = 0,
                     keys: Tuple[str, str, str] = ("label", "ids", "values")):
    """Parse n raw batches on the GPU → (ids int32 [n,B,F], vals f32 [n,B,F], labels f32 [n,B],
    err int32 [4] = (status, batch, record, 0) of the first failing record)."""
    H = require_hip()
    dev = torch.device(device)
    cap = int(raw.shape[1])
    d_raw = torch.zeros(n * cap + 64, dtype=torch.uint8, device=dev)
    d_raw[:n * cap].copy_(raw[:n].reshape(-1))
    d_offs = offs[:n].to(dev, torch.int32).contiguous()
    ids = torch.full((n, B, F), -7, dtype=torch.int32, device=dev)
    vals = torch.full((n, B, F), -7.0, dtype=torch.float32, device=dev)
    labels = torch.full((n, B), -7.0, dtype=torch.float32, device=dev)
    err = torch.zeros(4, dtype=torch.int32, device=dev)
    p = H.DecodeParams()
    p.bytes, p.offs, p.cap, p.nb, p.B, p.F = d_raw.data_ptr(), d_offs.data_ptr(), cap, int(n), int(B), int(F)
    p.ids, p.vals, p.labels = ids.data_ptr(), vals.data_ptr(), labels.data_ptr()
    p.slot0, p.R, p.max_id, p.batch0, p.err = 0, max(1, int(n)), int(max_id), 0, err.data_ptr()
    p.set_keys(*keys)
    H.decode_examples(p, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    return ids, vals, labels, err
