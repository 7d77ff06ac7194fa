"""Per-workgroup time to load 8 waves × 16 MFMA B fragments (128 KiB per WG): B-operand pattern vs
pre-swizzled contiguous layout, at 1..256 workgroups."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from rocfm.ops import require_hip

H = require_hip()
K = 128
W = torch.randint(0, 1 << 15, (8 * 2 * 16 * 4, K), dtype=torch.int16, device="cuda")  # ≥ rows needed
sink = torch.zeros(512, dtype=torch.int32, device="cuda")
for nb in (1, 64, 256):
    for swz in (0, 1):
        st = torch.zeros(nb * 2, dtype=torch.int64, device="cuda")
        for _ in range(3):
            H.frag_probe(W.data_ptr(), K, swz, nb, st.data_ptr(), sink.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        d = (st.view(-1, 2)[:, 1] - st.view(-1, 2)[:, 0]).double() * 0.01
        print(f"blocks {nb:4d} swizzled {swz}: per-WG load time mean {d.mean():.2f} us max {d.max():.2f} us "
              f"({8 * 16 * 64 * 16 / 1024:.0f} KiB per WG)", flush=True)
