"""Process-wide side streams of the fused engines.

Every FusedDeepFM used to create its own side (fetch + sort), aux and copy streams.  HIP maps
streams onto a small pool of hardware queues (GPU_MAX_HW_QUEUES, 4 on the MI355X boxes) in creation
order, and PyTorch hands out its pooled streams round-robin, so WHICH hardware queue an engine's
streams landed on — and whether the side or copy stream shared one with the step's stream or with
each other — depended on how many streams the process had created before: the TFRecord-fed
window measured 25.2 M ex/s after two earlier streams and 28.2 M after none, and the bench's window
order changed its rate by up to 20 % (profiles/r5_stream_queues.md).

Engines therefore take their streams from here: created once per device, in a fixed order (side,
aux, copy) by the first engine of the process, and shared by every later engine.  Engines run one
after another in a process, so sharing only adds ordering between work that never overlaps.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

_STREAMS: Dict[int, Tuple[torch.cuda.Stream, torch.cuda.Stream, torch.cuda.Stream]] = {}


def engine_streams(device) -> Tuple[torch.cuda.Stream, torch.cuda.Stream, torch.cuda.Stream]:
    """(side, aux, copy) streams of ``device`` — the same objects for every engine of the process."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _STREAMS.get(idx)
    if s is None:
        s = tuple(torch.cuda.Stream(device=torch.device("cuda", idx)) for _ in range(3))
        _STREAMS[idx] = s
    return s
