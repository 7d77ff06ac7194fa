"""Fault injection for tests — driven by the ``ROCFM_FAULT`` environment variable:

    ROCFM_FAULT=kill_rank:R@step:S     rank R exits abruptly (os._exit(17)) after global step S
    ROCFM_FAULT=hang_rank:R@step:S     rank R stops making progress after step S (watchdog tests)
    ROCFM_FAULT=nan_loss@step:S        the loss check sees NaN at step S (numerics-guard tests)

Several faults may be given separated by ','.  Faults fire only in the first attempt of a job
(``ROCFM_RESTART`` unset or 0, see rocfm.launch) so that restart tests converge.  ``corrupt_record(path, index)`` flips payload bytes
of one TFRecord (CRC then fails: tests of ``on_bad_record=fail|skip``).
"""
from __future__ import annotations

import os
import re
import struct
import time
from typing import List, Optional, Tuple

_RX = re.compile(r"^(kill_rank|hang_rank):(\d+)@step:(\d+)$|^(nan_loss)@step:(\d+)$")


def parse(spec: Optional[str] = None) -> List[Tuple[str, int, int]]:
    spec = os.environ.get("ROCFM_FAULT", "") if spec is None else spec
    out = []
    for part in filter(None, (p.strip() for p in spec.split(","))):
        m = _RX.match(part)
        if not m:
            raise ValueError(f"bad ROCFM_FAULT entry {part!r}")
        if m.group(1):
            out.append((m.group(1), int(m.group(2)), int(m.group(3))))
        else:
            out.append((m.group(4), -1, int(m.group(5))))
    return out


class FaultInjector:
    def __init__(self, rank: int, spec: Optional[str] = None):
        self.rank = rank
        restarted = os.environ.get("ROCFM_RESTART", "0") not in ("", "0")
        self.faults = [] if (restarted and spec is None) else parse(spec)

    def __bool__(self) -> bool:
        return bool(self.faults)

    def after_step(self, step: int) -> None:
        for kind, r, s in self.faults:
            if step != s or (r >= 0 and r != self.rank):
                continue
            if kind == "kill_rank":
                os._exit(17)
            if kind == "hang_rank":
                while True:
                    time.sleep(3600)

    def corrupt_loss(self, step: int) -> bool:
        return any(k == "nan_loss" and s == step for k, _, s in self.faults)


def corrupt_record(path: str, index: int) -> None:
    """Flip the first payload byte of record ``index`` (its data CRC no longer matches)."""
    with open(path, "r+b") as f:
        for _ in range(index):
            (n,) = struct.unpack("<Q", f.read(8))
            f.seek(4 + n + 4, os.SEEK_CUR)
        (n,) = struct.unpack("<Q", f.read(8))
        f.seek(4, os.SEEK_CUR)
        pos = f.tell()
        b = f.read(1)
        f.seek(pos)
        f.write(bytes([b[0] ^ 0xFF]))
