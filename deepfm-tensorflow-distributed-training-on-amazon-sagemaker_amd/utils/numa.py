"""Host threads next to the GPU: the CPUs of the current GPU's NUMA node (sysfs, read-only) and an
opt-in affinity binding of the calling thread (its children — the loader's reader / worker
threads, created afterwards — inherit it, and the pinned staging buffers they first touch land
on that node).  profiles/r5_stream_queues.md: the TFRecord window's copy stream (H2D + device
parse) took 2-3× longer per group in some processes, with the GPU's clock and temperature equal.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_numa_node(device_index: int = 0) -> Optional[int]:
    """NUMA node of the GPU's PCI function, or None (no sysfs entry / -1)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        paths = glob.glob(f"/sys/bus/pci/devices/{bdf}/numa_node")
        if not paths:
            return None
        n = int(open(paths[0]).read().strip())
        return n if n >= 0 else None
    except Exception:  # noqa: BLE001 — diagnostics / an optional binding never fail a run
        return None


def gpu_local_cpus(device_index: int = 0) -> Optional[List[int]]:
    """This process's allowed CPUs that sit on the GPU's NUMA node (None if unknown or empty)."""
    n = gpu_numa_node(device_index)
    if n is None:
        return None
    try:
        node = set(_parse_cpulist(open(f"/sys/devices/system/node/node{n}/cpulist").read()))
    except OSError:
        return None
    local = sorted(node & os.sched_getaffinity(0))
    return local or None


def bind_to_gpu_node(device_index: int = 0, min_cpus: int = 4) -> Optional[List[int]]:
    """Restrict the calling thread (and the threads it creates afterwards) to the GPU-local CPUs
    of its allowed set, if there are at least ``min_cpus`` of them.  Returns the CPUs bound to."""
    local = gpu_local_cpus(device_index)
    if not local or len(local) < min_cpus or set(local) == os.sched_getaffinity(0):
        return None
    os.sched_setaffinity(0, local)
    return local
