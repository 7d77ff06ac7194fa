"""Read-only snapshot of the current GPU's clock / temperature / power / throttle state (amdsmi).

Diagnostics for windows whose speed depends on the device's state rather than on the code (the
same step measured 29.5 µs cold and 36 µs after 2,000 steps, profiles/r5_stream_queues.md).  Pure
queries — nothing is set.  Returns {} when amdsmi or the metrics are unavailable.
"""
from __future__ import annotations

from typing import Dict

_HANDLE = None


def _handle():
    global _HANDLE
    if _HANDLE is not None:
        return _HANDLE
    import amdsmi
    import torch

    amdsmi.amdsmi_init()
    props = torch.cuda.get_device_properties(torch.cuda.current_device())
    want = (props.pci_domain_id, props.pci_bus_id, props.pci_device_id)
    for h in amdsmi.amdsmi_get_processor_handles():
        try:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
            dom, bus, rest = bdf.split(":")
            if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                _HANDLE = h
                return h
        except Exception:  # noqa: BLE001
            continue
    raise RuntimeError("gpu_state: no amdsmi handle matches the current device")


def snapshot() -> Dict[str, float]:
    """{gfxclk_mhz, temp_hotspot_c, power_w, throttle (the metrics' throttle/violation word)}."""
    try:
        import amdsmi

        m = amdsmi.amdsmi_get_gpu_metrics_info(_handle())
    except Exception:  # noqa: BLE001 — diagnostics never fail a run
        return {}
    out = {}
    for key, name in (("current_gfxclk", "gfxclk_mhz"), ("average_gfxclk_frequency", "gfxclk_avg_mhz"),
                      ("temperature_hotspot", "temp_hotspot_c"), ("temperature_mem", "temp_mem_c"),
                      ("current_socket_power", "power_w"), ("average_socket_power", "power_avg_w"),
                      ("throttle_status", "throttle"), ("indep_throttle_status", "throttle_indep")):
        v = m.get(key) if isinstance(m, dict) else None
        if isinstance(v, (list, tuple)):
            v = next((x for x in v if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF)), None)
        if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
            out[name] = v
    return out
