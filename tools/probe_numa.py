"""Probe: the current GPU's NUMA node, the nodes' CPU lists and this process's allowed CPUs."""
import glob
import os

import torch

props = torch.cuda.get_device_properties(0)
bdf = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
print("gpu bdf", bdf)
for p in glob.glob(f"/sys/bus/pci/devices/{bdf}/numa_node"):
    print("gpu numa_node", open(p).read().strip())
for n in sorted(glob.glob("/sys/devices/system/node/node*/cpulist")):
    print(n.split("/")[-2], open(n).read().strip())
aff = sorted(os.sched_getaffinity(0))
print("allowed cpus", len(aff), aff[:8], "...", aff[-8:])
print("cpu_count", os.cpu_count())
