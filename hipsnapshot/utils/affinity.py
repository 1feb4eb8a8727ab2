"""NUMA locality of a rank: keep its CPU work next to its GPU.

One process drives one MI355X.  Its D2H lands in pinned memory that HIP
allocates near the GPU, and the I/O engine's threads then copy those bytes
into the page cache; when the threads run on the other socket every byte
crosses the inter-socket link twice.  ``bind_to_gpu_numa`` restricts the
process (and every thread it creates afterwards) to the CPUs of the GPU's
NUMA node, intersected with the CPUs the process may use.  It is opt-in for
the library (``HIPSNAPSHOT_NUMA_BIND=1`` or an explicit call) because it
changes process state the trainer may manage itself; ``bench.py`` uses it.
"""

from __future__ import annotations

import os
from typing import List, Optional, Set

_SYS_PCI = "/sys/bus/pci/devices"
_SYS_NODE = "/sys/devices/system/node"


def _parse_cpulist(text: str) -> Set[int]:
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-")
            cpus.update(range(int(lo), int(hi) + 1))
        else:
            cpus.add(int(part))
    return cpus


def gpu_pci_bus_id(device: int) -> Optional[str]:
    try:
        import torch

        props = torch.cuda.get_device_properties(device)
        dom = getattr(props, "pci_domain_id", 0)
        return f"{dom:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    except Exception:  # noqa: BLE001
        return None


def gpu_numa_node(device: int) -> Optional[int]:
    bus = gpu_pci_bus_id(device)
    if bus is None:
        return None
    try:
        with open(os.path.join(_SYS_PCI, bus, "numa_node")) as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return node if node >= 0 else None


def node_cpus(node: int) -> Set[int]:
    try:
        with open(os.path.join(_SYS_NODE, f"node{node}", "cpulist")) as f:
            return _parse_cpulist(f.read())
    except OSError:
        return set()


def bind_to_gpu_numa(device: int, min_cpus: int = 4) -> dict:
    """Restrict this process to the allowed CPUs on ``device``'s NUMA node.

    Does nothing (and says why) when the topology is unknown, the node has
    fewer than ``min_cpus`` usable CPUs, or the process may already only run
    there.  Returns a small report dict."""
    report = {"device": device, "bound": False}
    node = gpu_numa_node(device)
    report["numa_node"] = node
    if node is None:
        report["reason"] = "GPU NUMA node unknown"
        return report
    allowed = os.sched_getaffinity(0)
    local = node_cpus(node) & allowed
    report.update(allowed=len(allowed), local=len(local))
    if len(local) < min_cpus:
        report["reason"] = f"only {len(local)} usable CPUs on node {node}"
        return report
    if local == allowed:
        report["reason"] = "already local"
        return report
    os.sched_setaffinity(0, local)
    report["bound"] = True
    return report


def maybe_bind_from_env(device: int) -> Optional[dict]:
    v = os.environ.get("HIPSNAPSHOT_NUMA_BIND", "0").strip().lower()
    if v in ("1", "true", "yes", "on"):
        return bind_to_gpu_numa(device)
    return None


def describe(devices: List[int]) -> List[dict]:
    out = []
    for d in devices:
        node = gpu_numa_node(d)
        out.append({"device": d, "pci": gpu_pci_bus_id(d), "numa_node": node,
                    "node_cpus": len(node_cpus(node)) if node is not None else None})
    return out
