"""Pin a rank's host threads to the NUMA node of its GPU.

One process per GPU: the host side of a step (request arena, pinned
staging, the scanner's worker threads, the H2D copies they feed) should sit
on the socket the GPU's PCIe root hangs off, or every copy crosses the
inter-socket link and the host work runs on remote memory. The reference
has no GPU and no equivalent; its servers are plain processes
(server_helper.hpp:66-290).

The node comes from sysfs (``/sys/bus/pci/devices/<bdf>/numa_node``) for
the device's PCI address. ``sched_setaffinity`` applies to the calling
thread and to threads it starts later, so call ``bind_to_device`` right
after selecting the device, before worker pools and pinned buffers exist.

``JB_NUMA_BIND``: ``auto`` (default: the GPU's node), ``off``, or a node
number (measurements: ``tools/bench_numa.sh``).
"""
from __future__ import annotations

import os

_bound: dict = {}


def _cpulist(text: str) -> set[int]:
    cpus: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def node_cpus(node: int, sysfs: str = "/sys/devices/system/node") -> set[int]:
    try:
        with open(f"{sysfs}/node{node}/cpulist") as f:
            return _cpulist(f.read())
    except OSError:
        return set()


def device_node(index: int) -> int | None:
    """NUMA node of GPU ``index`` (None when unknown)."""
    import torch
    p = torch.cuda.get_device_properties(index)
    bdf = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            n = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return n if n >= 0 else None


def bind_to_device(index: int) -> dict:
    """Restrict this thread (and threads started later) to the CPUs of the
    GPU's NUMA node that it may already run on. Returns what was done:
    {"node", "cpus", "before"}; {} when disabled or unknown."""
    mode = os.environ.get("JB_NUMA_BIND", "auto").strip().lower()
    if mode in ("off", "0", "no", "none"):
        return {}
    if not hasattr(os, "sched_setaffinity"):
        return {}
    node = device_node(index) if mode == "auto" else int(mode)
    if node is None:
        return {}
    before = os.sched_getaffinity(0)
    cpus = node_cpus(node) & before
    if not cpus:
        return {}
    os.sched_setaffinity(0, cpus)
    _bound.update(node=node, cpus=len(cpus), before=len(before))
    return dict(_bound)


def binding() -> dict:
    return dict(_bound)
