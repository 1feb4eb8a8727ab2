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
from typing import Dict, List, Optional, Set

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
    """PCI address of HIP device ``device``: three attribute queries through
    the native library (``hipGetDeviceProperties``, which
    ``torch.cuda.get_device_properties`` runs, took ~130 ms the first time
    in a process), torch as the fallback."""
    try:
        from ..ops import native

        if native.hsgpu_loaded() or native.gpu_available():
            loc = native.pci_location(device)
            if loc is not None:
                return f"{loc[0]:04x}:{loc[1]:02x}:{loc[2]:02x}.0"
    except Exception:  # noqa: BLE001
        pass
    try:
        import torch

        props = torch.cuda.get_device_properties(device)
        dom = getattr(props, "pci_domain_id", 0)
        return f"{dom:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}.0"
    except Exception:  # noqa: BLE001
        return None


_numa_nodes: dict = {}


def gpu_numa_node(device: int) -> Optional[int]:
    """NUMA node of HIP device ``device`` (cached per process)."""
    if device in _numa_nodes:
        return _numa_nodes[device]
    node = None
    bus = gpu_pci_bus_id(device)
    if bus is not None:
        try:
            with open(os.path.join(_SYS_PCI, bus, "numa_node")) as f:
                node = int(f.read().strip())
        except (OSError, ValueError):
            node = None
    node = node if node is not None and node >= 0 else None
    if bus is not None:
        _numa_nodes[device] = node
    return node


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


# ---- keeping background threads off the trainer's core -----------------------
#
# A launch-bound training step (seq 512 Llama-3-8B: ~8400 kernel launches per
# 240 ms step from one Python thread) slows down whenever that thread shares
# its physical core: an SMT sibling busy with a drain writer's page-cache
# memcpy takes a large share of the core's issue slots.  ``async_take`` notes
# the core its caller runs on; the native drain's threads are created with an
# affinity mask that excludes that core's hardware threads, or every CPU of
# its L3 domain (``knobs.TUNING.drain_avoid_caller_core`` = core (default) / l3
# / 0).

_caller_cpu: List[Optional[int]] = [None]


_getcpu: list = []


def current_cpu() -> Optional[int]:
    """The CPU the calling thread last ran on: glibc's ``sched_getcpu`` (a
    vDSO call), else /proc/thread-self/stat (a file read on every
    ``async_take``)."""
    if not _getcpu:
        try:
            import ctypes

            fn = ctypes.CDLL(None, use_errno=True).sched_getcpu
            fn.restype = ctypes.c_int
            fn.argtypes = []
            _getcpu.append(fn)
        except (OSError, AttributeError):
            _getcpu.append(None)
    fn = _getcpu[0]
    if fn is not None:
        c = fn()
        if c >= 0:
            return c
    try:
        with open("/proc/thread-self/stat") as f:
            stat = f.read()
        # fields after the command name "(...)": field 39 = processor
        return int(stat.rsplit(")", 1)[1].split()[36])
    except (OSError, ValueError, IndexError):
        return None


def core_siblings(cpu: int) -> Set[int]:
    """The hardware threads of ``cpu``'s physical core (``cpu`` itself if
    the topology is unknown)."""
    try:
        with open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list") as f:
            sib = _parse_cpulist(f.read())
        return sib or {cpu}
    except OSError:
        return {cpu}


def l3_siblings(cpu: int) -> Set[int]:
    """The CPUs sharing ``cpu``'s last-level (L3) cache: one CCD on EPYC
    hosts (``cpu`` itself if the topology is unknown)."""
    base = f"/sys/devices/system/cpu/cpu{cpu}/cache"
    try:
        for idx in sorted(os.listdir(base)):
            if not idx.startswith("index"):
                continue
            with open(os.path.join(base, idx, "level")) as f:
                if f.read().strip() != "3":
                    continue
            with open(os.path.join(base, idx, "shared_cpu_list")) as f:
                return _parse_cpulist(f.read()) or {cpu}
    except OSError:
        pass
    return {cpu}


def note_caller_cpu() -> None:
    """Record the core the calling (training) thread runs on."""
    _caller_cpu[0] = current_cpu()


def mask_avoiding_caller(mode: str = "core") -> Optional[Set[int]]:
    """This thread's allowed CPUs minus the noted caller's core (``mode``
    "core") or its whole L3 domain ("l3"; the core alone when fewer than 2
    CPUs would remain), or None when nothing was noted or too few CPUs
    would remain."""
    cpu = _caller_cpu[0]
    if cpu is None or not mode:
        return None
    try:
        allowed = os.sched_getaffinity(0)
    except OSError:
        return None
    if mode == "l3":
        rest = allowed - l3_siblings(cpu) - core_siblings(cpu)
        if len(rest) >= 2 and rest != allowed:
            return rest
    rest = allowed - core_siblings(cpu)
    if len(rest) < 2 or rest == allowed:
        return None
    return rest


class threads_avoiding_caller:
    """Context manager: threads created inside it (they inherit the creating
    thread's mask) never run on the noted caller's core; the calling
    thread's own mask is restored on exit."""

    def __init__(self, enabled=True) -> None:
        # True / "core": the caller's core; "l3": its L3 domain; falsy: off
        self.mode = "core" if enabled is True else (enabled or "")
        self.prev: Optional[Set[int]] = None

    def __enter__(self) -> "threads_avoiding_caller":
        if not self.mode:
            return self
        mask = mask_avoiding_caller(self.mode)
        if mask is not None:
            try:
                self.prev = os.sched_getaffinity(0)
                os.sched_setaffinity(0, mask)
            except OSError:
                self.prev = None
        return self

    def __exit__(self, *exc) -> None:
        if self.prev is not None:
            try:
                os.sched_setaffinity(0, self.prev)
            except OSError:
                pass


# ---- native I/O threads next to their GPU --------------------------------------
#
# The native restore's readers copy page-cache pages into pinned slots that
# the GPU's SDMA engine then reads: with the threads (and the slots they
# first touch) on the GPU's NUMA node, one rank's W = 8 share restored in
# 29 ms instead of 42 (profiles/r4/restore_native/).  Binding the whole
# process is the caller's choice (``bind_to_gpu_numa``); the native jobs only
# create their own threads under the GPU node's mask.


def gpu_node_mask(device: int, min_cpus: int = 4) -> Optional[Set[int]]:
    """This thread's allowed CPUs on ``device``'s NUMA node, or None when
    unknown / too few / no narrower than the current mask."""
    node = gpu_numa_node(device)
    if node is None:
        return None
    try:
        allowed = os.sched_getaffinity(0)
    except OSError:
        return None
    local = node_cpus(node) & allowed
    if len(local) < min_cpus or local == allowed:
        return None
    return local


_SYS_MOVE_PAGES = {"x86_64": 279, "aarch64": 239}


def pages_node(addr: int, nbytes: int, samples: int = 32) -> Optional[int]:
    """The NUMA node holding most of the host pages of ``[addr, addr +
    nbytes)``, from ``samples`` pages spread over the range (``move_pages``
    with no target nodes only reports where pages are); None when unknown
    (no pages faulted in yet, no NUMA, not Linux)."""
    import ctypes
    import platform

    nr = _SYS_MOVE_PAGES.get(platform.machine())
    if nr is None or nbytes <= 0:
        return None
    page = os.sysconf("SC_PAGE_SIZE")
    first = addr // page * page
    n_pages = max(1, (addr + nbytes - first + page - 1) // page)
    k = max(1, min(samples, n_pages))
    ptrs = (ctypes.c_void_p * k)(*[first + (i * n_pages // k) * page for i in range(k)])
    status = (ctypes.c_int * k)()
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        rc = libc.syscall(ctypes.c_long(nr), ctypes.c_int(0), ctypes.c_ulong(k), ptrs, None,
                          status, ctypes.c_int(0))
    except Exception:  # noqa: BLE001
        return None
    if rc != 0:
        return None
    counts: Dict[int, int] = {}
    for s in status:
        if s >= 0:
            counts[s] = counts.get(s, 0) + 1
    if not counts:
        return None
    return max(counts, key=counts.get)


class threads_with_mask:
    """Context manager: threads created inside it inherit ``mask`` (None: no
    change); the calling thread's own mask is restored on exit."""

    def __init__(self, mask: Optional[Set[int]]) -> None:
        self.mask = mask
        self.prev: Optional[Set[int]] = None

    def __enter__(self) -> "threads_with_mask":
        if self.mask:
            try:
                self.prev = os.sched_getaffinity(0)
                os.sched_setaffinity(0, self.mask)
            except OSError:
                self.prev = None
        return self

    def __exit__(self, *exc) -> None:
        if self.prev is not None:
            try:
                os.sched_setaffinity(0, self.prev)
            except OSError:
                pass


def drain_thread_mask(device: int, avoid: str, numa_local: bool) -> Optional[Set[int]]:
    """Mask for an async drain's native threads: off the noted caller's core
    / L3 (``avoid``, see ``mask_avoiding_caller``), and within ``device``'s
    NUMA node when ``numa_local`` and at least 2 CPUs remain; None = leave
    the threads' mask as the caller's."""
    mask = mask_avoiding_caller(avoid) if avoid else None
    if numa_local:
        node = gpu_node_mask(device)
        if node is not None:
            both = (mask if mask is not None else os.sched_getaffinity(0)) & node
            if len(both) >= 2:
                mask = both
    return mask
