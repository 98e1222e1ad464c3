"""NUMA-local CPU binding for one-process-per-GPU jobs.

On an 8-GPU MI355X node every rank streams ~190 B per raw tweet from pinned
host memory over its own PCIe link (~56 GB/s each, ~450 GB/s for the node):
host DRAM and the socket interconnect sit on that path.  Binding a rank's
threads to the CPUs of its GPU's NUMA node before it allocates its pinned
staging buffers keeps those buffers on the local node (Linux first-touch
policy), so no rank's H2D crosses sockets.  Spark has no equivalent (the
reference's ingest is 2 tweets/s); this exists for the DP=8
configuration of BASELINE.json.

``TWTML_NUMA_BIND=0`` disables it.  Every step is best effort: no sysfs
entry, a single-node machine or a cpuset that excludes the node leaves the
affinity unchanged.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Set

__all__ = ["parse_cpulist", "gpu_numa_node", "bind_local_numa", "share_host_threads", "cgroup_cpu_limit"]

SYSFS = "/sys"
CGROUP = "/sys/fs/cgroup"


def parse_cpulist(text: str) -> Set[int]:
    """Kernel cpulist format: ``0-3,8,10-11``."""
    out: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def cgroup_cpu_limit(root: str = CGROUP) -> int:
    """CPUs the cgroup's CFS quota allows (v2 ``cpu.max``, else v1
    ``cpu.cfs_quota_us`` / ``cpu.cfs_period_us``), rounded up; 0 = no limit.
    Mirrors ``csrc/common/host_threads.h``: a container may see 256 CPUs in
    its affinity mask and be allowed 16, and threads past the quota get the
    whole cgroup throttled for the rest of a 100 ms period."""
    quota = period = 0
    txt = _read(os.path.join(root, "cpu.max"))
    if txt is not None:
        parts = txt.split()
        if len(parts) == 2 and parts[0] != "max":
            quota, period = int(parts[0]), int(parts[1])
    else:
        q = _read(os.path.join(root, "cpu", "cpu.cfs_quota_us"))
        p = _read(os.path.join(root, "cpu", "cpu.cfs_period_us"))
        if q is not None and p is not None:
            quota, period = int(q.strip()), int(p.strip())
    if quota <= 0 or period <= 0:
        return 0
    return max(1, -(-quota // period))


def gpu_numa_node(pci_bus_id: str, sysfs: str = SYSFS) -> Optional[int]:
    """NUMA node of a PCI device (``0000:05:00.0``), None if unknown."""
    txt = _read(os.path.join(sysfs, "bus", "pci", "devices", pci_bus_id.lower(), "numa_node"))
    if txt is None:
        return None
    try:
        node = int(txt.strip())
    except ValueError:
        return None
    return node if node >= 0 else None


def bind_local_numa(device: int, pci_bus_id: Optional[Callable[[int], str]] = None,
                    sysfs: str = SYSFS,
                    setaffinity: Callable[[int, Set[int]], None] = os.sched_setaffinity,
                    getaffinity: Callable[[int], Set[int]] = os.sched_getaffinity) -> Optional[Set[int]]:
    """Restrict the calling thread (and threads it starts later) to the CPUs
    of ``device``'s NUMA node.  Returns the CPU set, or None if unchanged."""
    if os.environ.get("TWTML_NUMA_BIND", "1") == "0":
        return None
    if pci_bus_id is None:
        from ..ops._native import hip
        pci_bus_id = hip().pci_bus_id
    try:
        bdf = pci_bus_id(int(device))
    except Exception:   # noqa: BLE001 -- no device / runtime: keep the affinity
        return None
    node = gpu_numa_node(bdf, sysfs)
    if node is None:
        return None
    txt = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    if txt is None:
        return None
    cpus = parse_cpulist(txt) & set(getaffinity(0))
    if not cpus or cpus == set(getaffinity(0)):
        return None
    setaffinity(0, cpus)
    return cpus


def share_host_threads(device: int, local_rank: int, local_world: int, n_devices: int,
                       pci_bus_id: Optional[Callable[[int], str]] = None, sysfs: str = SYSFS,
                       getaffinity: Callable[[int], Set[int]] = os.sched_getaffinity,
                       cgroup: str = CGROUP) -> int:
    """Host worker threads for this rank: the CPUs it may run on divided by
    the local ranks that share them, and at most its share of the cgroup CPU
    quota (all local ranks share one), exported as ``TWTML_HOST_THREADS`` for
    the native runtime (``csrc/common/host_threads.h``: the synthetic
    generator, the CPU featurizer, the wire packer and the staging pool).
    Local rank r drives device ``r % n_devices``; ranks whose devices sit on
    the same NUMA node as ours share its CPUs (all local ranks share them when
    the node is unknown).  An explicit ``TWTML_HOST_THREADS`` wins."""
    if os.environ.get("TWTML_HOST_THREADS"):
        return int(os.environ["TWTML_HOST_THREADS"])
    cpus = len(getaffinity(0))
    n_dev = max(1, int(n_devices))
    sharing = max(1, int(local_world))
    if pci_bus_id is None:
        try:
            from ..ops._native import hip
            pci_bus_id = hip().pci_bus_id
        except Exception:   # noqa: BLE001 -- no runtime: every local rank shares
            pci_bus_id = None
    if pci_bus_id is not None and local_world > 1:
        def node(d: int):
            try:
                return gpu_numa_node(pci_bus_id(d), sysfs)
            except Exception:   # noqa: BLE001
                return None
        mine = node(int(device))
        if mine is not None:
            nodes = [node(r % n_dev) for r in range(int(local_world))]
            if all(x is not None for x in nodes):
                sharing = max(1, sum(1 for x in nodes if x == mine))
    n = max(1, cpus // sharing)
    quota = cgroup_cpu_limit(cgroup)
    if quota > 0:
        n = max(1, min(n, quota // max(1, int(local_world))))
    os.environ["TWTML_HOST_THREADS"] = str(n)
    return n
