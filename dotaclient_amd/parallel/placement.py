"""Host placement of a node's ranks: which CPUs a rank's learner threads and its actor process run on, and how many
actor / decode threads fit in that share.

The reference sizes and isolates CPU per pod (ks-app/components/agent.jsonnet:45-49 — agent 700m + dotaservice 800m;
ks-app/components/optimizer.jsonnet:143-148 — optimizer 600m / 4 GiB) and lets the scheduler place pods. Here one
node runs ``LOCAL_WORLD_SIZE`` learner ranks (one per GPU) plus one actor process per rank, so the placement is
explicit:

* **budget** — the CPUs this process may use: ``os.sched_getaffinity(0)``, capped by the cgroup CPU quota
  (``/sys/fs/cgroup/cpu.max``; a container's share can be far below the machine's CPU count);
* **GPU-local CPUs** — the NUMA node of the rank's GPU (``/sys/bus/pci/devices/<bdf>/numa_node`` and the node's
  ``cpulist``), the rank's GPU found by its PCI bus id;
* **share** — the GPU-local CPUs are split evenly between the ranks whose GPUs sit on that NUMA node (in local-rank
  order), intersected with the budget; without topology information the budget is split evenly over the node's
  ranks. The actor process spawned by a rank inherits the mask set here.

``plan(local_rank, local_world)`` is pure (reads sysfs, no side effects) so the CPU tests pin its arithmetic; ``apply``
sets the calling thread's affinity — call it from the main thread before any worker thread or process starts.
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Sequence


@dataclass
class Placement:
    local_rank: int
    local_world: int
    cpus: List[int]                      # the rank's CPU share (sorted)
    numa_node: int = -1                  # the rank's GPU's NUMA node (-1: unknown)
    source: str = 'even-split'           # 'numa' | 'even-split' | 'affinity'
    budget: int = 0                      # CPUs available to the whole node's ranks (affinity ∩ cgroup quota)
    share: int = 0                       # CPUs of the budget that are this rank's (thread sizing)
    extra: Dict[str, object] = field(default_factory=dict)

    def threads(self, reserve: int, minimum: int = 1) -> int:
        """Worker threads that fit the share after ``reserve`` CPUs for the learner's main / stager / decode threads."""
        return max(minimum, min(len(self.cpus), self.share or len(self.cpus)) - reserve)

    def actor_threads(self, cap: int = 14, floor: int = 1) -> int:
        """Host threads of the rank's actor runtime: the share minus the learner's main / stager / decode threads
        (2 CPUs kept from a share of ≥ 6, 1 from a share of 2-5), at least ``floor``, at most ``cap`` (beyond 14 the
        one-GPU node loop stopped gaining, profiles/r4_e2e_threads_ab.jsonl). 8 ranks on a 16-CPU quota get 1 thread
        each, not the 2 that the old fixed floor gave (which oversubscribed the quota 1.5×)."""
        share = min(len(self.cpus), self.share or len(self.cpus))
        reserve = 2 if share >= 6 else 1 if share >= 2 else 0
        return max(floor, min(cap, share - reserve))

    def describe(self) -> Dict[str, object]:
        d = asdict(self)
        d['cpus'] = cpulist_str(self.cpus)
        d['n_cpus'] = len(self.cpus)
        return d


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' → [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out: List[int] = []
    for part in s.strip().split(','):
        part = part.strip()
        if not part:
            continue
        if '-' in part:
            a, b = part.split('-', 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def cpulist_str(cpus: Sequence[int]) -> str:
    cpus = sorted(set(cpus))
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(str(cpus[i]) if i == j else f'{cpus[i]}-{cpus[j]}')
        i = j + 1
    return ','.join(runs)


def cgroup_cpu_quota(root: str = '/sys/fs/cgroup') -> Optional[int]:
    """CPUs granted by the cgroup v2 ``cpu.max`` quota (rounded down, ≥ 1), None when unlimited / unreadable."""
    try:
        with open(os.path.join(root, 'cpu.max')) as f:
            quota, period = f.read().split()[:2]
        if quota == 'max':
            return None
        return max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        return None


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_numa_nodes(local_world: int, sysfs: str = '/sys') -> Optional[List[int]]:
    """NUMA node of each local GPU (device index order), from the PCI bus ids HIP reports; None if unknown."""
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        nodes = []
        for i in range(min(local_world, torch.cuda.device_count())):
            p = torch.cuda.get_device_properties(i)
            bus = getattr(p, 'pci_bus_id', None)
            dom = getattr(p, 'pci_domain_id', 0) or 0
            dev = getattr(p, 'pci_device_id', 0) or 0
            if bus is None:
                return None
            bdf = f'{dom:04x}:{bus:02x}:{dev:02x}.0'
            v = _read(os.path.join(sysfs, 'bus', 'pci', 'devices', bdf, 'numa_node'))
            nodes.append(int(v) if v is not None else -1)
        return nodes if len(nodes) == local_world else None
    except Exception:
        return None


def numa_cpus(node: int, sysfs: str = '/sys') -> Optional[List[int]]:
    v = _read(os.path.join(sysfs, 'devices', 'system', 'node', f'node{node}', 'cpulist'))
    return parse_cpulist(v) if v else None


def plan(local_rank: int, local_world: int, affinity: Optional[Sequence[int]] = None,
         quota: Optional[int] = None, gpu_nodes: Optional[Sequence[int]] = None,
         node_cpus: Optional[Dict[int, Sequence[int]]] = None) -> Placement:
    """The CPU share of ``local_rank`` among ``local_world`` ranks of this node. Arguments default to the live
    system (affinity mask, cgroup quota, the GPUs' NUMA nodes and the nodes' CPU lists); tests pass them in."""
    local_world = max(1, int(local_world))
    local_rank = int(local_rank) % local_world
    allowed = sorted(affinity if affinity is not None else os.sched_getaffinity(0))
    q = quota if quota is not None else cgroup_cpu_quota()
    budget = min(len(allowed), q) if q else len(allowed)
    if gpu_nodes is None:
        gpu_nodes = gpu_numa_nodes(local_world)
    share = max(1, budget // local_world)
    if gpu_nodes is not None and len(gpu_nodes) == local_world and all(n >= 0 for n in gpu_nodes):
        node = gpu_nodes[local_rank]
        local = (node_cpus or {}).get(node) if node_cpus is not None else numa_cpus(node)
        if local:
            aset = set(allowed)
            local = [c for c in local if c in aset]
            peers = [r for r in range(local_world) if gpu_nodes[r] == node]
            k, idx = len(peers), peers.index(local_rank)
            if len(local) >= k:
                per = len(local) // k                # the node's CPUs split between the ranks whose GPUs sit on it
                return Placement(local_rank, local_world, local[idx * per:(idx + 1) * per], node, 'numa', budget,
                                 min(share, per))
    if len(allowed) >= local_world:
        span = len(allowed) // local_world
        return Placement(local_rank, local_world, allowed[local_rank * span:(local_rank + 1) * span], -1,
                         'even-split', budget, min(share, span))
    return Placement(local_rank, local_world, allowed, -1, 'affinity', budget, share)


def apply(p: Placement) -> bool:
    """Pin the calling thread (and every thread / process it starts afterwards) to the rank's share."""
    if os.environ.get('DCA_NO_PIN') == '1' or not p.cpus:
        return False
    try:
        os.sched_setaffinity(0, p.cpus)
        return True
    except (OSError, AttributeError):
        return False


def for_this_rank(pin: bool = True) -> Placement:
    """Plan (and optionally apply) the placement of the calling rank from LOCAL_RANK / LOCAL_WORLD_SIZE."""
    lr = int(os.environ.get('LOCAL_RANK', '0'))
    lw = int(os.environ.get('LOCAL_WORLD_SIZE', os.environ.get('WORLD_SIZE', '1')))
    p = plan(lr, lw)
    p.extra['pinned'] = apply(p) if pin else False
    return p
