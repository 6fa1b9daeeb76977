"""Worker topology for one node: how many ingest workers to run and which
GPU / CPU set each one gets.

The reference scales by running more service replicas that compete for
the sharded queues (job-level data parallelism, prefetch 1,
one job per process).  On an MI355X node we run one worker per GPU by default
(each owns that GPU for batch piece verification through
``HIP_VISIBLE_DEVICES``), or one per ``cpus_per_worker`` CPUs on GPU-less
hosts.  ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` follow torchrun's contract
so a worker can also be launched by ``torch.distributed.run``.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field


@dataclass
class WorkerSpec:
    rank: int
    local_rank: int
    world_size: int
    gpu: int | None
    cpus: list[int] = field(default_factory=list)
    bt_listen_port: int = 0

    def env(self) -> dict[str, str]:
        e = {"RANK": str(self.rank), "LOCAL_RANK": str(self.local_rank), "WORLD_SIZE": str(self.world_size)}
        if self.bt_listen_port:         # else the worker default (42069, busy → ephemeral)
            e["TRITONDL_BT_LISTEN_PORT"] = str(self.bt_listen_port)
        if self.gpu is not None:
            e["HIP_VISIBLE_DEVICES"] = str(self.gpu)
        else:
            e["TRITONDL_GPU_VERIFY"] = "off"
        return e


def detect_gpus() -> int:
    """Number of visible HIP devices, without initialising a HIP runtime."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return len([x for x in vis.split(",") if x.strip() != ""])
    try:
        return len([d for d in os.listdir("/dev/dri") if d.startswith("renderD")]) if os.path.exists(
            "/sys/module/amdgpu") else 0
    except OSError:
        return 0


def plan(workers: int | None = None, *, gpus: int | None = None, cpus: int | None = None,
         cpus_per_worker: int = 2, base_port: int = 0, node_rank: int = 0, nnodes: int = 1,
         busy: list[float] | None = None) -> list[WorkerSpec]:
    """One :class:`WorkerSpec` per worker: its rank, GPU and CPU set.  With at
    least one L3 domain per worker, each worker gets a whole domain, spread
    evenly over the node like the GPUs; within its share of the spread it
    takes the idlest domain (``busy``: each domain's load, sampled for 0.2 s
    when not given)."""
    gpus = detect_gpus() if gpus is None else gpus
    doms: list[list[int]] = []
    if cpus is None:
        # ordered by last-level-cache domain, so each worker's slice (its receive
        # pump, hashers and send pump hand a job's bytes to each other) shares an L3
        doms = l3_domains()
        avail = [c for d in doms for c in d]
        cpus = len(avail)
    else:
        avail = list(range(cpus))
    if workers is None:
        workers = gpus if gpus > 0 else max(1, cpus // max(1, cpus_per_worker))
    world = workers * nnodes
    out = []
    per = max(1, cpus // workers)
    # one whole L3 domain (CCD + SMT siblings) per worker when there are enough:
    # a single worker measured faster on one CCD than on two (profiles/r03_pin_ab/)
    by_domain = len(doms) > 1 and len(doms) >= workers
    stride = max(1, len(doms) // max(1, workers))   # spread over both sockets, as the GPUs are
    if by_domain and stride > 1 and busy is None:
        busy = domain_busy(doms)
    for i in range(workers):
        gpu = (i % gpus) if gpus > 0 else None
        if by_domain:
            # the idlest domain of the worker's own stride window (a window stays on its
            # socket, so the spread over the GPUs' sockets holds)
            window = range(i * stride, min(len(doms), (i + 1) * stride))
            cset = doms[min(window, key=lambda j: (_load_step(busy[j]), j)) if busy else i * stride]
        else:
            cset = avail[i * per:(i + 1) * per] if cpus >= workers else []
        out.append(WorkerSpec(node_rank * workers + i, i, world, gpu, cset,
                              (base_port + i) if base_port else 0))
    return out


# ---------------------------------------------------------------- CPU sets

def parse_cpulist(s: str) -> list[int]:
    """Linux cpulist syntax (``0-7,128-135``, as in ``shared_cpu_list``)."""
    out: list[int] = []
    for part in s.replace(" ", "").split(","):
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            out.extend(range(int(lo), int(hi) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def l3_domains(allowed: list[int] | None = None, sysfs: str = "/sys/devices/system/cpu") -> list[list[int]]:
    """CPUs grouped by shared last-level cache (one group per Zen CCD),
    restricted to ``allowed`` (default: this process's affinity), ordered by
    their lowest CPU.  One group with every allowed CPU if sysfs has no
    cache topology."""
    if allowed is None:
        allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
            list(range(os.cpu_count() or 1))
    ok = set(allowed)
    groups: dict[tuple[int, ...], list[int]] = {}
    for c in allowed:
        try:
            with open(f"{sysfs}/cpu{c}/cache/index3/shared_cpu_list") as f:
                key = tuple(x for x in parse_cpulist(f.read().strip()) if x in ok)
        except (OSError, ValueError):
            return [sorted(ok)]
        groups.setdefault(key or (c,), []).append(c)
    return sorted((sorted(g) for g in groups.values()), key=lambda g: g[0])


def compact_cpuset(n: int, index: int = 0, allowed: list[int] | None = None) -> list[int]:
    """``n`` CPUs packed into as few last-level-cache domains as possible;
    ``index`` selects the index-th such set (one per rank), wrapping round.
    Keeps a process's threads — and the data they hand each other — on one
    CCD's L3 instead of spread over the socket."""
    doms = l3_domains(allowed)
    flat = [c for d in doms for c in d]
    if n <= 0 or n >= len(flat):
        return flat
    start = (index * n) % len(flat)
    return (flat + flat)[start:start + n]


def pin(spec: str, index: int = 0, count: int = 1) -> list[int]:
    """Pin the calling process (and every thread and child it starts later)
    to ``spec``: a cpulist; ``auto`` = the ``index``-th of ``count`` whole
    last-level-cache domains spaced evenly over the node (a lone worker:
    the idlest domain, :func:`idle_first`; one CCD with its
    SMT siblings per worker: on the box that beat 8 cores without siblings
    and two CCDs, ``profiles/r03_pin_ab/``);
    ``auto:N`` = the ``index``-th :func:`compact_cpuset` of N CPUs.  Returns
    the CPUs, or [] when ``spec`` is empty/"none" or pinning is unavailable."""
    spec = spec.strip()
    if not spec or spec == "none" or not hasattr(os, "sched_setaffinity"):
        return []
    if spec.startswith("auto"):
        if ":" in spec:
            cpus = compact_cpuset(int(spec.split(":", 1)[1]), index)
        else:
            doms = l3_domains()
            if max(1, count) == 1 and index == 0 and len(doms) > 1:
                # a lone worker: the idlest domain (sampled for 0.2 s), not always the
                # first one, which a shared node's other tenants may keep busy
                cpus = idle_first(doms, domain_busy(doms))[0]
            else:
                # ``count`` workers on this node (LOCAL_WORLD_SIZE) spread over all the
                # domains, so half of 8 GPU workers land on each socket with their GPUs
                stride = max(1, len(doms) // max(1, count, index + 1))
                cpus = doms[(index * stride) % len(doms)]
    else:
        cpus = parse_cpulist(spec)
    os.sched_setaffinity(0, cpus)
    return cpus


def pin_from_env(var: str = "TRITONDL_BENCH_FAKE_CPUS") -> list[int]:
    """Bench fakes (broker, origin, S3, producer) call this first thing: the
    bench puts them on their own L3 domain, standing in for remote endpoints."""
    spec = os.environ.get(var, "")
    if not spec or not hasattr(os, "sched_setaffinity"):
        return []
    try:
        cpus = parse_cpulist(spec)
        os.sched_setaffinity(0, cpus)
    except (OSError, ValueError):      # placement is an optimisation: run where we are
        return []
    return cpus


def gpu_numa_node(device: int = 0) -> int | None:
    """NUMA node of a visible HIP device (its PCI function's ``numa_node``),
    or None if unknown.  Initialises the HIP runtime (torch)."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if bus is None or dev is None:
            return None
        with open(f"/sys/bus/pci/devices/{int(dom or 0):04x}:{int(bus):02x}:{int(dev):02x}.0/numa_node") as f:
            n = int(f.read().strip())
        return n if n >= 0 else None
    except Exception:  # noqa: BLE001 - diagnostics only
        return None


def _cpu_ticks() -> dict[int, tuple[int, int]]:
    """Per-CPU (busy, total) jiffies from /proc/stat."""
    out: dict[int, tuple[int, int]] = {}
    with open("/proc/stat") as f:
        for line in f:
            if not line.startswith("cpu") or line.startswith("cpu "):
                continue
            parts = line.split()
            v = [int(x) for x in parts[1:]]
            idle = v[3] + (v[4] if len(v) > 4 else 0)          # idle + iowait
            tot = sum(v[:8])                                      # guest time is inside user
            out[int(parts[0][3:])] = (tot - idle, tot)
    return out


def domain_busy(doms: list[list[int]], interval: float = 0.2) -> list[float]:
    """Fraction of each domain's CPU time spent busy over ``interval``
    seconds (other tenants of a shared host included).  Zeros if /proc/stat
    is unreadable."""
    import time
    try:
        a = _cpu_ticks()
        time.sleep(interval)
        b = _cpu_ticks()
    except (OSError, ValueError, IndexError):
        return [0.0] * len(doms)
    out = []
    for d in doms:
        busy = sum(b[c][0] - a[c][0] for c in d if c in a and c in b)
        tot = sum(b[c][1] - a[c][1] for c in d if c in a and c in b)
        out.append(busy / tot if tot > 0 else 0.0)
    return out


# Load step for ordering L3 domains.  10 % steps ranked a domain another
# tenant touches now and then (2-10 % busy over the sample) with the idle
# ones, and L3 order then often picked it.  Over 31 driver-form runs on
# shared MI355X hosts, the 13 placed on a domain <= 1 % busy ran 362-409
# jobs/s; the 18 on busier ones ran 238-411, and all five runs under 310
# were among them (profiles/r06_final4/SUMMARY.md).
IDLE_STEP = 0.02


def _load_step(b: float) -> int:
    return round(b / IDLE_STEP)


def idle_first(doms: list[list[int]], busy: list[float]) -> list[list[int]]:
    """Domains ordered by load in :data:`IDLE_STEP` steps, L3 order within
    a step: an idle host keeps the topology order (neighbours share a
    socket), a shared one sends our ranks past the CCDs another tenant
    keeps busy, even a little."""
    order = sorted(range(len(doms)), key=lambda i: (_load_step(busy[i]), i))
    return [doms[i] for i in order]


def numa_node_of(cpu: int, sysfs: str = "/sys/devices/system/cpu") -> int:
    """NUMA node of a CPU (its ``cpuN/nodeM`` link), else its socket
    (``physical_package_id``), else 0."""
    try:
        for name in os.listdir(f"{sysfs}/cpu{cpu}"):
            if name.startswith("node") and name[4:].isdigit():
                return int(name[4:])
    except OSError:
        pass
    try:
        with open(f"{sysfs}/cpu{cpu}/topology/physical_package_id") as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return 0


def pair_domains(doms: list[list[int]], k: int, n: int, node_of=None) -> list[tuple[list[list[int]], list[int]]] | None:
    """Give each of ``n`` ranks ``k`` L3 domains plus one for its fakes, all
    on ONE NUMA node where a node has room.  ``doms`` comes idle-first
    (:func:`shared_idle_order`); rank after rank takes the node whose
    ``k + 1`` most idle free domains rank best, its ``k`` most idle for
    itself and the next for the fakes.  Only when no node has ``k + 1`` free
    domains left does a group span nodes.

    Taking "the next domain in idle order" for the fakes, as before, put
    them on the other socket whenever the idle ranking crossed it: a 10 MiB
    job's loopback fetch then took 2.5-2.8 ms instead of 1.6-1.9 and the
    headline fell from 300-376 to 243-299 jobs/s (``profiles/r04_fresh4/``).
    Returns None when there are fewer than ``n * (k + 1)`` domains."""
    if n <= 0 or k <= 0 or len(doms) < n * (k + 1):
        return None
    node_of = node_of or (lambda d: numa_node_of(d[0]))
    nodes = [node_of(d) for d in doms]
    free = list(range(len(doms)))                  # positions in the idle order
    out: list[tuple[list[list[int]], list[int]]] = []
    for _ in range(n):
        by_node: dict[int, list[int]] = {}
        for i in free:
            by_node.setdefault(nodes[i], []).append(i)
        groups = [idx[:k + 1] for idx in by_node.values() if len(idx) >= k + 1]
        # the group whose worst member is the most idle; else the k+1 most idle anywhere
        g = min(groups, key=lambda x: (x[-1], x[0])) if groups else free[:k + 1]
        for i in g:
            free.remove(i)
        out.append(([doms[i] for i in g[:k]], doms[g[k]]))
    return out


def shared_idle_order(local_rank: int, local_world: int, tag: str, timeout: float = 10.0) -> tuple[list, list]:
    """(domains idle-first, their busy fractions), sampled ONCE per launch:
    local rank 0 samples and publishes the order in a small file named by
    ``tag`` (e.g. the launcher's pid and port); the other local ranks read it,
    so every rank places itself against the same ranking.  A rank that
    cannot read it in ``timeout`` samples for itself."""
    import json
    import tempfile
    import time
    doms = l3_domains()
    if len(doms) <= 1:
        return doms, [0.0] * len(doms)
    path = os.path.join(tempfile.gettempdir(), f"tritondl-place-{tag}.json")
    if local_rank == 0 or local_world <= 1:
        busy = domain_busy(doms)
        order = sorted(range(len(doms)), key=lambda i: (_load_step(busy[i]), i))
        if local_world > 1:
            tmp = f"{path}.{os.getpid()}"
            with open(tmp, "w") as f:
                json.dump({"t": time.time(), "doms": doms, "order": order, "busy": busy}, f)
            os.replace(tmp, path)
        return [doms[i] for i in order], [busy[i] for i in order]
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        try:
            with open(path) as f:
                d = json.load(f)
            if time.time() - d["t"] < 120 and d["doms"] == doms:
                return [doms[i] for i in d["order"]], [d["busy"][i] for i in d["order"]]
        except (OSError, ValueError, KeyError):
            pass
        time.sleep(0.05)
    busy = domain_busy(doms)
    return idle_first(doms, busy), sorted(busy, key=_load_step)
