"""Host-side facts for bench.py's CPU baseline leg: the CPUs and cores this
process may use (affinity, cgroup quota, NUMA node and L3 domain per
core), an explicit thread placement, and what can slow a pass -- cgroup
quota throttling, the host's CPU load, NUMA locality of the pages each
OpenMP thread sums, page migration -- with the cause named from them
("CPU baseline spread").  Reads /proc and /sys only;
no GPU, no oracle."""
import ctypes
import os

import numpy as np


def _read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def host_cpus():
    """CPUs this process may use: the affinity set, capped by a cgroup CPU
    quota (a GPU box slice); and the physical cores among them, one entry per
    core (its first CPU in the set) with its package, NUMA node and L3
    domain."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = _read("/sys/fs/cgroup/cpu.max").split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (AttributeError, ValueError):
        pass
    cores = {}
    for c in aff:
        base = f"/sys/devices/system/cpu/cpu{c}"
        key = (_read(f"{base}/topology/physical_package_id") or "?", _read(f"{base}/topology/core_id") or str(c))
        if key in cores:
            continue
        node = next((int(e[4:]) for e in (os.listdir(base) if os.path.isdir(base) else [])
                     if e.startswith("node") and e[4:].isdigit()), 0)
        cores[key] = {"cpu": c, "pkg": key[0], "node": node, "l3": _read(f"{base}/cache/index3/id") or key[0]}
    phys = sorted(cores.values(), key=lambda r: r["cpu"])
    threads = min(len(phys) or len(aff), quota) if quota else (len(phys) or len(aff))
    return {"threads": threads, "affinity_cpus": len(aff), "cgroup_quota_cpus": quota,
            "physical_cores_in_affinity": len(phys), "cores": phys}


def cpu_placement(cores, threads, policy):
    """The CPUs the baseline's OpenMP threads are pinned to, one per thread
    (an explicit OMP_PLACES list, so the placement is the same on every box
    with the same topology).  `l3spread`: round-robin over the L3 domains
    (CCDs) of every NUMA node -- one thread per CCD first, the placement
    that fed the host's memory fastest in round 2's sweep
    (profiles/r02_cpu_sweep.txt: spread over cores 400 GB/s, close 141);
    `node`: the same, restricted to the NUMA node holding the most cores."""
    if policy == "node":
        per = {}
        for r in cores:
            per.setdefault(r["node"], []).append(r)
        cores = max(per.values(), key=len) if per else cores
    doms = {}
    for r in cores:
        doms.setdefault((r["node"], r["l3"]), []).append(r["cpu"])
    order = [doms[k] for k in sorted(doms, key=lambda k: (str(k[1]).zfill(8), k[0]))]
    picked = []
    while len(picked) < threads and any(order):
        for d in order:
            if d and len(picked) < threads:
                picked.append(d.pop(0))
    return picked


def cpu_model():
    for line in (_read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return ""


def cgroup_cpu_stat():
    """The cgroup's CPU accounting (cgroup v2 cpu.stat): throttled periods
    and time, so a slow pass can be told apart from CFS quota throttling."""
    st = {}
    for line in (_read("/sys/fs/cgroup/cpu.stat") or "").splitlines():
        k, _, v = line.partition(" ")
        if v.isdigit():
            st[k] = int(v)
    return st


def host_cpu_busy():
    """(busy, total) jiffies of the whole host from /proc/stat's first line
    (every CPU, every tenant): the share of the host's CPUs busy between two
    reads, this process included."""
    f = (_read("/proc/stat") or "cpu 0 0 0 1").splitlines()[0].split()[1:]
    v = [int(x) for x in f[:8]]
    idle = v[3] + (v[4] if len(v) > 4 else 0)
    return sum(v) - idle, sum(v)


def vmstat(keys=("numa_pages_migrated", "pgmigrate_success", "numa_hint_faults", "thp_fault_alloc",
                 "thp_collapse_alloc")):
    st = {}
    for line in (_read("/proc/vmstat") or "").splitlines():
        k, _, v = line.partition(" ")
        if k in keys:
            st[k] = int(v)
    return st


def cpu_node(c):
    base = f"/sys/devices/system/cpu/cpu{c}"
    return next((int(e[4:]) for e in (os.listdir(base) if c >= 0 and os.path.isdir(base) else [])
                 if e.startswith("node") and e[4:].isdigit()), None)


def numa_locality(bufs, thread_cpus, per_block=32):
    """How many of the pages each OpenMP thread sums sit on its own NUMA
    node: reduce_kernel's `omp parallel for` (libgomp's static schedule)
    gives thread t one contiguous block of every buffer; 32 pages per block
    and buffer are located with move_pages(2) (query only).  Returns the
    local fraction and the page count per node, or None if the query fails."""
    libc = ctypes.CDLL(None, use_errno=True)
    T = len(thread_cpus)
    nodes = [cpu_node(c) for c in thread_cpus]
    addrs, want = [], []
    for b in bufs:
        count, base = b.size, b.ctypes.data
        q, r = divmod(count, T)
        for t in range(T):
            lo = q * t + min(t, r)
            hi = lo + q + (1 if t < r else 0)
            for j in range(per_block):
                i = lo + (hi - lo) * j // per_block
                addrs.append((base + b.itemsize * i) & ~4095)
                want.append(nodes[t])
    n = len(addrs)
    pages = (ctypes.c_void_p * n)(*addrs)
    status = (ctypes.c_int * n)()
    # move_pages(2) (x86_64 syscall 279) with nodes == NULL: a query, nothing moves
    rc = libc.syscall(ctypes.c_long(279), ctypes.c_int(0), ctypes.c_ulong(n), pages, None, status, ctypes.c_int(0))
    if rc != 0:
        return None
    got = list(status)
    hist = {}
    for g in got:
        hist[str(g)] = hist.get(str(g), 0) + 1
    ok = sum(1 for g, w in zip(got, want) if g >= 0 and g == w)
    return {"local_frac": round(ok / n, 4), "pages_sampled": n, "pages_per_node": hist}


def spread_cause(times, thr, busy, local0, local1, vm, threads):
    """Why the passes of the CPU leg spread by more than 1.3x, from what the
    leg recorded: the share of the slow passes' excess time the cgroup's
    quota throttling covers; else, with the pages local before and after,
    no page migrated and the host's CPUs mostly idle, the cause is memory
    bandwidth taken outside this container (other tenants' CPU jobs or
    host-memory DMA of other GPUs), which no counter here sees -- the slow
    passes then come in runs (regimes), not singly."""
    fast = min(times)
    excess = [t - fast for t in times if t > 1.15 * fast]
    if thr is not None:
        covered = sum(min(m * 1e-3, t - fast) for t, m in zip(times, thr) if t > 1.15 * fast)
        if excess and covered >= 0.5 * sum(excess):
            return {"cause": "cgroup CPU quota throttling", "throttle_covers_frac": round(covered / sum(excess), 3)}
    else:
        covered = 0.0
    slow = [t > 1.15 * fast for t in times]
    runs = sum(1 for i, x in enumerate(slow) if x and (i == 0 or not slow[i - 1]))
    own = threads / (os.cpu_count() or threads)
    local = all(loc and loc["local_frac"] == 1.0 for loc in (local0, local1))
    moved = vm.get("numa_pages_migrated", 0) + vm.get("pgmigrate_success", 0)
    others = round(float(np.median(busy)) - own, 3) if busy else None
    out = {"slow_passes": sum(slow), "slow_runs": runs, "throttle_covers_frac":
           round(covered / sum(excess), 3) if excess else None, "pages_local": local, "pages_migrated": moved,
           "host_busy_others_median": others}
    if local and not moved and others is not None and others < 0.5:
        out["cause"] = ("host memory bandwidth taken outside this container (other tenants' CPU jobs or other "
                        "GPUs' host-memory DMA): not throttling, every page local, none migrated, the host's "
                        "CPUs mostly idle")
    else:
        out["cause"] = "unnamed: see the fields"
    return out


def places_desc():
    pl = os.environ.get("OMP_PLACES", "")
    return f"{len(pl.split(','))} explicit places" if pl.startswith("{") else f"OMP_PLACES={pl}"
