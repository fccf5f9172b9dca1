#!/usr/bin/env python3
"""bench.py -- HiCCL bucket-reduction stage on MI355X (driver contract).

Default workload = BASELINE config 2: N = 8 inputs x 2^28 fp32 (1 GiB each)
-> one 1 GiB output, device-resident.  One "step" = one hiccl_reduce launch
over the whole bucket.  value = whole-job GB/s = world_size x (N+1) x count x
4 B x steps / max-over-ranks wall time (the reference's own byte accounting,
source/compute.h:197-203).  Multi-GPU: every rank reduces its own bucket
(replicas, weak scaling -- the stage is per-GPU local).

Extra objects on the JSON line:
  roofline      achieved = algorithmic bytes per launch / mean kernel time from
                HIP events on the launch stream; peak = 8000 GB/s (MI355X HBM3E
                spec); traffic = PMC HBM bytes per launch from the committed
                profiles/ PMC summary when one matches this workload AND
                kernel, else null; plus measured ceilings on the same
                buckets: 8R+1W XOR probe, 8-stream read-only probe (tile
                order), plain copy.
  cpu_baseline  the reference's own CPU reduce_kernel (compute.h:14-23, built
                from /root/reference into oracle/_ref by oracle/build_ref.sh;
                kind "reference") or the C restatement (kind "port"), timed on
                this host, rank 0 at N=1 only.

Other modes (not the driver's line; tools/bench_modes.py): --nway (config 3),
--chunks (config 4), --c3vsc2, --roundtrip (host memory H2D + kernel + D2H
rate for DESIGN.md), --progstep (one C5 step); --c5 RANKS (the config-5 leg
alone, a rehearsal when ranks share GPUs).  Closed tuning probes:
tools/archive/bench_probes.py.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hiccl_amd  # noqa: E402
from hiccl_amd import _lib as L  # noqa: E402

METRIC = "GB/s device-resident N-way float bucket sum, 1 GB/input; % HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED = 1234


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------- dist ----

class Dist:
    """One process per GPU (torchrun env).  The control plane -- the barrier
    around the timed region and the max-over-ranks time -- is gloo on the
    host: it is started before any GPU is touched (the config-5 leg runs an
    MPI job on every GPU first) and there is no data-path collective (the
    stage is per-GPU local)."""

    def __init__(self, gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != gpus:
            if self.world == 1:
                log(f"bench: --gpus {gpus} without a launcher; running 1 rank")
                self.world = 1
            else:
                log(f"bench: WORLD_SIZE={self.world} but --gpus {gpus}")
        self.pg = init_control_plane() if self.world > 1 else None
        self.backend = "gloo" if self.pg else None
        ndev = torch.cuda.device_count()
        self.device = self.local % max(ndev, 1)
        if ndev:  # (no device: only the control plane, as in tests/test_bench_dist.py)
            torch.cuda.set_device(self.device)

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def max(self, x):
        if not self.pg:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.pg:
            self.pg.destroy_process_group()


def init_control_plane():
    """The gloo process group over the torchrun ranks (CPU only)."""
    import torch.distributed as tdist
    if not tdist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo announces its connections on stdout; the driver reads rank 0's
        # stdout for the one JSON line, so route them to stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            tdist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return tdist


# ------------------------------------------------------------ config 5 -----

C5_EXE = os.path.join(ROOT, "build", "collectives_hip_f32")
C5_MPIRUN = None  # None: mpirun from PATH (tests put a stub launcher here)


def c5_leg(args):
    """Config 5 in situ (collectives/main.cpp:151-155): the all-reduce
    composition (reduce-scatter + fence + all-gather) over every GPU of the
    job, hierarchy {1, N/2, 2} = {1,4,2} at N = 8 with {MPI, IPC, IPC},
    pipedepth 128, 2^25 floats per rank per chunk (a 1 GiB send buffer per
    rank at 8 ranks), this build's C++ Comm<float> with the HIP reduction
    stage -- run by rank 0 as an MPI job (one rank per GPU) BEFORE any torch
    rank touches a GPU; the other ranks wait on the gloo control plane.
    Returns the job's JSON (per mode) or why it was skipped; never the bench
    `value`."""
    tdist = init_control_plane()
    res = None
    if tdist.get_rank() == 0:
        try:
            res = run_c5(tdist.get_world_size(), args)
        except Exception as e:  # the leg must not cost the headline line
            res = {"skipped": f"error: {e}"}
    obj = [res]
    tdist.broadcast_object_list(obj, src=0)
    return obj[0]


def run_c5(world, args, allow_shared=False, only=None, force_stream=False):
    """`allow_shared`: run even with fewer GPUs than ranks (a rehearsal on a
    1-GPU box, tests/test_c5_leg_gpu.py; the library then runs host-driven).
    `force_stream` (rehearsals only): HICCL_STREAM_ORDERED=force in the
    stream-ordered modes, so with ranks sharing a GPU they still run the
    protocol an 8-GPU run takes (fenced tokens, graph, fused) instead of
    falling back to host-driven.  `only`: run just these mode keys."""
    import shutil
    import tempfile
    # the MPI ranks pick their GPU by local rank (CommBench::init); a per-rank
    # device mask inherited from this torchrun rank would show them one GPU
    # each and put every rank on it -- drop the masks from the job's
    # environment and say which were dropped
    base_env, scrubbed = c5_child_env(os.environ)
    ndev = visible_gpus(base_env)
    if ndev < world and not allow_shared:
        return {"skipped": f"{world} ranks on {ndev} GPU(s): config 5 needs one GPU per rank",
                "env_scrubbed": scrubbed, "devices_counted_unmasked": ndev}
    if force_stream and not allow_shared:
        return {"skipped": "force_stream is for rehearsals (allow_shared) only"}
    if not os.path.exists(C5_EXE):
        return {"skipped": f"{C5_EXE} not built"}
    mpirun = C5_MPIRUN or shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    hier = f"1,{world // 2},2" if world % 2 == 0 and world >= 4 else str(world)
    libs = "mpi,ipc,ipc" if hier.count(",") == 2 else "ipc"
    count = 1 << args.c5_log2count
    out = {"workload": f"C5: all-reduce of {count * world * 4 >> 20} MiB fp32 per rank, {world} ranks, hierarchy "
                       f"{{{hier}}} {{{libs}}}, pipedepth 128 (collectives/main.cpp:151-155)",
           "env_scrubbed": scrubbed, "devices_counted_unmasked": ndev}
    # Stream-ordered modes.  The library's default protocol is fenced token
    # phases (release stores, acquire polls: hiccl_token_mode) and one launch
    # per element of a step (hiccl_step_program_default() off) -- what the GPU
    # suite verifies.  Step programs with fenced tokens (`_fenced`) and with
    # round 3's light tokens (`stream_graph_fused`) run as named A/B twins;
    # every mode carries its own KAT and mode_used, and the riskiest
    # (light tokens, never run across GPUs) goes last, since a mode killed at
    # its limit stops the leg.  Every knob is set explicitly so the A/B holds
    # whatever the defaults are.
    fenced = {"HICCL_STREAM_ORDERED": "1", "HICCL_GRAPH": "1", "HICCL_FUSED_GATHER": "1", "HICCL_STEP_PROGRAM": "0",
              "HICCL_PROG_FENCES": "full"}
    modes = [("host", {"HICCL_STREAM_ORDERED": "0"}, hier, libs),
             ("stream_graph", dict(fenced, HICCL_FUSED_GATHER="0"), hier, libs),
             ("stream_graph_fused_noprog", fenced, hier, libs),
             ("stream_graph_fused_fenced", dict(fenced, HICCL_STEP_PROGRAM="1"), hier, libs)]
    if hier != str(world):
        # not the reference's config: the same all-reduce on one flat IPC
        # level, every peer over its own xGMI link of the full mesh ({1,4,2}
        # gives its last level one link per rank; it was laid out for
        # Frontier's GCD pairs)
        out["flat_workload"] = f"same, hierarchy {{{world}}} {{ipc}}"
        modes.append(("flat_stream_graph_fused", fenced, str(world), "ipc"))
    # the reference's main.cu runs its levels on XCCL (main.cu:25): RCCL
    # point-to-point per level, opted into here (HICCL_XCCL=rccl; on shared
    # GPUs the library falls back to IPC, and mode_used says which ran)
    modes.append(("xccl", {"HICCL_STREAM_ORDERED": "0", "HICCL_XCCL": "rccl"}, hier, libs.replace("ipc", "xccl")))
    modes.append(("stream_graph_fused", dict(fenced, HICCL_STEP_PROGRAM="1", HICCL_PROG_FENCES="light"), hier, libs))
    deadline = time.perf_counter() + 300.0  # the whole leg: never more than ~5 min of the bench run
    if only is not None:
        modes = [m for m in modes if m[0] in only]
    if force_stream:
        modes = [(nm, dict(ex, HICCL_STREAM_ORDERED="force") if ex.get("HICCL_STREAM_ORDERED") == "1" else ex, h, lb)
                 for nm, ex, h, lb in modes]
        out["forced_stream_ordered"] = True
    for name, extra, hier, libs in modes:
        left = int(deadline - time.perf_counter())
        if left < 30:
            out[name] = {"skipped": "time budget of the config-5 leg spent"}
            continue
        fd, path = tempfile.mkstemp(prefix="hiccl_c5_", suffix=".json", dir="/tmp")
        os.close(fd)
        env = dict(base_env, HSA_ENABLE_IPC_MODE_LEGACY="0", HICCL_DRIVER_JSON=path, OMP_NUM_THREADS="1",
                   HICCL_SIGNAL_TIMEOUT="20", **extra)
        if ndev < world:
            # a rehearsal with ranks sharing GPUs: HIP's 4 hardware queues per
            # process oversubscribe a device at 8 ranks and the queues
            # time-slice (2.6 s instead of 24 ms per run at 8 ranks,
            # profiles/r02i_c5_rehearsal_1gpu.jsonl)
            env["GPU_MAX_HW_QUEUES"] = "2"
        cmd = ["timeout", "-k", "10", str(min(120, left)), mpirun, "-np", str(world), C5_EXE, "8", str(count), "1", "1", "128",
               "2", str(args.c5_iters), hier, libs]
        t0 = time.perf_counter()
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, cwd="/tmp")
        try:
            r = json.load(open(path))
        except (OSError, ValueError):
            r = {"error": f"rc {p.returncode}: {(p.stdout + p.stderr)[-600:]}"}
        finally:
            os.unlink(path)
        r["wall_s"] = round(time.perf_counter() - t0, 1)
        r["rc"] = p.returncode
        out[name] = r
        log(f"bench: c5 {name}: {r}")
        if p.returncode < 0 or p.returncode in (124, 137) or p.returncode >= 128:
            # killed at its limit, hung or crashed: start nothing more on the
            # GPUs (a mode that failed its check or its own signal time-out
            # exits 1 and leaves the GPUs usable: the next mode still runs)
            out["stopped_after"] = name
            break
    out["protocol_ab"] = c5_protocol_ab(out)
    return out


def c5_protocol_ab(out):
    """The config-5 leg's protocol A/B: each stream-ordered + graph + fused
    variant's median collective time against the default protocol's (fenced
    tokens, one launch per element), with whether its KAT passed -- the data
    the stream-ordered default is to be decided on across GPUs."""
    base = out.get("stream_graph_fused_noprog", {})
    ab = {"baseline": "stream_graph_fused_noprog (fenced tokens, per-element launches: the default)",
          "baseline_ms": base.get("collective_ms_median"), "baseline_kat": base.get("kat")}
    for name in ("stream_graph_fused_fenced", "stream_graph_fused"):
        r = out.get(name, {})
        t = r.get("collective_ms_median")
        ab[name] = {"ms": t, "kat": r.get("kat"), "mode_used": r.get("mode_used"),
                    "over_baseline": round(t / ab["baseline_ms"], 4) if t and ab["baseline_ms"] else None}
    return ab


DEVICE_MASKS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def c5_child_env(env):
    """The config-5 MPI job's environment: `env` without per-process GPU
    masks.  Returns (env, {mask: dropped value})."""
    child = dict(env)
    dropped = {k: child.pop(k) for k in DEVICE_MASKS if k in child}
    return child, dropped


def visible_gpus(env):
    """GPUs a process started with `env` sees (hipGetDeviceCount in a child,
    so this process's HIP state and device mask do not matter); 0 if none."""
    code = ("import ctypes\n"
            "try:\n h = ctypes.CDLL('libamdhip64.so')\nexcept OSError:\n h = ctypes.CDLL('/opt/rocm/lib/libamdhip64.so')\n"
            "n = ctypes.c_int(0)\nprint(n.value if h.hipGetDeviceCount(ctypes.byref(n)) == 0 else 0)\n")
    try:
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        return int(p.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def whole_job_gbps(world, bytes_per_step, steps, wall_max_s):
    """Every rank reduces its own bucket (replicas): the job moves world x
    bytes_per_step per step, and the job's time is the slowest rank's."""
    return world * bytes_per_step * steps / wall_max_s / 1e9


# ----------------------------------------------------------- workloads -----

def make_bucket(n, count, dtype=torch.float32, seed=SEED, layout="bucket"):
    """n inputs (generator-filled) and an output.  layout "bucket": the
    library's layout, one allocation (hiccl_amd.bucket / hiccl_bucket_alloc);
    "separate": one torch allocation per buffer."""
    # integer buckets (size_t: the reference drivers' T) get the float
    # generator's bits
    fill_as = {torch.int64: torch.float64, torch.int32: torch.float32}.get(dtype, dtype)
    if layout == "bucket":
        ins, out = hiccl_amd.bucket(n, count, fill_as)
    else:
        ins = [torch.empty(count, dtype=fill_as, device="cuda") for _ in range(n)]
        out = torch.empty(count, dtype=fill_as, device="cuda")
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    ins = [t.view(dtype) for t in ins]
    out = out.view(dtype)
    torch.cuda.synchronize()
    return ins, out


def time_launches(fn, steps, warmup, dist=None):
    """W untimed launches, then K timed: barrier + sync on both sides.
    Returns (wall seconds for K steps, list of per-launch kernel ms)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for a, b in evs:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    return t1 - t0, [a.elapsed_time(b) for a, b in evs]


def time_queued(fn, steps, warmup):
    """GPU time per launch with the stream kept busy: one event pair around
    `steps` back-to-back launches, so host submission gaps are not counted
    (small kernels: the per-launch event pairs of time_launches include the
    time the GPU waits for the host to submit)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def mix_ceiling(ins, out, count, reps=10, mode=0):
    """Achievable HBM rate for this very access mix (n streams read + 1
    written, 16 B/lane, XOR instead of add; mode 1: the n reads only) from
    tools/libhbm_probe.so, tile order, at grids 256 and 192; None if not
    built.  Rate = bytes the probe moves / time."""
    pso = os.path.join(ROOT, "tools", "libhbm_probe.so")
    if not os.path.exists(pso):
        return None
    probe = ctypes.CDLL(pso)
    probe.probe_run.restype = ctypes.c_int
    probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_uint64, ctypes.c_void_p]
    n = len(ins)
    if n > 64:  # the probe kernels take at most 64 streams
        return None
    tab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    best = 0.0
    for grid in (256, 192):
        fn = lambda: probe.probe_run(mode, 256, 4, 2, 2, 0, grid, tab, n, ctypes.c_void_p(out.data_ptr()),  # noqa: E731
                                     count * 4, st)
        _, ms = time_launches(fn, reps, 3)
        moved = (n + 1 if mode == 0 else n if mode == 1 else 1) * count * 4
        best = max(best, moved / (np.median(ms) * 1e-3) / 1e9)
    return best


def serial_rw_model(read_bytes, write_bytes, read_gbps, copy_gbps, kern_s, write_gbps_probe=None):
    """The box's own HBM bound for a read/write mix: a DRAM channel either
    reads or writes, so a kernel that reads R and writes W bytes needs at
    least R / read_rate + W / write_rate.  read_rate = the 8-stream read-only
    probe on the bench's buckets; write_rate from the copy probe (X read + X
    written in t: X / t_write = X / (t - X / read_rate))."""
    if not read_gbps or not copy_gbps or 2.0 / copy_gbps <= 1.0 / read_gbps:
        return None
    write_gbps = 1.0 / (2.0 / copy_gbps - 1.0 / read_gbps)
    t = read_bytes / read_gbps / 1e9 + write_bytes / write_gbps / 1e9
    m = {"read_GBps": round(read_gbps, 1), "write_GBps_from_copy": round(write_gbps, 1),
         "predicted_ms": round(t * 1e3, 4), "frac": round(t / kern_s, 4)}
    if write_gbps_probe:
        # the same model with the write-only probe's rate (nt stores, no
        # reads): the copy kernel's implied write rate is a pessimistic one
        t2 = read_bytes / read_gbps / 1e9 + write_bytes / write_gbps_probe / 1e9
        m.update({"write_GBps_probe": round(write_gbps_probe, 1), "predicted_ms_write_probe": round(t2 * 1e3, 4),
                  "frac_write_probe": round(t2 / kern_s, 4)})
    return m


def copy_ceiling(nbytes=1 << 30, reps=10):
    src = torch.empty(nbytes // 4, device="cuda")
    dst = torch.empty_like(src)
    hiccl_amd.fill_uniform(src, 1, 0)
    _, ms = time_launches(lambda: hiccl_amd.stream_copy(dst, src), reps, 3)
    del src, dst
    return 2 * nbytes / (np.mean(ms) * 1e-3) / 1e9


# --------------------------------------------------------- CPU baseline ----

sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_report import compact_c5, compact_line  # noqa: E402,F401
from host_cpu import (_read, cgroup_cpu_stat, cpu_model, cpu_placement, host_cpu_busy, host_cpus,  # noqa: E402
                      numa_locality, places_desc, spread_cause, vmstat)

CPU_POLICIES = ("l3spread", "node", "spread")


def cpu_baseline(n, count, budget_s=10.0, gpu_out=None, policy=None, threads=None):
    """The reference's CPU reduce_kernel on this host, in a child process so
    OpenMP starts pinned as chosen here (libgomp reads OMP_* once, at load;
    BASELINE.md:34): `threads` (default: the cgroup quota, at most one per
    physical core) on an explicit OMP_PLACES list from cpu_placement
    (`policy`, default HICCL_CPU_PLACEMENT or l3spread; `spread`: round 4's
    OMP_PROC_BIND=spread over OMP_PLACES=cores, no list).  `gpu_out`: the
    GPU's output of the same bucket (a host float32 array): the child
    compares all `count` words with the reference's own output (the
    full-bucket parity check)."""
    cpus = host_cpus()
    policy = policy or os.environ.get("HICCL_CPU_PLACEMENT", "l3spread")
    threads = threads or cpus["threads"]
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    placed = None
    if policy == "spread" or not cpus["cores"]:
        env.update(OMP_PROC_BIND="spread", OMP_PLACES="cores")
    else:
        placed = cpu_placement(cpus["cores"], threads, policy)
        env.update(OMP_PROC_BIND="close", OMP_PLACES=",".join("{%d}" % c for c in placed),
                   OMP_NUM_THREADS=str(len(placed)))
    path = None
    if gpu_out is not None:
        import tempfile
        fd, path = tempfile.mkstemp(prefix="hiccl_gpu_out_", suffix=".f32", dir="/tmp")
        with os.fdopen(fd, "wb") as fh:
            gpu_out.tofile(fh)
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-leg", "--n", str(n), "--log2count",
           str(int(np.log2(count))), "--cpu-budget", str(budget_s)]
    if path:
        cmd += ["--expect-file", path]
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=max(120.0, 6 * budget_s))
    finally:
        if path:
            os.unlink(path)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        log("bench: cpu leg failed:", p.returncode, p.stderr[-2000:])
        return None, None
    res = json.loads(lines[-1])
    parity = res.pop("parity_full", None)
    res["cores"] = res.pop("threads")
    by = {r["cpu"]: r for r in cpus["cores"]}
    res["placement"] = {"policy": policy, "cpus": placed,
                        "numa_nodes": sorted({by[c]["node"] for c in placed}) if placed else None,
                        "l3_domains": len({(by[c]["node"], by[c]["l3"]) for c in placed}) if placed else None,
                        "numa_nodes_in_affinity": len({r["node"] for r in cpus["cores"]}),
                        "l3_domains_in_affinity": len({(r["node"], r["l3"]) for r in cpus["cores"]})}
    res.update({k: v for k, v in cpus.items() if k not in ("threads", "cores")})
    return res, parity


def cpu_leg(args):
    """Child of cpu_baseline(): time the reference reduce_kernel (or the C
    restatement) over the full bucket; optionally compare with a GPU output.
    Per pass: its time and the cgroup's throttling during it."""
    n, count = args.n, 1 << args.log2count
    ref_so = os.path.join(ROOT, "oracle", "_ref", "libhiccl_ref.so")
    ora = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    ora.oracle_num_threads.restype = ctypes.c_int
    if os.path.exists(ref_so):
        lib, kind = ctypes.CDLL(ref_so), "reference"
        fn = lib.ref_reduce_f32
        fn.restype = None
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    else:
        kind = "port"
        fn = ora.oracle_reduce_f32
        fn.restype = None
        fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    threads = ora.oracle_num_threads()
    fill = ora.oracle_fill_uniform_f32
    fill.restype = None
    fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t]
    bufs = [np.empty(count, np.float32) for _ in range(n)]
    # parallel first touch inside the generator: the same static partition
    # over the same pinned threads as reduce_kernel's loop, so every page is
    # on the NUMA node of the thread that sums it
    for k, b in enumerate(bufs):
        fill(b.ctypes.data, count, SEED, k, 0)
    out = np.empty(count, np.float32)
    fill(out.ctypes.data, count, SEED, 99, 0)  # first touch of the output
    tab = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
    tc = (ctypes.c_int * 512)()
    team = ora.oracle_thread_cpus(tc, 512)
    thread_cpus = list(tc)[:team]
    local0 = numa_locality(bufs + [out], thread_cpus)

    def one():
        t = time.perf_counter()
        if kind == "reference":
            fn(out.ctypes.data, count, tab, n)
        else:
            fn(out.ctypes.data, tab, n, count)
        return time.perf_counter() - t

    one()  # warm
    times, thr, busy = [], [], []
    st0 = st = cgroup_cpu_stat()
    vm0, hb0 = vmstat(), host_cpu_busy()
    hb = hb0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < args.cpu_budget and len(times) < 50:
        times.append(one())
        st1, hb1 = cgroup_cpu_stat(), host_cpu_busy()
        thr.append(round((st1.get("throttled_usec", 0) - st.get("throttled_usec", 0)) * 1e-3, 2))
        busy.append(round((hb1[0] - hb[0]) / max(1, hb1[1] - hb[1]), 3))
        st, hb = st1, hb1
    vm1 = vmstat()
    local1 = numa_locality(bufs + [out], thread_cpus)
    med = float(np.median(times))
    rate = lambda t: round((n + 1) * count * 4 / t / 1e9, 2)  # noqa: E731
    # the spread over the passes, as the reference prints min / median / max
    # for its own timings (compute.h:165-195), and the cgroup's throttling
    # over the timed passes (per pass in throttled_ms)
    throttle = {k: st.get(k, 0) - st0.get(k, 0) for k in ("nr_periods", "nr_throttled", "throttled_usec")} \
        if st0 else None
    slow = max(times) / min(times)
    res = {"value": rate(med), "unit": "GB/s", "threads": threads, "kind": kind,
           "min": rate(max(times)), "max": rate(min(times)), "max_over_min": round(slow, 3), "passes": len(times),
           "pass_ms": [round(t * 1e3, 2) for t in times], "throttle": throttle,
           "throttled_ms": thr if st0 else None,
           # the whole host's CPU busy share per pass (/proc/stat: every
           # tenant; this leg's own threads are threads / host CPUs of it)
           "host_busy_frac": busy, "host_cpus": os.cpu_count(),
           "thread_cpus": thread_cpus, "numa_locality_before": local0, "numa_locality_after": local1,
           "vmstat_delta": {k: vm1.get(k, 0) - vm0.get(k, 0) for k in vm1},
           "numa_balancing": _read("/proc/sys/kernel/numa_balancing"),
           "thp": _read("/sys/kernel/mm/transparent_hugepage/enabled"),
           "cpuset_mems": _read("/sys/fs/cgroup/cpuset.mems.effective"),
           "sample": f"{n} x 2^{args.log2count} fp32 -> 1 output (the full config-2 bucket), median of "
                     f"{len(times)} passes ({med * 1e3:.1f} ms each), OpenMP {threads} threads "
                     f"(OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND', '')}, "
                     f"{places_desc()}), {cpu_model()}"}
    if slow > 1.3:
        res["spread_cause"] = spread_cause(times, thr if st0 else None, busy, local0, local1,
                                           {k: vm1.get(k, 0) - vm0.get(k, 0) for k in vm1}, threads)
    if args.expect_file:
        got = np.fromfile(args.expect_file, dtype=np.float32)
        ok = got.size == count
        bad = int(np.count_nonzero(got.view(np.uint32) != out.view(np.uint32))) if ok else count
        res["parity_full"] = {"ok": ok and bad == 0, "mismatches": bad, "words": count,
                              "against": f"{kind} reduce_kernel (compute.h:14-23) on the same generator and seed"}
    print(json.dumps(res), flush=True)
    return 0


def sample_check(out, n, count, bf16=False, seed=SEED, nsample=1024):
    """Bitwise check of `out` at random indices against the oracle generator."""
    ora_so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(ora_so):
        return None
    ora = ctypes.CDLL(ora_so)
    fn = ora.oracle_sample_sum_bf16 if bf16 else ora.oracle_sample_sum_f32
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int]
    idx = np.random.default_rng(0).integers(0, count, nsample).astype(np.uint64)
    idx[:2] = [0, count - 1]
    exp = np.empty(nsample, np.uint16 if bf16 else np.float32)
    fn(exp.ctypes.data, idx.ctypes.data, nsample, seed, n)
    got = out[torch.from_numpy(idx.astype(np.int64)).to(out.device)]
    got = got.view(torch.int16).cpu().numpy().view(np.uint16) if bf16 else got.cpu().numpy()
    return bool(np.array_equal(got.view(np.uint8), exp.view(np.uint8)))


# The kernel the default (auto) config runs on C2: the tile engine's f32
# default shape on the dynamic schedule (hiccl_amd/csrc/reduce.hip: 256
# lanes x 4 packets, nt/nt).
DEFAULT_KERNEL = "OpF32, 256, 4, 11, 0>"


def traffic_from_profiles(n, count, kernel=DEFAULT_KERNEL, run_kernel_ms=None):
    """HBM bytes per launch from a committed PMC summary of this workload AND
    this kernel (profiles/*_pmc.json written by tools/profile.sh).  The
    traffic ratio carries over between boxes; a profile's kernel time does
    not, so among the matching profiles the newest whose rocprofv3 kernel
    time is at or below this run's kernel mean (`run_kernel_ms`) is cited --
    a profile that fits this run -- else the newest, with `fits_this_run`
    False."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    matches = []
    for f in sorted(os.listdir(pdir)):
        if f.endswith("_pmc.json"):
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except (OSError, ValueError):
                continue
            if (d.get("n_inputs") == n and d.get("count") == count and d.get("hbm_bytes_per_launch")
                    and not d.get("variant")  # e.g. the misaligned-input run: not the headline's buckets
                    and kernel and kernel in d.get("kernel", "")):
                matches.append(d)
    if not matches:
        return None
    fit = [d for d in matches if run_kernel_ms and d.get("rocprof_avg_kernel_ns")
           and d["rocprof_avg_kernel_ns"] * 1e-6 <= run_kernel_ms]
    best = dict(fit[-1] if fit else matches[-1])
    best["fits_this_run"] = bool(fit)
    best["profiles_considered"] = len(matches)
    return best


# ------------------------------------------------------------------ main ----

# flag -> (tools/bench_modes.py function, help)
MODES = {"nway": ("nway", "config 3: N = 2..64 inputs x 256 MiB"),
         "c3vsc2": ("c3_vs_c2", "config 3 per n interleaved with config 2 on one box"),
         "chunks": ("chunks", "config 4: 16 MiB..4 GiB per input in 1 MiB computes"),
         "roundtrip": ("roundtrip", "inputs and output in host memory: H2D + kernel + D2H"),
         "progstep": ("progstep", "one C5 step: separate launches vs one step program")}

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=8, help="inputs per bucket")
    ap.add_argument("--log2count", type=int, default=28, help="elements per input = 2^x")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-placement", default="", help="CPU baseline thread placement: " + " | ".join(CPU_POLICIES)
                    + " (default HICCL_CPU_PLACEMENT or l3spread); --cpu-only: a comma list")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (default: the cgroup quota)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="only the CPU baseline (no GPU touched), once per --cpu-placement policy")
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--bpc", type=int, default=0)
    ap.add_argument("--nt", type=int, default=-1)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--store", type=int, default=-1)
    ap.add_argument("--engine", type=int, default=0, help="0 auto, 1 tile, 2 phase")
    # secondary modes (tools/bench_modes.py); the closed tuning probes are in
    # tools/archive/bench_probes.py
    for flag, what in MODES.items():
        ap.add_argument("--" + flag, action="store_true", help=what[1])
    ap.add_argument("--rounds", type=int, default=5, help="c3vsc2: interleaved rounds")
    ap.add_argument("--cpu-leg", action="store_true", help=argparse.SUPPRESS)  # child of cpu_baseline()
    ap.add_argument("--expect-file", default="", help=argparse.SUPPRESS)
    ap.add_argument("--no-misaligned", action="store_true",
                    help="skip the misaligned second C2 run (rocprofv3 runs: one kernel shape per trace)")
    ap.add_argument("--no-c5", action="store_true", help="N > 1: skip the config-5 all-reduce leg")
    ap.add_argument("--c5-log2count", type=int, default=25,
                    help="config-5 leg: elements per rank per chunk = 2^x (25: 1 GiB fp32 send buffer at 8 ranks)")
    ap.add_argument("--c5-iters", type=int, default=5)
    ap.add_argument("--c5", type=int, default=0, metavar="RANKS",
                    help="run only the config-5 leg with RANKS MPI ranks (one per GPU when there are enough; "
                         "otherwise a rehearsal with ranks sharing GPUs) and print its JSON")
    ap.add_argument("--c5-force-stream", action="store_true",
                    help="--c5 rehearsal: HICCL_STREAM_ORDERED=force, so the stream-ordered modes run "
                         "stream-ordered with ranks sharing a GPU")
    ap.add_argument("--c5-only", default="", help="--c5: comma list of mode keys to run")
    args = ap.parse_args()
    if args.cpu_leg:
        return cpu_leg(args)
    if args.cpu_only:
        for pol in (args.cpu_placement or "l3spread").split(","):
            res, _ = cpu_baseline(args.n, 1 << args.log2count, args.cpu_budget, policy=pol,
                                  threads=args.cpu_threads or None)
            print(json.dumps({"mode": "cpu_only", "policy": pol, "cpu_baseline": res}), flush=True)
        return 0
    if args.c5:
        only = tuple(args.c5_only.split(",")) if args.c5_only else None
        print(json.dumps({"mode": "c5", **run_c5(args.c5, args, allow_shared=True, only=only,
                                                 force_stream=args.c5_force_stream)}), flush=True)
        return 0

    c5 = None
    if os.environ.get("WORLD_SIZE", "1") != "1" and not args.no_c5:
        # before this process touches a GPU: the MPI job owns every GPU meanwhile
        c5 = c5_leg(args)
    dist = Dist(args.gpus)
    for flag, (fn, _) in MODES.items():
        if getattr(args, flag):
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import bench_modes
            return getattr(bench_modes, fn)(args)

    n, count = args.n, 1 << args.log2count
    cfg = None
    if args.block or args.unroll or args.bpc or args.grid or args.nt >= 0 or args.store >= 0 or args.engine:
        cfg = dict(block=args.block, unroll=args.unroll, blocks_per_cu=args.bpc, grid=args.grid,
                   nontemporal=args.nt + 1 if args.nt >= 0 else 0, store_policy=args.store + 1 if args.store >= 0 else 0,
                   engine=args.engine)
    ins, out = make_bucket(n, count)
    step = lambda: hiccl_amd.reduce(out, ins, config=cfg)  # noqa: E731
    wall, kms = time_launches(step, args.steps, args.warmup, dist)
    wall_max = dist.max(wall)
    bytes_step = (n + 1) * count * 4
    value = whole_job_gbps(dist.world, bytes_step, args.steps, wall_max)
    kern_s = float(np.mean(kms)) * 1e-3
    achieved = bytes_step / kern_s / 1e9

    # full-bucket parity (N = 1, rank 0): the GPU's whole output against the
    # reference's own CPU reduce_kernel on the same generator and seed, done
    # by the CPU baseline leg below
    gpu_out = None
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu and cfg is None:
        gpu_out = out.cpu().numpy()
    # parity spot check of this very output against the oracle generator
    parity = None
    ora_so = os.path.join(ROOT, "oracle", "liboracle.so")
    if os.path.exists(ora_so):
        ora = ctypes.CDLL(ora_so)
        idx = np.random.default_rng(dist.rank).integers(0, count, 1024).astype(np.uint64)
        exp = np.empty(len(idx), np.float32)
        ora.oracle_sample_sum_f32.restype = None
        ora.oracle_sample_sum_f32(ctypes.c_void_p(exp.ctypes.data), ctypes.c_void_p(idx.ctypes.data),
                                  ctypes.c_size_t(len(idx)), ctypes.c_uint64(SEED), ctypes.c_int(n))
        got = out[torch.from_numpy(idx.astype(np.int64)).cuda()].cpu().numpy()
        parity = bool(np.array_equal(got.view(np.uint32), exp.view(np.uint32)))
        if not parity:
            log("bench: PARITY FAILURE against the oracle sample")
    mix_gbps = mix_ceiling(ins, out, count) if dist.rank == 0 else None
    read_gbps = mix_ceiling(ins, out, count, mode=1) if dist.rank == 0 else None
    write_gbps = mix_ceiling(ins, out, count, mode=2) if dist.rank == 0 else None
    del ins, out
    torch.cuda.empty_cache()

    parity = bool(dist.max(0.0 if parity in (True, None) else 1.0) == 0.0) if parity is not None else None
    copy_gbps = copy_ceiling() if dist.rank == 0 else None
    misaligned = (c2_misaligned(n, count, args.steps, args.warmup, headline_s=kern_s)
                  if dist.rank == 0 and cfg is None and not args.no_misaligned else None)
    layout_ab = (c2_layout_ab(n, count, args.steps, args.warmup, headline_s=kern_s)
                 if dist.rank == 0 and cfg is None and not args.no_misaligned else None)
    prof = traffic_from_profiles(n, count, run_kernel_ms=kern_s * 1e3) if cfg is None else None
    cpu, parity_full = None, None
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu:
        cpu, parity_full = cpu_baseline(n, count, args.cpu_budget, gpu_out, policy=args.cpu_placement or None,
                                        threads=args.cpu_threads or None)
        if parity_full and not parity_full["ok"]:
            log(f"bench: FULL-BUCKET PARITY FAILURE: {parity_full['mismatches']} of {count} words differ")
    del gpu_out
    dist.close()
    if dist.rank != 0:
        return 0
    props = torch.cuda.get_device_properties(0)
    cus, mclk, bus = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.check(L.lib().hiccl_device_info(torch.cuda.current_device(), ctypes.byref(cus), ctypes.byref(mclk),
                                      ctypes.byref(bus)), "device_info")
    # HBM3E moves 4 bits per pin per reported memory clock (8 Gb/s per pin at
    # the 2 GHz the runtime reports on MI355X): 8192 bits -> 8.19 TB/s, the spec
    props_peak = 4.0 * mclk.value * 1e3 * bus.value / 8 / 1e9
    serial = serial_rw_model(n * count * 4, count * 4, read_gbps, copy_gbps, kern_s, write_gbps)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform [-1,1) counter-hash, device-generated)",
        "config": {"workload": f"C2: {n} inputs x 2^{args.log2count} fp32 ({count * 4 >> 20} MiB/input) -> 1 output, "
                               "device-resident, one hiccl_reduce launch per step",
                   "layout": "one bucket allocation (hiccl_bucket_alloc layout: buffer j at j x "
                             f"{int(L.lib().hiccl_bucket_stride(L.HICCL_FLOAT32, count))} B); separate "
                             "allocations in c2_layout_ab",
                   "n_inputs": n, "count": count, "bytes_per_step": bytes_step,
                   "kernel_config": cfg or "default", "parallelism": f"replicas x{dist.world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     # the HBM-read view: the n input reads only
                     "read_achieved_GBps": round(n * count * 4 / kern_s / 1e9, 1),
                     "read_frac": round(n * count * 4 / kern_s / 1e9 / HBM_PEAK_GBPS, 4),
                     # the read view against what this box's HBM delivers to a
                     # read-only 8-stream probe on the same buckets
                     "read_frac_of_read_ceiling": round(n * count * 4 / kern_s / 1e9 / read_gbps, 4)
                     if read_gbps else None,
                     # PMC bytes per launch of this kernel on this workload from a
                     # committed rocprofv3 profile (traffic_source), not counted in
                     # this run: bench.py does not run under rocprofv3
                     "traffic": (prof or {}).get("hbm_bytes_per_launch"),
                     "traffic_from_profile": (
                         {"tag": prof.get("tag"), "file": f"profiles/{prof.get('tag')}_pmc.json",
                          "box_kernel_ms": round(prof["rocprof_avg_kernel_ns"] * 1e-6, 4)
                          if prof.get("rocprof_avg_kernel_ns") else None,
                          "over_algorithmic": round(prof["traffic_over_algorithmic"], 5)
                          if prof.get("traffic_over_algorithmic") else None,
                          # the profile's kernel time at or below this run's kernel mean
                          "fits_this_run": prof["fits_this_run"],
                          "profiles_considered": prof["profiles_considered"],
                          "measured_in_this_run": False} if prof else None),
                     "kernel_ms_mean": round(kern_s * 1e3, 4), "kernel_ms_min": round(min(kms), 4),
                     "kernel_ms_median": round(float(np.median(kms)), 4), "kernel_ms_max": round(max(kms), 4),
                     "mix_ceiling_GBps": round(mix_gbps, 1) if mix_gbps else None,
                     "frac_of_mix_ceiling": round(achieved / mix_gbps, 4) if mix_gbps else None,
                     "read_ceiling_GBps": round(read_gbps, 1) if read_gbps else None,
                     "frac_of_read_ceiling": round(achieved / read_gbps, 4) if read_gbps else None,
                     "copy_ceiling_GBps": round(copy_gbps, 1) if copy_gbps else None,
                     "frac_of_copy": round(achieved / copy_gbps, 4) if copy_gbps else None,
                     "serial_rw_model": serial,
                     "traffic_source": (prof or {}).get("source")},
        "cpu_baseline": cpu,
        "parity_full": parity_full,
        "parity_sample_ok": parity,
        "device": props.name,
        "device_props": {"gcn_arch": props.gcnArchName, "cus": cus.value, "mem_clock_khz": mclk.value,
                         "mem_bus_width_bits": bus.value, "peak_GBps_from_props_x4": round(props_peak, 1),
                         "total_mem_GiB": round(props.total_memory / 2**30, 1)},
        "control_plane": dist.backend,
    }
    if misaligned is not None:
        line["c2_misaligned"] = misaligned
    if layout_ab is not None:
        line["c2_layout_ab"] = layout_ab
    if c5 is not None:
        line["c5"] = c5
    # the full record on stderr, the driver's one line (compact: the driver
    # keeps a tail of stdout) on stdout
    log("bench-detail " + json.dumps(line))
    print(json.dumps(compact_line(line)), flush=True)
    return 0


def c2_misaligned(n, count, steps, warmup, headline_s=None):
    """SURVEY.md 8d's second C2 run, as an interleaved A/B on ONE set of
    allocations: input k is read either from its 16-B-aligned base or from
    1 + k mod 3 elements past it (the mutual misalignment partition()
    produces, reduce.h:401-415), output aligned; launches alternate between
    the two views so placement and box state are common to both.  A sampled
    bitwise check of each view's output against the oracle generator.
    Both legs are also given over the headline's own kernel mean
    (`headline_s`, the same process's C2 launches on their own buffers):
    the A/B's aligned leg runs on other allocations and can land slower than
    the headline (BENCH_r05: 1.5918 vs 1.4744 ms), so the absolute shifted
    rate is `shifted_frac` and `shifted_over_headline`."""
    offs = [1 + k % 3 for k in range(n)]
    # the headline's layout (one bucket allocation), each input 4 elements
    # longer for the shifted view
    bases, out = hiccl_amd.bucket(n, count + 4)
    out = out[:count]
    for k, b in enumerate(bases):  # element j of base k = generator(k, j), shifted views included
        hiccl_amd.fill_uniform(b, SEED, k)
    aligned = [b[:count] for b in bases]
    shifted = [b[o:o + count] for b, o in zip(bases, offs)]
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    runs = {"aligned": lambda: hiccl_amd.reduce(out, aligned), "shifted": lambda: hiccl_amd.reduce(out, shifted)}
    for _ in range(warmup):
        for fn in runs.values():
            fn()
    torch.cuda.synchronize()
    ms = {k: [] for k in runs}
    for _ in range(steps):
        for k, fn in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            b.record(s)
            ms[k].append((a, b))
    torch.cuda.synchronize()
    t = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in ms.items()}
    parity = {}
    for k, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        parity[k] = sample_check_shifted(out, [0] * n if k == "aligned" else offs, count)
    bytes_step = (n + 1) * count * 4
    res = {"ab": "interleaved launches on the same allocations", "input_offsets": offs,
           "aligned_kernel_ms_mean": round(t["aligned"] * 1e3, 4), "shifted_kernel_ms_mean": round(t["shifted"] * 1e3, 4),
           "shifted_over_aligned": round(t["shifted"] / t["aligned"], 4),
           "aligned_GBps": round(bytes_step / t["aligned"] / 1e9, 1),
           "shifted_GBps": round(bytes_step / t["shifted"] / 1e9, 1),
           "shifted_frac": round(bytes_step / t["shifted"] / 1e9 / HBM_PEAK_GBPS, 4),
           "aligned_frac": round(bytes_step / t["aligned"] / 1e9 / HBM_PEAK_GBPS, 4),
           "parity_sample_ok": parity}
    if headline_s:
        res["headline_kernel_ms_mean"] = round(headline_s * 1e3, 4)
        res["aligned_over_headline"] = round(t["aligned"] / headline_s, 4)
        res["shifted_over_headline"] = round(t["shifted"] / headline_s, 4)
    del bases, aligned, shifted, out
    torch.cuda.empty_cache()
    return res


def c2_layout_ab(n, count, steps, warmup, headline_s=None):
    """The bucket layout against separate allocations, as an interleaved A/B
    in one process: the headline's layout (one allocation, hiccl_amd.bucket)
    and the same buffers as n + 1 separate torch allocations (the layout
    rounds 1-5 measured), launches alternating; outputs compared bit for
    bit.  Separate allocations leave the streams' relative physical
    placement to chance: up to 8 % apart between buckets of one process
    (profiles/r06d_alloc.jsonl)."""
    legs = {"bucket": make_bucket(n, count), "separate": make_bucket(n, count, layout="separate")}
    runs = {k: (lambda i=i, o=o: hiccl_amd.reduce(o, i)) for k, (i, o) in legs.items()}
    for _ in range(warmup):
        for fn in runs.values():
            fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ms = {k: [] for k in runs}
    for _ in range(steps):
        for k, fn in runs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            b.record(s)
            ms[k].append((a, b))
    torch.cuda.synchronize()
    t = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) * 1e-3 for k, v in ms.items()}
    same = bool(torch.equal(legs["bucket"][1].view(torch.int32), legs["separate"][1].view(torch.int32)))
    bytes_step = (n + 1) * count * 4
    res = {"ab": "interleaved launches, one bucket allocation vs n + 1 separate allocations",
           "bucket_stride_bytes": int(L.lib().hiccl_bucket_stride(L.HICCL_FLOAT32, count)),
           "bucket_kernel_ms_mean": round(t["bucket"] * 1e3, 4), "separate_kernel_ms_mean": round(t["separate"] * 1e3, 4),
           "separate_over_bucket": round(t["separate"] / t["bucket"], 4),
           "bucket_frac": round(bytes_step / t["bucket"] / 1e9 / HBM_PEAK_GBPS, 4),
           "separate_frac": round(bytes_step / t["separate"] / 1e9 / HBM_PEAK_GBPS, 4),
           "outputs_identical": same}
    if headline_s:
        res["separate_over_headline"] = round(t["separate"] / headline_s, 4)
    del legs, runs
    torch.cuda.empty_cache()
    return res


def sample_check_shifted(out, offs, count, seed=SEED, nsample=512):
    """Bitwise check of out[i] = (((0 + g(0, i + offs[0])) + g(1, i + offs[1]))
    + ...) at random i, g = the oracle generator (oracle_fill_uniform_f32
    at a start index)."""
    ora_so = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(ora_so):
        return None
    ora = ctypes.CDLL(ora_so)
    fill = ora.oracle_fill_uniform_f32
    fill.restype = None
    fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t]
    idx = np.random.default_rng(1).integers(0, count, nsample)
    idx[:2] = [0, count - 1]
    exp = np.zeros(nsample, np.float32)
    v = np.empty(1, np.float32)
    for k, o in enumerate(offs):
        col = np.empty(nsample, np.float32)
        for j, i in enumerate(idx):
            fill(v.ctypes.data, 1, seed, k, int(i) + o)
            col[j] = v[0]
        exp = (exp + col).astype(np.float32)  # one f32 add per input, in input order
    got = out[torch.from_numpy(idx.astype(np.int64)).to(out.device)].cpu().numpy()
    return bool(np.array_equal(got.view(np.uint32), exp.view(np.uint32)))


if __name__ == "__main__":
    sys.exit(main())
