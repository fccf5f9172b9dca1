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

Other modes (not the driver's line): --sweep (tuning variants, interleaved in
one process), --nway (config 3), --chunks (config 4), --roundtrip (host
memory H2D + kernel + D2H rate for DESIGN.md).
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


def run_c5(world, args, allow_shared=False, only=None):
    """`allow_shared`: run even with fewer GPUs than ranks (a rehearsal on a
    1-GPU box, tests/test_c5_leg_gpu.py; the library then runs host-driven).
    `only`: run just these mode keys."""
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
    if not os.path.exists(C5_EXE):
        return {"skipped": f"{C5_EXE} not built"}
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
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

def make_bucket(n, count, dtype=torch.float32, seed=SEED):
    # integer buckets (size_t: the reference drivers' T) get the float
    # generator's bits
    fill_as = {torch.int64: torch.float64, torch.int32: torch.float32}.get(dtype, dtype)
    ins = [torch.empty(count, dtype=fill_as, device="cuda") for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    ins = [t.view(dtype) for t in ins]
    out = torch.empty(count, dtype=dtype, device="cuda")
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

def host_cpus():
    """CPUs this process may use: the affinity set, capped by a cgroup CPU
    quota (a GPU box slice), and the physical cores among them."""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    cores = set()
    for c in aff:
        try:
            pkg = open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id").read().strip()
            core = open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id").read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", str(c)))
    threads = min(len(aff), quota) if quota else len(aff)
    return {"threads": threads, "affinity_cpus": len(aff), "cgroup_quota_cpus": quota,
            "physical_cores_in_affinity": len(cores)}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(n, count, budget_s=10.0, gpu_out=None):
    """The reference's CPU reduce_kernel on this host, in a child process so
    OpenMP starts with OMP_NUM_THREADS = every CPU this process may use and
    OMP_PROC_BIND=spread (libgomp reads them once, at load; BASELINE.md:34).
    `gpu_out`: the GPU's output of the same bucket (a host float32 array):
    the child compares all `count` words with the reference's own output
    (the full-bucket parity check)."""
    cpus = host_cpus()
    env = dict(os.environ, OMP_NUM_THREADS=str(cpus["threads"]), OMP_PROC_BIND="spread", OMP_PLACES="cores"
               if cpus["physical_cores_in_affinity"] >= cpus["threads"] else "threads")
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
    res.update({k: v for k, v in cpus.items() if k != "threads"})
    return res, parity


def cpu_leg(args):
    """Child of cpu_baseline(): time the reference reduce_kernel (or the C
    restatement) over the full bucket; optionally compare with a GPU output."""
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
    for k, b in enumerate(bufs):  # parallel first touch inside the generator
        fill(b.ctypes.data, count, SEED, k, 0)
    out = np.empty(count, np.float32)
    fill(out.ctypes.data, count, SEED, 99, 0)  # first touch of the output
    tab = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])

    def one():
        t = time.perf_counter()
        if kind == "reference":
            fn(out.ctypes.data, count, tab, n)
        else:
            fn(out.ctypes.data, tab, n, count)
        return time.perf_counter() - t

    one()  # warm
    times = []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < args.cpu_budget and len(times) < 50:
        times.append(one())
    med = float(np.median(times))
    rate = lambda t: round((n + 1) * count * 4 / t / 1e9, 2)  # noqa: E731
    # the spread over the passes, as the reference prints min / median / max
    # for its own timings (compute.h:165-195): the host's other tenants move
    # this rate 2-3x between runs
    res = {"value": rate(med), "unit": "GB/s", "threads": threads, "kind": kind,
           "min": rate(max(times)), "max": rate(min(times)), "passes": len(times),
           "pass_ms": [round(t * 1e3, 2) for t in times],
           "sample": f"{n} x 2^{args.log2count} fp32 -> 1 output (the full config-2 bucket), median of "
                     f"{len(times)} passes ({med * 1e3:.1f} ms each), OpenMP {threads} threads "
                     f"(OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND', '')}), {cpu_model()}"}
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


def traffic_from_profiles(n, count, kernel=DEFAULT_KERNEL):
    """HBM bytes per launch from a committed PMC summary of this workload AND
    this kernel (profiles/*_pmc.json written by tools/profile.sh)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if not os.path.isdir(pdir):
        return None
    for f in sorted(os.listdir(pdir)):
        if f.endswith("_pmc.json"):
            try:
                d = json.load(open(os.path.join(pdir, f)))
            except (OSError, ValueError):
                continue
            if (d.get("n_inputs") == n and d.get("count") == count and d.get("hbm_bytes_per_launch")
                    and not d.get("variant")  # e.g. the misaligned-input run: not the headline's buckets
                    and kernel and kernel in d.get("kernel", "")):
                best = d
    return best


# ------------------------------------------------------------------ main ----

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=8, help="inputs per bucket")
    ap.add_argument("--log2count", type=int, default=28, help="elements per input = 2^x")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--bpc", type=int, default=0)
    ap.add_argument("--nt", type=int, default=-1)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--store", type=int, default=-1)
    ap.add_argument("--engine", type=int, default=0, help="0 auto, 1 tile, 2 phase")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--nway", action="store_true")
    ap.add_argument("--c3vsc2", action="store_true", help="C3 per n interleaved with C2 on one box")
    ap.add_argument("--c3offsets", action="store_true", help="C3 few inputs: relative input placement")
    ap.add_argument("--rounds", type=int, default=5, help="c3vsc2: interleaved rounds")
    ap.add_argument("--chunks", action="store_true")
    ap.add_argument("--roundtrip", action="store_true")
    ap.add_argument("--progstep", action="store_true", help="one C5 step: separate launches vs one step program")
    ap.add_argument("--stepscale", action="store_true",
                    help="the C5 step's batched kernel scaled 1/8x..16x: fixed cost + bytes / rate fit")
    ap.add_argument("--c2variants", action="store_true")
    ap.add_argument("--crossover", action="store_true")
    ap.add_argument("--planvs", action="store_true")
    ap.add_argument("--schedsweep", action="store_true")
    ap.add_argument("--sweepdtype", default="f32", help="schedsweep: f32 | bf16 | bf16wide | f64 | u64 | i32")
    ap.add_argument("--sweepset", default="", help="schedsweep: '' (schedule/grab) | occupancy")
    ap.add_argument("--xdtype", default="both", help="crossover: f32 | bf16 | both")
    ap.add_argument("--xmib", default="", help="crossover: comma list of MiB per input")
    ap.add_argument("--xn", default="", help="crossover: comma list of input counts")
    ap.add_argument("--buckets", type=int, default=0, help="schedsweep: this many fresh --n x 2^--log2count buckets")
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
    args = ap.parse_args()
    if args.cpu_leg:
        return cpu_leg(args)
    if args.c5:
        print(json.dumps({"mode": "c5", **run_c5(args.c5, args, allow_shared=True)}), flush=True)
        return 0

    c5 = None
    if os.environ.get("WORLD_SIZE", "1") != "1" and not args.no_c5:
        # before this process touches a GPU: the MPI job owns every GPU meanwhile
        c5 = c5_leg(args)
    dist = Dist(args.gpus)
    if args.sweep:
        return sweep(args)
    if args.nway:
        return nway(args)
    if args.c3vsc2:
        return c3_vs_c2(args)
    if args.c3offsets:
        return c3_offsets(args)
    if args.chunks:
        return chunks(args)
    if args.c2variants:
        return c2variants(args)
    if args.crossover:
        return crossover(args)
    if args.planvs:
        return planvs(args)
    if args.schedsweep:
        return schedsweep(args)
    if args.roundtrip:
        return roundtrip(args)
    if args.progstep:
        return progstep(args)
    if args.stepscale:
        return stepscale(args)

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
    misaligned = c2_misaligned(n, count, args.steps, args.warmup) if dist.rank == 0 and cfg is None and not args.no_misaligned else None
    prof = traffic_from_profiles(n, count) if cfg is None else None
    cpu, parity_full = None, None
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu:
        cpu, parity_full = cpu_baseline(n, count, args.cpu_budget, gpu_out)
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
    if c5 is not None:
        line["c5"] = c5
    print(json.dumps(line), flush=True)
    return 0


def sweep(args):
    """Interleaved A/B of kernel variants in one process (rule 24), with the
    no-arithmetic 8R+1W probe (tools/libhbm_probe.so) as the ceiling row."""
    n, count = args.n, 1 << args.log2count
    ins, out = make_bucket(n, count)
    variants = [dict(engine=1), dict(engine=1, grid=192), dict(engine=1, block=512, unroll=4, grid=512)]
    for shape in ((512, 16), (1024, 4), (512, 8), (1024, 8), (256, 16)):
        for grid in (0, 512):
            variants.append(dict(engine=2, block=shape[0], unroll=shape[1], grid=grid))
    for nt, store in ((1, 1), (1, 2), (2, 1), (2, 3)):
        variants.append(dict(engine=2, nontemporal=nt, store_policy=store))
    probe = None
    pso = os.path.join(ROOT, "tools", "libhbm_probe.so")
    if os.path.exists(pso):
        probe = ctypes.CDLL(pso)
        probe.probe_run.restype = ctypes.c_int
        probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                         ctypes.c_uint64, ctypes.c_void_p]
        tab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ins])
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for g in (192, 256):
            variants.append(dict(probe=True, block=256, unroll=4, nontemporal=2, store_policy=2, grid=g))

    def runner(v):
        if v.get("probe"):
            return lambda: probe.probe_run(0, 256, 4, 2, 2, 0, v["grid"], tab, n, ctypes.c_void_p(out.data_ptr()),
                                           count * 4, st)
        return lambda: hiccl_amd.reduce(out, ins, config=v)

    res = {i: [] for i in range(len(variants))}
    for rnd in range(3):
        for i, v in enumerate(variants):
            try:
                _, ms = time_launches(runner(v), 5, 2)
            except Exception as e:  # unsupported combination
                log("skip", v, e)
                continue
            res[i].append(float(np.median(ms)))
        log(f"sweep round {rnd} done")
    bytes_step = (n + 1) * count * 4
    rows = []
    for i, v in enumerate(variants):
        if res[i]:
            t = float(np.median(res[i]))
            rows.append((bytes_step / t / 1e6, t, v))
    rows.sort(key=lambda r: -r[0])
    for gbps, t, v in rows:
        print(json.dumps({"GBps": round(gbps, 1), "ms": round(t, 4), "frac": round(gbps / HBM_PEAK_GBPS, 4), **v}))
    return 0


def nway(args):
    """Config 3: N in 2..64 inputs x 2^26 fp32 (256 MiB each)."""
    count = 1 << 26
    copy_gbps = copy_ceiling()
    for n in (2, 3, 4, 8, 16, 32, 64):
      ins, out = make_bucket(n, count)
      # the box's bound for this read/write mix on these very buckets
      read_gbps = mix_ceiling(ins, out, count, mode=1)
      write_gbps = mix_ceiling(ins, out, count, mode=2)
      for eng in (0, 1):  # auto (= phase at this size), tile
        cfg = dict(engine=eng) if eng else None
        _, ms = time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), args.steps, args.warmup)
        t = float(np.median(ms)) * 1e-3
        b = (n + 1) * count * 4
        print(json.dumps({"config": "C3", "engine": ["auto", "tile"][eng], "n": n, "count": count,
                          "kernel_ms": round(t * 1e3, 4),
                          "GBps": round(b / t / 1e9, 1), "frac_hbm": round(b / t / 1e9 / HBM_PEAK_GBPS, 4),
                          "read_GBps": round(n * count * 4 / t / 1e9, 1),
                          "frac_of_copy": round(b / t / 1e9 / copy_gbps, 4),
                          "serial_rw_model": serial_rw_model(n * count * 4, count * 4, read_gbps, copy_gbps, t, write_gbps)}),
              flush=True)
      del ins, out
      torch.cuda.empty_cache()
    return 0


def c3_vs_c2(args):
    """Config 3 per n on ONE box with config 2 as the control: C2 (8 x 2^28)
    and C3 n in {2, 3, 4, 8, 16, 32, 64} x 2^26 fp32, every bucket allocated
    once, then `--rounds` interleaved rounds (C2, then each n, `--steps`
    launches each, AUTO).  Per n: GB/s (median over rounds of the per-round
    median kernel time), its ratio to the same round's C2, and the serial
    read/write model on its own buckets (the box's read-only and write-only
    probe rates: R / read + W / write, roofline.serial_rw_model) -- so a
    gap between n is either the box's HBM bound for that n's buckets or
    named.  One JSON line per bucket, then a summary line."""
    sizes = [("C2", 8, 1 << 28)] + [("C3", n, 1 << 26) for n in (2, 3, 4, 8, 16, 32, 64)]
    copy_gbps = copy_ceiling()
    buckets = []
    for cfg, n, count in sizes:
        ins, out = make_bucket(n, count, seed=SEED + 17 * n + (count >> 26))
        read = mix_ceiling(ins, out, count, mode=1)
        write = mix_ceiling(ins, out, count, mode=2)
        buckets.append({"config": cfg, "n": n, "count": count, "ins": ins, "out": out, "read": read, "write": write,
                        "ms": []})
        log(f"c3vsc2: {cfg} n={n} allocated, probes read {read} write {write} GB/s")
    for rnd in range(args.rounds):
        for b in buckets:
            _, ms = time_launches(lambda: hiccl_amd.reduce(b["out"], b["ins"]), args.steps, args.warmup)
            b["ms"].append(float(np.median(ms)))
        log(f"c3vsc2: round {rnd} done")
    c2 = buckets[0]
    c2_rates = [(c2["n"] + 1) * c2["count"] * 4 / (t * 1e-3) / 1e9 for t in c2["ms"]]
    rows = []
    for b in buckets:
        n, count = b["n"], b["count"]
        alg = (n + 1) * count * 4
        rates = [alg / (t * 1e-3) / 1e9 for t in b["ms"]]
        t = float(np.median(b["ms"])) * 1e-3
        ok = sample_check(b["out"], n, count, seed=SEED + 17 * n + (count >> 26))
        row = {"config": b["config"], "n": n, "count": count, "kernel_ms": round(t * 1e3, 4),
               "GBps": round(alg / t / 1e9, 1), "frac_hbm": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4),
               "GBps_per_round": [round(r, 1) for r in rates],
               "ratio_to_c2": round(float(np.median([r / c for r, c in zip(rates, c2_rates)])), 4),
               "read_probe_GBps": round(b["read"], 1) if b["read"] else None,
               "write_probe_GBps": round(b["write"], 1) if b["write"] else None,
               "serial_rw_model": serial_rw_model(n * count * 4, count * 4, b["read"], copy_gbps, t, b["write"]),
               "sample_exact": ok}
        rows.append(row)
        print(json.dumps(row), flush=True)
    c3 = [r for r in rows if r["config"] == "C3"]
    print(json.dumps({"summary": "c3_vs_c2", "rounds": args.rounds, "steps": args.steps, "copy_GBps": round(copy_gbps, 1),
                      "c2_GBps": rows[0]["GBps"], "c2_model_frac": (rows[0]["serial_rw_model"] or {}).get("frac_write_probe"),
                      "c3_ratio_to_c2": {r["n"]: r["ratio_to_c2"] for r in c3},
                      "c3_model_frac": {r["n"]: (r["serial_rw_model"] or {}).get("frac_write_probe") for r in c3},
                      "device": torch.cuda.get_device_properties(0).name}), flush=True)
    return 0


def c3_offsets(args):
    """Config 3 with few inputs: does where the inputs sit relative to each
    other move the rate?  n in {2, 3, 4, 8} x 2^26 fp32; input k is a view
    starting k x `off` bytes into a padded allocation (off = 0, 4 KiB,
    64 KiB, 1 MiB + 4 KiB), so element i of every input no longer shares its
    address bits below the offset with the other inputs; AUTO and every
    engine form that leads somewhere, interleaved rounds, one set of
    allocations per n (the same physical pages for every offset)."""
    count = 1 << 26
    offs = (0, 4 << 10, 64 << 10, (1 << 20) + (4 << 10))
    forms = [("auto", None), ("phase", dict(engine=2, schedule=1)), ("tile_u4_static", dict(engine=1, schedule=1))]
    for n in (2, 3, 4, 8):
        pad = (n - 1) * max(offs) // 4 + 64
        raw = [torch.empty(count + pad, device="cuda") for _ in range(n)]
        out = torch.empty(count, device="cuda")
        res = {}
        for rnd in range(args.rounds):
            for off in offs:
                ins = [raw[k][k * off // 4:k * off // 4 + count] for k in range(n)]
                if rnd == 0:
                    for k, t in enumerate(ins):
                        hiccl_amd.fill_uniform(t, SEED + off, k)
                for name, cfg in forms:
                    _, ms = time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), args.steps, args.warmup)
                    res.setdefault((off, name), []).append(float(np.median(ms)))
                if rnd == 0:
                    torch.cuda.synchronize()
                    res[(off, "ok")] = sample_check(out, n, count, seed=SEED + off)
        alg = (n + 1) * count * 4
        row = {"mode": "c3offsets", "n": n, "count": count}
        for off in offs:
            row[f"off{off}"] = {name: round(alg / (float(np.median(res[(off, name)])) * 1e-3) / 1e9, 1)
                                for name, _ in forms}
            row[f"off{off}"]["sample_exact"] = res[(off, "ok")]
        print(json.dumps(row), flush=True)
        del raw, out
        torch.cuda.empty_cache()
    return 0


def schedsweep(args):
    """Static vs dynamic unit schedule (and grab size) for both engines,
    fp32, interleaved rounds.  Default cases n = 2/4/8/16 at 256 MiB and
    1 GiB per input; --n N --log2count L: that shape on 3 fresh buckets."""
    cases = ((2, 256), (2, 1024), (4, 256), (4, 1024), (8, 256), (8, 1024), (16, 256))
    if args.buckets:
        cases = ((args.n, (1 << args.log2count) * 4 >> 20),) * args.buckets
    elif args.xmib:
        ns = [int(v) for v in args.xn.split(",")] if args.xn else [args.n]
        cases = tuple((n, int(m)) for n in ns for m in args.xmib.split(","))
    variants = [("tile_static", dict(engine=1, schedule=1)), ("tile_dyn_g1", dict(engine=1, schedule=2, grab=1)),
                ("tile512_dyn_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=4)),
                ("tile_dyn_g2", dict(engine=1, schedule=2, grab=2)),
                ("phase_static", dict(engine=2, schedule=1)), ("phase_dyn_g1", dict(engine=2, schedule=2, grab=1)),
                ("auto", None)]
    if args.sweepset == "occupancy":  # C2-shaped: workgroups per CU / tile shape on the dynamic schedule
        variants = [("auto", None),
                    ("t256x4_bpc2_g1", dict(engine=1, schedule=2, grab=1, blocks_per_cu=2)),
                    ("t256x4_bpc2_g2", dict(engine=1, schedule=2, grab=2, blocks_per_cu=2)),
                    ("t512x2_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=2)),
                    ("t512x2_bpc2_g1", dict(engine=1, schedule=2, grab=1, block=512, unroll=2, blocks_per_cu=2)),
                    ("t256x2_bpc2_g2", dict(engine=1, schedule=2, grab=2, unroll=2, blocks_per_cu=2)),
                    ("t256x2_g2", dict(engine=1, schedule=2, grab=2, unroll=2)),
                    ("t256x4_g1_drain", dict(engine=1, schedule=2, grab=1, drain=1))]
    if args.sweepset == "small":  # few tiles per workgroup: more workgroups / smaller tiles
        variants = [("auto", None),
                    ("t256x4_bpc2", dict(engine=1, blocks_per_cu=2)),
                    ("t256x4_bpc4", dict(engine=1, blocks_per_cu=4)),
                    ("t256x2", dict(engine=1, unroll=2)),
                    ("t256x2_bpc2", dict(engine=1, unroll=2, blocks_per_cu=2)),
                    ("t256x1_bpc4", dict(engine=1, unroll=1, blocks_per_cu=4)),
                    ("t256x4_dyn", dict(engine=1, schedule=2, grab=1)),
                    ("phase", dict(engine=2))]
    if args.sweepset == "bf16occ":  # bf16 tile: hide the packed accumulator's VALU time
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_dyn_bpc2", dict(engine=1, schedule=2, blocks_per_cu=2)),
                    ("tile_dyn_bpc2_u2", dict(engine=1, schedule=2, blocks_per_cu=2, unroll=2)),
                    ("tile_dyn_b512u2", dict(engine=1, schedule=2, block=512, unroll=2)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_bpc2", dict(engine=2, schedule=1, blocks_per_cu=2))]
    if args.sweepset == "widetile":  # few inputs: wide TILE tiles (32 packets per lane in flight)
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("tile_u4_static", dict(engine=1, schedule=1)),
                    ("tile_u8_static", dict(engine=1, unroll=8, schedule=1)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u16_static", dict(engine=1, unroll=16, schedule=1)),
                    ("tile_u16_dyn", dict(engine=1, unroll=16, schedule=2, grab=1))]
    if args.sweepset == "widedyn":  # wide tiles on the dynamic schedule vs AUTO, larger buckets
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("tile_u4_dyn", dict(engine=1, unroll=4, schedule=2)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u8_dyn_g2", dict(engine=1, unroll=8, schedule=2, grab=2)),
                    ("tile_u16_dyn", dict(engine=1, unroll=16, schedule=2, grab=1))]
    if args.sweepset == "c3":  # config 3 per n: engine / occupancy / tile size
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_dyn_bpc2", dict(engine=1, schedule=2, blocks_per_cu=2)),
                    ("tile_dyn_u2_bpc2", dict(engine=1, schedule=2, unroll=2, blocks_per_cu=2)),
                    ("tile_static", dict(engine=1, schedule=1)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2))]
    if args.sweepset == "fewn":  # config 3's few-input buckets (n = 2-4): every engine form, interleaved
        variants = [("auto", None),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2)),
                    ("tile_u4_static", dict(engine=1, schedule=1)),
                    ("tile_u4_dyn", dict(engine=1, schedule=2)),
                    ("tile_u8_static", dict(engine=1, unroll=8, schedule=1)),
                    ("tile_u8_dyn", dict(engine=1, unroll=8, schedule=2, grab=1)),
                    ("tile_u4_static_bpc2", dict(engine=1, schedule=1, blocks_per_cu=2))]
    if args.sweepset == "phaseshapes":  # the phased engine's chunk shapes (block x packets per lane)
        variants = [("auto", None),
                    ("p512x16", dict(engine=2, block=512, unroll=16)),
                    ("p1024x8", dict(engine=2, block=1024, unroll=8)),
                    ("p512x8", dict(engine=2, block=512, unroll=8)),
                    ("p1024x4", dict(engine=2, block=1024, unroll=4)),
                    ("p256x16", dict(engine=2, block=256, unroll=16)),
                    ("p256x16_bpc2", dict(engine=2, block=256, unroll=16, blocks_per_cu=2))]
    if args.sweepset == "xover":  # engine x schedule crossover (sets AUTO)
        variants = [("auto", None),
                    ("tile_dyn", dict(engine=1, schedule=2)),
                    ("tile_static", dict(engine=1, schedule=1)),
                    ("tile_bpc4_static", dict(engine=1, schedule=1, blocks_per_cu=4)),
                    ("phase_static", dict(engine=2, schedule=1)),
                    ("phase_dyn", dict(engine=2, schedule=2))]
    for n, mib in cases:
        sdt = {"bf16": torch.bfloat16, "bf16wide": torch.bfloat16, "f64": torch.float64, "u64": torch.int64,
               "i32": torch.int32}.get(args.sweepdtype, torch.float32)
        wide = args.sweepdtype == "bf16wide"  # f32 accumulation (HICCL_ACC_WIDE) in every variant
        esz = torch.tensor([], dtype=sdt).element_size()
        count = (mib << 20) // esz
        ins, out = make_bucket(n, count, sdt)
        res = {}
        for rnd in range(5):
            for name, cfg in variants:
                if wide:
                    cfg = dict(cfg or {}, acc=1)
                try:
                    _, ms = time_launches(lambda: hiccl_amd.reduce(out, ins, config=cfg), max(args.steps, 10),
                                          args.warmup)
                except hiccl_amd.HicclError:  # a shape this type does not have (f64 / u64: block 256 only)
                    res[name] = None
                    continue
                res.setdefault(name, []).append(float(np.median(ms)))
        row = {"mode": "schedsweep", "n": n, "mib_per_input": mib}
        for name, v in res.items():
            if v is None:
                row[name] = None
                continue
            t = float(np.median(v)) * 1e-3
            row[name] = round((n + 1) * count * esz / t / 1e9, 1)
        row["dtype"] = str(sdt).split(".")[-1]
        if sdt in (torch.float64, torch.int64, torch.int32):  # in-order sum on the device (f64 adds, wrap-around ints)
            acc = torch.zeros_like(out)
            for t in ins:
                acc = acc + t
            iv = torch.int32 if sdt == torch.int32 else torch.int64
            row["parity_sample_ok"] = bool(torch.equal(acc.view(iv), out.view(iv)))
        elif wide:  # one f32 accumulation, rounded once
            acc = torch.zeros(out.shape, dtype=torch.float32, device=out.device)
            for t in ins:
                acc = acc + t.float()
            row["parity_sample_ok"] = bool(torch.equal(acc.to(torch.bfloat16).view(torch.int16), out.view(torch.int16)))
        else:
            row["parity_sample_ok"] = sample_check(out, n, count, bf16=(sdt == torch.bfloat16))
        print(json.dumps(row), flush=True)
        del ins, out
        torch.cuda.empty_cache()
    return 0


def planvs(args):
    """Plan-kernel overhead on the C2 bucket: one-shot launch vs a plan of
    1, 1024 (1 MiB) and 8192 (128 KiB) computes, interleaved rounds."""
    n, count = 8, 1 << 28
    ins, out = make_bucket(n, count)
    stream = torch.cuda.current_stream()
    plans = {}
    for name, ncomp, eng in (("plan_1", 1, 0), ("plan_1024", 1024, 0), ("plan_8192", 8192, 0),
                             ("plan_1024_tile", 1024, 1)):
        comp = hiccl_amd.Compute(torch.float32, device=torch.cuda.current_device(), engine=eng)
        off = 0
        for b in range(ncomp):
            c = count // ncomp + (1 if b < count % ncomp else 0)
            comp.add([(t, off) for t in ins], (out, off), c, compid=0)
            off += c
        plans[name] = comp
    runs = {"single": lambda: hiccl_amd.reduce(out, ins)}
    for name, comp in plans.items():
        runs[name] = (lambda c: (lambda: c.start(stream=stream)))(comp)
    res = {k: [] for k in runs}
    for _ in range(3):
        for k, fn in runs.items():
            _, ms = time_launches(fn, max(args.steps, 10), args.warmup)
            res[k].append(float(np.median(ms)))
    for k, v in res.items():
        t = float(np.median(v)) * 1e-3
        eng = plans[k].engine() if k in plans else None
        print(json.dumps({"mode": "planvs", "run": k, "engine": eng, "kernel_ms": round(t * 1e3, 4),
                          "GBps": round(9 * count * 4 / t / 1e9, 1)}), flush=True)
    ok = sample_check(out, n, count)
    print(json.dumps({"mode": "planvs", "parity_sample_ok": ok}), flush=True)
    for comp in plans.values():
        comp.close()
    return 0


def crossover(args):
    """Engine crossover: one-shot reduce of n = 2/4/8 inputs, 1-512 MiB per
    input, f32 and bf16, TILE vs PHASE (sets the AUTO threshold)."""
    dtypes = {"f32": (torch.float32,), "bf16": (torch.bfloat16,), "f64": (torch.float64,), "u64": (torch.int64,),
              "i32": (torch.int32,), "wide": (torch.float32, torch.float64, torch.int64, torch.int32)}.get(
                  args.xdtype, (torch.float32, torch.bfloat16))
    mibs = [int(m) for m in args.xmib.split(",")] if args.xmib else (1, 4, 16, 32, 64, 128, 256, 512)
    ns = [int(m) for m in args.xn.split(",")] if args.xn else (2, 4, 8)
    for dtype in dtypes:
        esz = torch.tensor([], dtype=dtype).element_size()
        for n in ns:
            for mib in mibs:
                count = (mib << 20) // esz
                ins, out = make_bucket(n, count, dtype)
                row = {"mode": "crossover", "dtype": str(dtype).split(".")[-1], "n": n, "mib_per_input": mib}
                for eng, name in ((1, "tile"), (2, "phase"), (0, "auto")):
                    _, ms = time_launches(lambda: hiccl_amd.reduce(out, ins, config=dict(engine=eng)),
                                          max(args.steps, 10), args.warmup)
                    t = float(np.median(ms)) * 1e-3
                    row[name + "_GBps"] = round((n + 1) * count * esz / t / 1e9, 1)
                print(json.dumps(row), flush=True)
                del ins, out
                torch.cuda.empty_cache()
    return 0


def progstep(args):
    """One C5 pipeline step on one GPU, without peers: the step's enqueue
    sequence -- a ready phase, the transport's copies (five 1 MiB byte
    copies), a done phase, the reductions (4 x n=2 + 1 x n=4 computes of
    2^18 f32, the {1,4,2} step shape), a tail phase --
    as separate launches (k_sigwait_phases + plan kernels: 5 kernels, the
    round-2 stream-ordered path) and as programs (each phase folded into the
    launch of the batch after it: 2 kernels + the tail phase, which in a
    pipeline folds into the next step's first program); queued GPU time per
    step (events around 200 back-to-back steps), interleaved rounds.  The
    phases signal and await this process's own flags (always satisfied)."""
    c = 1 << 18
    dev = torch.cuda.current_device()
    bufs = [torch.empty(c, device="cuda") for _ in range(12)]
    for k, t in enumerate(bufs):
        hiccl_amd.fill_uniform(t, SEED, k)
    outs = [torch.empty(c, device="cuda") for _ in range(5)]
    comp = hiccl_amd.Compute(torch.float32, device=dev)
    for j in range(4):
        comp.add([bufs[2 * j], bufs[2 * j + 1]], outs[j], c, compid=0)
    comp.add(bufs[8:12], outs[4], c, compid=0)
    src = [torch.empty(c, device="cuda") for _ in range(5)]
    dst = [torch.empty(c, device="cuda") for _ in range(5)]
    cp = hiccl_amd.Compute(torch.uint8, device=dev)
    for a, b in zip(src, dst):
        cp.add([a.view(torch.uint8)], b.view(torch.uint8), c * 4, compid=0)
    flags = torch.zeros(16, dtype=torch.int32, device="cuda")
    f = [flags.data_ptr() + 4 * i for i in range(3)]
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    st = ctypes.c_void_p(stream.cuda_stream)
    lib = L.lib()
    epoch = [0]

    def phase(flag, e):
        tab = (ctypes.c_void_p * 1)(flag)
        L.check(lib.hiccl_signal_wait(tab, 1, tab, 1, e, ctypes.c_void_p(err.data_ptr()), 10.0, st), "signal_wait")

    def separate():
        epoch[0] += 1
        phase(f[0], epoch[0])
        cp.enqueue(stream)
        phase(f[1], epoch[0])
        comp.enqueue(stream)
        phase(f[2], epoch[0])

    def build(phase_flag, plan):
        pr = hiccl_amd.Program(torch.float32, device=dev)
        if phase_flag is not None:
            pr.add_signal([phase_flag], [phase_flag])
        if plan is not None:
            pr.add_plan(plan)
        return pr

    p_copy, p_comp, p_tail = build(f[0], cp), build(f[1], comp), build(f[2], None)

    def program():
        epoch[0] += 1
        for pr in (p_copy, p_comp, p_tail):
            pr.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)

    def program_tail_folded():  # the tail phase rides in the next step's first program, as in a pipeline
        epoch[0] += 1
        p_copy.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)
        p_comp.launch([epoch[0]], err=err.data_ptr(), timeout_s=10.0, stream=stream)

    def tokens(mode, fn):  # run fn with the token protocol `mode` (HICCL_PROG_FENCES, read at each launch)
        def run():
            os.environ["HICCL_PROG_FENCES"] = mode
            try:
                fn()
            finally:
                os.environ.pop("HICCL_PROG_FENCES", None)
        return run

    def separate_nophase():
        cp.enqueue(stream)
        comp.enqueue(stream)

    q_copy, q_comp = build(None, cp), build(None, comp)

    def program_nophase():
        q_copy.launch(stream=stream)
        q_comp.launch(stream=stream)

    # unsuffixed: the library's default token protocol (fenced); _light:
    # HICCL_PROG_FENCES=light
    runs = {"separate": separate, "separate_light": tokens("light", separate), "program": program,
            "program_tail_folded": program_tail_folded,
            "program_tail_folded_light": tokens("light", program_tail_folded),
            "separate_no_phases": separate_nophase, "program_no_phases": program_nophase}
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(time_queued(fn, 200, 10) * 1e3)
    # The same steps captured into one hipGraph of 200 steps and replayed, as
    # HICCL_GRAPH=1 runs a pipeline: every phase's epoch is e + *ctr, ctr
    # bumped by the graph's first node (a kernel boundary between graph
    # nodes costs less than between eager launches: bench --stepscale).
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    cptr = ctypes.c_void_p(ctr.data_ptr())
    erp = ctypes.c_void_p(err.data_ptr())

    def phase_dev(flag, e, s_):
        tab = (ctypes.c_void_p * 1)(flag)
        L.check(lib.hiccl_signal_wait_dev(tab, 1, tab, 1, e, cptr, erp, 10.0, s_), "signal_wait_dev")

    side = torch.cuda.Stream()
    graphs = {}
    for name in ("separate_graph", "separate_light_graph", "program_tail_folded_graph",
                 "program_tail_folded_light_graph", "separate_no_phases_graph", "program_no_phases_graph"):
        if "_light" in name:
            os.environ["HICCL_PROG_FENCES"] = "light"  # read at each launch: the capture keeps it
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            cs = torch.cuda.current_stream()
            s_ = ctypes.c_void_p(cs.cuda_stream)
            with torch.cuda.graph(g, stream=cs):
                L.check(lib.hiccl_counter_add(cptr, 1, s_), "counter_add")
                for i in range(200):
                    e = 1000 + i
                    if name in ("separate_graph", "separate_light_graph"):
                        phase_dev(f[0], e, s_)
                        cp.enqueue(cs)
                        phase_dev(f[1], e, s_)
                        comp.enqueue(cs)
                        phase_dev(f[2], e, s_)
                    elif name in ("program_tail_folded_graph", "program_tail_folded_light_graph"):
                        p_copy.launch([e], epoch_dev=ctr.data_ptr(), err=err.data_ptr(), timeout_s=10.0, stream=cs)
                        p_comp.launch([e], epoch_dev=ctr.data_ptr(), err=err.data_ptr(), timeout_s=10.0, stream=cs)
                    elif name == "separate_no_phases_graph":
                        cp.enqueue(cs)
                        comp.enqueue(cs)
                    else:
                        q_copy.launch(stream=cs)
                        q_comp.launch(stream=cs)
        graphs[name] = g
        os.environ.pop("HICCL_PROG_FENCES", None)
    for name, g in graphs.items():
        v = []
        for _ in range(5):
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            v.append(a.elapsed_time(b) * 1e3 / 200)
        res[name] = v
    del graphs
    ref = torch.empty(c, device="cuda")
    ok = True
    for j in range(4):
        hiccl_amd.reduce(ref, [bufs[2 * j], bufs[2 * j + 1]])
        ok = ok and torch.equal(ref.view(torch.int32), outs[j].view(torch.int32))
    hiccl_amd.reduce(ref, bufs[8:12])
    ok = ok and torch.equal(ref.view(torch.int32), outs[4].view(torch.int32))
    ok = ok and all(torch.equal(a.view(torch.int32), b.view(torch.int32)) for a, b in zip(src, dst))
    torch.cuda.synchronize()
    mib = 1 << 20
    alg = (12 + 5) * mib + (5 + 5) * mib  # reductions: 12 MiB read + 5 written; copies: 5 MiB read + 5 written
    row = {"mode": "progstep", "err": int(err.item()), "bits_ok": bool(ok), "algorithmic_bytes": alg,
           "default_tokens": "fenced" if lib.hiccl_token_mode() == L.HICCL_TOKENS_FENCED else "light"}
    for k, v in res.items():
        row[k + "_us"] = round(float(np.median(v)), 3)
    row["saved_us_per_step"] = round(row["separate_us"] - row["program_us"], 3)
    print(json.dumps(row), flush=True)
    for pr in (p_copy, p_comp, p_tail, q_copy, q_comp):
        pr.close()
    return 0


def stepscale(args):
    """The C5 step's batched reduction (4 computes of n = 2 and one of n = 4,
    2^18 f32 each at scale 1) at scales 1/8 ... 16, one
    plan launch each, queued GPU time per launch (events around 200
    back-to-back launches), interleaved rounds.  A least-squares fit
    t = t0 + bytes / rate over the scales splits a launch into a fixed part
    (dispatch, first-byte latency, drain) and a bandwidth part; at scale 1
    it says how far the step kernel is from its HBM roofline and why."""
    scales = (0.125, 0.25, 0.5, 1, 2, 4, 8, 16)
    base = 1 << 18
    dev = torch.cuda.current_device()
    cases = {}
    keep = []
    for f in scales:
        c = int(base * f)
        bufs = [torch.empty(c, device="cuda") for _ in range(12)]
        for k, t in enumerate(bufs):
            hiccl_amd.fill_uniform(t, SEED, k)
        outs = [torch.empty(c, device="cuda") for _ in range(5)]
        comp = hiccl_amd.Compute(torch.float32, device=dev)
        for j in range(4):
            comp.add([bufs[2 * j], bufs[2 * j + 1]], outs[j], c, compid=0)
        comp.add(bufs[8:12], outs[4], c, compid=0)
        keep.append((bufs, outs))
        cases[f] = (comp, 17 * c * 4)  # 12 inputs read + 5 outputs written
    stream = torch.cuda.current_stream()
    res = {f: [] for f in scales}
    for _ in range(5):
        for f in scales:
            comp = cases[f][0]
            res[f].append(time_queued(lambda: comp.enqueue(stream), 200, 10) * 1e3)
    xs = np.array([cases[f][1] for f in scales], dtype=np.float64)
    ys = np.array([float(np.median(res[f])) for f in scales])  # us
    A = np.vstack([np.ones_like(xs), xs]).T
    (t0, slope), *_ = np.linalg.lstsq(A, ys, rcond=None)
    rate_GBps = (1.0 / slope) * 1e6 / 1e9  # slope: us per byte
    rows = [{"scale": f, "algorithmic_bytes": int(cases[f][1]), "queued_us": round(float(y), 3),
             "GBps": round(cases[f][1] / y * 1e6 / 1e9, 1), "fit_us": round(float(t0 + slope * cases[f][1]), 3),
             "engine": cases[f][0].engine()}
            for f, y in zip(scales, ys)]
    # the same launches with the engine / occupancy pinned (what AUTO chose
    # against the alternatives, per scale)
    variants = {"tile": dict(engine=1), "tile_bpc2": dict(engine=1, blocks_per_cu=2),
                "tile_bpc4": dict(engine=1, blocks_per_cu=4), "phase": dict(engine=2)}
    for name, cfg in variants.items():
        vt = {f: [] for f in scales}
        for _ in range(3):
            for f in scales:
                comp = cases[f][0]
                comp.set_config(cfg)
                vt[f].append(time_queued(lambda: comp.enqueue(stream), 200, 10) * 1e3)
        for r, f in zip(rows, scales):
            r[name + "_us"] = round(float(np.median(vt[f])), 3)
    for f in scales:
        cases[f][0].set_config({})
    ok = True
    for f in scales:
        bufs, outs = keep[scales.index(f)]
        ref = torch.empty_like(outs[0])
        hiccl_amd.reduce(ref, [bufs[0], bufs[1]])
        ok = ok and torch.equal(ref.view(torch.int32), outs[0].view(torch.int32))
    torch.cuda.synchronize()
    # the kernel boundary alone: one 64-lane wave per launch (hiccl_counter_add),
    # back to back on the same stream
    ctr = torch.zeros(1, dtype=torch.int32, device="cuda")
    lib = L.lib()
    st = ctypes.c_void_p(stream.cuda_stream)
    empty = [time_queued(lambda: lib.hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1, st), 200, 10) * 1e3
             for _ in range(5)]
    # the same 200 launches, and 200 C5-step plan launches (scale 1, static
    # schedule inside a capture), as ONE hipGraph replay: the boundary
    # between graph nodes
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    comp1 = cases[1][0]
    comp1.enqueue(stream)  # re-uploads after the variants' set_config (an upload cannot be captured)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        cs = torch.cuda.current_stream()
        with torch.cuda.graph(g1, stream=cs):
            for _ in range(200):
                lib.hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1, ctypes.c_void_p(cs.cuda_stream))
        with torch.cuda.graph(g2, stream=cs):
            for _ in range(200):
                comp1.enqueue(cs)
    graph_us = {}
    for name, g in (("one_wave_kernel_graph_us", g1), ("scale1_graph_us", g2)):
        v = []
        for _ in range(5):
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            v.append(a.elapsed_time(b) * 1e3 / 200)
        graph_us[name] = round(float(np.median(v)), 3)
    del g1, g2
    one = rows[scales.index(1)]
    print(json.dumps({"mode": "stepscale", "shape": "4 x (n=2) + 1 x (n=4) computes of scale x 2^18 f32, one plan launch",
                      "rows": rows, "fit_fixed_us": round(float(t0), 3), "fit_rate_GBps": round(rate_GBps, 1),
                      "scale1_fixed_share": round(float(t0) / one["queued_us"], 3),
                      "scale1_frac_of_8TBps": round(one["GBps"] / 8000.0, 3),
                      "one_wave_kernel_us": round(float(np.median(empty)), 3), **graph_us,
                      "bits_ok": bool(ok)}), flush=True)
    for comp, _ in cases.values():
        comp.close()
    return 0


def c2_misaligned(n, count, steps, warmup):
    """SURVEY.md 8d's second C2 run, as an interleaved A/B on ONE set of
    allocations: input k is read either from its 16-B-aligned base or from
    1 + k mod 3 elements past it (the mutual misalignment partition()
    produces, reduce.h:401-415), output aligned; launches alternate between
    the two views so placement and box state are common to both.  A sampled
    bitwise check of each view's output against the oracle generator."""
    offs = [1 + k % 3 for k in range(n)]
    bases = [torch.empty(count + 4, dtype=torch.float32, device="cuda") for _ in range(n)]
    for k, b in enumerate(bases):  # element j of base k = generator(k, j), shifted views included
        hiccl_amd.fill_uniform(b, SEED, k)
    aligned = [b[:count] for b in bases]
    shifted = [b[o:o + count] for b, o in zip(bases, offs)]
    out = torch.empty(count, dtype=torch.float32, device="cuda")
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
           "parity_sample_ok": parity}
    del bases, aligned, shifted, out
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


def c2variants(args):
    """Config 2 variants: the README's count 1e9/sizeof(T)
    = 2.5e8 (tail handling), and the 2^28 bucket with every input shifted by
    1-3 elements and the output by 0 or 1 (the mutual misalignment partition()
    produces)."""
    n = 8
    cases = [("readme_count", 250_000_000, [0] * n, 0),
             ("inputs_shifted", 1 << 28, [1 + k % 3 for k in range(n)], 0),
             ("inputs_and_output_shifted", 1 << 28, [1 + k % 3 for k in range(n)], 1),
             ("inputs_common_shift", 1 << 28, [1] * n, 0),
             ("output_shifted", 1 << 28, [0] * n, 1)]
    for name, count, in_off, out_off in cases:
        bases = [torch.empty(count + 4, dtype=torch.float32, device="cuda") for _ in range(n)]
        ins = [b[o:o + count] for b, o in zip(bases, in_off)]
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, SEED, k)
        obase = torch.empty(count + 4, dtype=torch.float32, device="cuda")
        out = obase[out_off:out_off + count]
        torch.cuda.synchronize()
        out.fill_(float("nan"))
        _, ms = time_launches(lambda: hiccl_amd.reduce(out, ins), args.steps, args.warmup)
        t = float(np.median(ms)) * 1e-3
        b = (n + 1) * count * 4
        print(json.dumps({"config": "C2", "variant": name, "count": count, "input_offsets": in_off,
                          "output_offset": out_off, "parity_sample_ok": sample_check(out, n, count),
                          "kernel_ms": round(t * 1e3, 4), "GBps": round(b / t / 1e9, 1),
                          "frac_hbm": round(b / t / 1e9 / HBM_PEAK_GBPS, 4)}), flush=True)
        del bases, ins, obase, out
        torch.cuda.empty_cache()
    return 0


def chunks(args):
    """Config 4: fp32/bf16, 16 MiB..4 GiB per input, split into 1 MiB computes
    (pipedepth = bytes / 1 MiB, reduce.h:406 split), batched plan launch vs
    one launch per compute (the reference structure, compute.h:88-91)."""
    n = 8
    for dtype in (torch.float32, torch.bfloat16):
        esz = torch.tensor([], dtype=dtype).element_size()
        for mib in (16, 64, 256, 1024, 4096):
            count = (mib << 20) // esz
            free, _ = torch.cuda.mem_get_info()
            if (n + 1) * count * esz * 1.05 > free:
                log(f"chunks: skip {mib} MiB ({dtype}): not enough memory")
                continue
            ins, out = make_bucket(n, count, dtype)
            depth = max(1, (mib << 20) // (1 << 20))
            comp = hiccl_amd.Compute(dtype, device=torch.cuda.current_device(), engine=args.engine)
            off = 0
            for b in range(depth):  # partition(): count/numbatch + (b < count%numbatch)
                c = count // depth + (1 if b < count % depth else 0)
                comp.add([(t, off) for t in ins], (out, off), c, compid=0)
                off += c
            stream = torch.cuda.current_stream()
            res, queued = {}, {}
            for mode in ("batched", "each"):
                launch = (lambda m=mode: comp.start(stream=stream, each=(m == "each")))
                _, ms = time_launches(launch, args.steps, args.warmup)
                res[mode] = float(np.median(ms)) * 1e-3
                queued[mode] = time_queued(launch, max(args.steps, 20), 2) * 1e-3
            b = (n + 1) * count * esz
            ok = sample_check(out, n, count, bf16=(dtype == torch.bfloat16))
            print(json.dumps({"config": "C4", "dtype": str(dtype).split(".")[-1], "mib_per_input": mib,
                              "parity_sample_ok": ok, "engine": comp.engine(),
                              "computes": depth, "batched_ms": round(res["batched"] * 1e3, 4),
                              "batched_GBps": round(b / res["batched"] / 1e9, 1),
                              "each_ms": round(res["each"] * 1e3, 4),
                              "each_GBps": round(b / res["each"] / 1e9, 1),
                              "queued_batched_GBps": round(b / queued["batched"] / 1e9, 1),
                              "queued_each_GBps": round(b / queued["each"] / 1e9, 1)}), flush=True)
            comp.close()
            del ins, out
            torch.cuda.empty_cache()
    return 0


def host_sum(host_in):
    """In-order fp32 sum on the host (torch adds two tensors element-wise in
    fp32 with round-to-nearest: the reference's acc += in[k][i] order)."""
    exp = torch.zeros_like(host_in[0])
    for h in host_in:
        exp = exp + h
    return exp


def roundtrip(args):
    """Inputs and output in pinned host memory: H2D of N inputs + kernel + D2H
    (serial, and chunk-pipelined over 3 streams)."""
    n, count = args.n, 1 << args.log2count
    host_in = [torch.empty(count, dtype=torch.float32).pin_memory() for _ in range(n)]
    for k, h in enumerate(host_in):
        h.copy_(torch.from_numpy(np.random.default_rng(k).uniform(-1, 1, count).astype(np.float32)))
    host_out = torch.empty(count, dtype=torch.float32).pin_memory()
    dev_in = [torch.empty(count, device="cuda") for _ in range(n)]
    dev_out = torch.empty(count, device="cuda")

    def serial():
        for h, d in zip(host_in, dev_in):
            d.copy_(h, non_blocking=True)
        hiccl_amd.reduce(dev_out, dev_in)
        host_out.copy_(dev_out, non_blocking=True)

    nchunk = 16
    streams = [torch.cuda.Stream() for _ in range(3)]
    csz = count // nchunk

    def pipelined():
        cur = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(cur)
        for c in range(nchunk):
            s = streams[c % 3]
            lo = c * csz
            hi = count if c == nchunk - 1 else lo + csz
            with torch.cuda.stream(s):
                for h, d in zip(host_in, dev_in):
                    d[lo:hi].copy_(h[lo:hi], non_blocking=True)
                hiccl_amd.reduce(dev_out[lo:], [d[lo:] for d in dev_in], count=hi - lo, stream=s)
                host_out[lo:hi].copy_(dev_out[lo:hi], non_blocking=True)
        for s in streams:
            cur.wait_stream(s)

    pipes = {f"host_pipe_{mib}MiB_d{d}": hiccl_amd.HostPipe(torch.float32, chunk_bytes=mib << 20, depth=d)
             for mib, d in ((64, 3), (32, 4), (128, 2))}
    legs = [("serial", serial), ("pipelined", pipelined)]
    expect = host_sum(host_in)
    legs += [(k, (lambda p=p: p.reduce(host_out, host_in))) for k, p in pipes.items()]
    out = {}
    for name, fn in legs:
        host_out.zero_()
        wall, _ = time_launches(fn, 5, 2)
        t = wall / 5
        out[name] = {"s": round(t, 4), "GBps_alg": round((n + 1) * count * 4 / t / 1e9, 2)}
        if name.startswith("host_pipe"):
            out[name]["parity_ok"] = bool(torch.equal(host_out.view(torch.int32), expect.view(torch.int32)))
    for p in pipes.values():
        p.close()
    # device-only reference, and the link alone: the n inputs H2D, the output D2H
    _, ms = time_launches(lambda: hiccl_amd.reduce(dev_out, dev_in), 10, 3)
    out["kernel_only_GBps"] = round((n + 1) * count * 4 / (np.median(ms) * 1e-3) / 1e9, 1)
    wall, _ = time_launches(lambda: [d.copy_(h, non_blocking=True) for h, d in zip(host_in, dev_in)], 3, 1)
    out["h2d_only_GBps"] = round(n * count * 4 * 3 / wall / 1e9, 2)
    wall, _ = time_launches(lambda: host_out.copy_(dev_out, non_blocking=True), 3, 1)
    out["d2h_only_GBps"] = round(count * 4 * 3 / wall / 1e9, 2)
    pipelined()
    torch.cuda.synchronize()
    exp = expect
    out["parity_ok"] = bool(torch.equal(exp.view(torch.int32), host_out.view(torch.int32)))
    print(json.dumps({"mode": "roundtrip", "n": n, "count": count, **out,
                      "pcie_bytes": (n + 1) * count * 4}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
