"""CPU tier: bench.py's multi-rank control plane (world_size 2, gloo).

With one process per GPU the driver launches bench.py under
torch.distributed.run; only the barrier and the max-over-ranks wall time
cross ranks (replicas, no data-path collective).  Here two CPU processes
run the same Dist object over gloo: the barrier completes, the max is the
slowest rank's time, and the whole-job rate is world x bytes / that time.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp
from conftest import make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    d = bench.Dist(world)
    d.barrier()
    wall = 1.0 + rank  # rank 1 is the slow one
    wmax = d.max(wall)
    q.put((rank, d.backend, d.world, wmax, bench.whole_job_gbps(d.world, 9 << 30, 10, wmax)))
    d.close()


def test_two_rank_gloo_control_plane():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, backend, w, wmax, gbps in res:
        assert backend == "gloo" and w == world
        assert wmax == 2.0  # the slowest rank's time
        assert gbps == pytest.approx(2 * (9 << 30) * 10 / 2.0 / 1e9)


def test_single_rank_no_launcher():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.whole_job_gbps(1, 9 << 30, 20, 0.0344) == pytest.approx(9 * 2**30 * 20 / 0.0344 / 1e9)


def _c5_rank(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import argparse

    import bench
    # the config-5 leg runs before Dist (no GPU touched); on a box without one
    # GPU per rank it is skipped, and every rank receives rank 0's verdict
    res = bench.c5_leg(argparse.Namespace(c5_log2count=10, c5_iters=1))
    d = bench.Dist(world)  # reuses the control plane the leg started
    d.barrier()
    q.put((rank, res, d.backend))
    d.close()


def test_c5_leg_broadcasts_rank0_result():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c5_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1]
    assert "skipped" in res[0][1] and "one GPU per rank" in res[0][1]["skipped"]
    assert all(r[2] == "gloo" for r in res)


def test_cpu_leg_full_bucket_parity(tmp_path):
    """bench.py's CPU baseline child: times the reference's reduce_kernel and
    compares a GPU output file word for word (here: the oracle's own output,
    then the same with one word flipped)."""
    import json
    import subprocess

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import Oracle, _build_oracle
    _build_oracle()
    ora = Oracle()
    n, log2c = 3, 16
    exp = ora.reduce(list(ora.fill(n, 1 << log2c, 1234)))
    good = tmp_path / "good.f32"
    exp.tofile(good)
    bad = exp.copy()
    bad.view(np.uint32)[777] ^= 1
    badf = tmp_path / "bad.f32"
    bad.tofile(badf)
    env = dict(os.environ, OMP_NUM_THREADS="2", OMP_PROC_BIND="spread")
    for path, ok, mism in ((good, True, 0), (badf, False, 1)):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-leg", "--n", str(n),
                            "--log2count", str(log2c), "--cpu-budget", "0.2", "--expect-file", str(path)],
                           capture_output=True, text=True, env=env, timeout=300)
        assert p.returncode == 0, p.stderr[-2000:]
        r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
        assert r["parity_full"]["ok"] is ok and r["parity_full"]["mismatches"] == mism
        assert r["threads"] == 2 and "OMP_PROC_BIND=spread" in r["sample"]
        # the spread over the passes: min <= median (value) <= max, one time per pass
        assert r["min"] <= r["value"] <= r["max"] and r["passes"] == len(r["pass_ms"]) >= 1


def test_serial_rw_model():
    """roofline.serial_rw_model: R / read_rate + W / write_rate, the write
    rate recovered from the copy probe (X read + X written)."""
    sys.path.insert(0, ROOT)
    import bench
    read, write = 7000.0, 4500.0
    copy = 2.0 / (1.0 / read + 1.0 / write)  # what a copy probe would measure
    r, w = 8 * 2**30, 2**30
    t = r / read / 1e9 + w / write / 1e9
    m = bench.serial_rw_model(r, w, read, copy, t)
    assert abs(m["write_GBps_from_copy"] - write) < 0.1
    assert abs(m["predicted_ms"] - t * 1e3) < 1e-3 and abs(m["frac"] - 1.0) < 1e-3
    assert bench.serial_rw_model(r, w, None, copy, t) is None
    assert bench.serial_rw_model(r, w, read, 2 * read, t) is None  # copy faster than reads: no model


def test_c5_child_env_drops_device_masks(monkeypatch):
    """The config-5 MPI job picks each rank's GPU by local rank: a device mask
    inherited from the torchrun rank (one GPU visible per process) would put
    every MPI rank on that one GPU.  run_c5 drops the masks from the job's
    environment, counts GPUs without them, and records what it dropped --
    here (no GPU) in the skip record."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench
    env = {"HIP_VISIBLE_DEVICES": "3", "ROCR_VISIBLE_DEVICES": "0", "CUDA_VISIBLE_DEVICES": "1", "KEEP": "x"}
    child, dropped = bench.c5_child_env(env)
    assert child == {"KEEP": "x"}
    assert dropped == {"HIP_VISIBLE_DEVICES": "3", "ROCR_VISIBLE_DEVICES": "0", "CUDA_VISIBLE_DEVICES": "1"}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    res = bench.run_c5(2, argparse.Namespace(c5_log2count=10, c5_iters=1))
    assert res["env_scrubbed"] == {"HIP_VISIBLE_DEVICES": "5"}
    assert res["devices_counted_unmasked"] == 0 and "one GPU per rank" in res["skipped"]


def test_c5_driver_json_records_devices_and_mode(tmp_path):
    """The C5 driver's JSON (HICCL_DRIVER_JSON; the same writer in the HIP
    build bench.py runs) carries every rank's visible device count, device,
    PCI bus id and the execution mode actually used, and parses as JSON --
    exercised here on the host port (2 MPI ranks, no GPU)."""
    import json
    import shutil
    import subprocess
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    if not os.path.exists(mpirun):
        pytest.skip("no mpirun")
    make(ROOT, "build/collectives_host_f32")
    path = tmp_path / "c5.json"
    env = dict(os.environ, OMP_NUM_THREADS="1", HICCL_DRIVER_JSON=str(path))
    p = subprocess.run([mpirun, "-np", "2", os.path.join(ROOT, "build", "collectives_host_f32"), "8", "4096", "1", "1",
                        "4", "1", "2", "2", "mpi"], capture_output=True, text=True, env=env, timeout=240, cwd="/tmp")
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    r = json.loads(path.read_text())
    assert r["kat"] == "PASSED" and r["ranks"] == 2
    assert r["devices_seen"] == [0, 0] and r["rank_devices"] == [-1, -1]
    assert r["bus_ids"] == ["host", "host"]
    assert r["mode_used"] == "host-driven"
    # the per-step host wall split, in comm.h:195-204's order (host-driven:
    # transport start / wait, compute launch / wait; the stream-ordered
    # parts stay 0 here), MAX over ranks
    hs = r["host_split_us_per_step"]
    assert hs["steps"] >= 4 and hs["runs"] == 1 and hs["over_ranks"] == "max"
    for k in ("transport_start", "transport_wait", "compute_launch", "compute_wait", "finish"):
        assert hs[k] >= 0.0, k
    assert hs["transport_wait"] + hs["compute_wait"] > 0.0
    assert hs["enqueue"] == 0.0 and hs["sync"] == 0.0


def test_c5_protocol_ab_summary():
    """protocol_ab: each program / light-token twin's median collective time
    over the default protocol's (stream_graph_fused_noprog), with its KAT and
    mode_used; a mode that did not run gives None, never a ratio."""
    sys.path.insert(0, ROOT)
    import bench
    out = {"stream_graph_fused_noprog": {"collective_ms_median": 2.0, "kat": "PASSED"},
           "stream_graph_fused_fenced": {"collective_ms_median": 1.5, "kat": "PASSED",
                                         "mode_used": "stream-ordered+graph+fused+program+tokens-fenced"},
           "stream_graph_fused": {"skipped": "time budget of the config-5 leg spent"}}
    ab = bench.c5_protocol_ab(out)
    assert ab["baseline_ms"] == 2.0 and ab["baseline_kat"] == "PASSED"
    assert ab["stream_graph_fused_fenced"]["over_baseline"] == 0.75
    assert ab["stream_graph_fused_fenced"]["mode_used"].endswith("tokens-fenced")
    assert ab["stream_graph_fused"]["ms"] is None and ab["stream_graph_fused"]["over_baseline"] is None
    assert bench.c5_protocol_ab({})["stream_graph_fused"]["over_baseline"] is None


STUB_MPIRUN = r'''
import json, os, sys
# a stand-in for mpirun: behaviour per call from STUB_PLAN (a comma list),
# the call number kept in STUB_COUNTER
ctr = os.environ["STUB_COUNTER"]
k = int(open(ctr).read()) if os.path.exists(ctr) else 0
open(ctr, "w").write(str(k + 1))
plan = os.environ["STUB_PLAN"].split(",")
what = plan[k] if k < len(plan) else "ok"
env_seen = {key: os.environ.get(key) for key in ("HICCL_STREAM_ORDERED", "GPU_MAX_HW_QUEUES", "HICCL_STEP_PROGRAM")}
if what in ("ok", "katfail"):
    with open(os.environ["HICCL_DRIVER_JSON"], "w") as f:
        json.dump({"kat": "PASSED" if what == "ok" else "FAILED", "collective_ms_median": 2.0 + k,
                   "mode_used": "stub", "env_seen": env_seen, "argv": sys.argv[1:]}, f)
    sys.exit(0 if what == "ok" else 1)
sys.exit({"killed": 124, "sigkill": 137, "crash": 139}[what])
'''


def _stub_leg(tmp_path, monkeypatch, plan):
    import argparse
    sys.path.insert(0, ROOT)
    import bench
    stub = tmp_path / "mpirun"
    stub.write_text(f"#!{sys.executable}\n" + STUB_MPIRUN)
    stub.chmod(0o755)
    exe = tmp_path / "collectives_stub"
    exe.write_text("")
    monkeypatch.setattr(bench, "C5_MPIRUN", str(stub))
    monkeypatch.setattr(bench, "C5_EXE", str(exe))
    monkeypatch.setattr(bench, "visible_gpus", lambda env: 0)
    monkeypatch.setenv("STUB_PLAN", ",".join(plan))
    monkeypatch.setenv("STUB_COUNTER", str(tmp_path / "ctr"))
    return bench, argparse.Namespace(c5_log2count=10, c5_iters=1)


def test_c5_leg_failed_kat_lets_next_mode_run(tmp_path, monkeypatch):
    """A mode whose MPI job exits 1 (its known-answer check failed, or its
    own signal time-out) leaves the GPUs usable: the leg records it and runs
    the next mode (bench.run_c5; stub launcher in place of mpirun)."""
    bench, args = _stub_leg(tmp_path, monkeypatch, ["ok", "katfail", "ok", "ok", "ok", "ok", "ok"])
    res = bench.run_c5(4, args, allow_shared=True)
    assert res["host"]["kat"] == "PASSED" and res["host"]["rc"] == 0
    assert res["stream_graph"]["kat"] == "FAILED" and res["stream_graph"]["rc"] == 1
    assert res["stream_graph_fused_noprog"]["kat"] == "PASSED"
    assert "stopped_after" not in res
    assert all(res[m]["rc"] == 0 for m in ("stream_graph_fused_fenced", "flat_stream_graph_fused", "xccl",
                                          "stream_graph_fused"))
    assert res["protocol_ab"]["baseline_kat"] == "PASSED"
    # a rehearsal on a shared GPU: 2 hardware queues per rank; the stream
    # modes ask for stream-ordered mode as "1" (the library falls back)
    assert res["stream_graph"]["env_seen"] == {"HICCL_STREAM_ORDERED": "1", "GPU_MAX_HW_QUEUES": "2",
                                               "HICCL_STEP_PROGRAM": "0"}


@pytest.mark.parametrize("rc_kind", ["killed", "sigkill", "crash"])
def test_c5_leg_killed_mode_stops_the_leg(tmp_path, monkeypatch, rc_kind):
    """A mode killed at its limit (124 / 137) or crashed (139) stops the leg:
    `stopped_after` names it, nothing more starts on the GPUs, and the leg
    still returns its record (the replica headline is computed after it)."""
    bench, args = _stub_leg(tmp_path, monkeypatch, ["ok", "ok", rc_kind])
    res = bench.run_c5(8, args, allow_shared=True)
    assert res["stopped_after"] == "stream_graph_fused_noprog"
    assert res["stream_graph_fused_noprog"]["rc"] == {"killed": 124, "sigkill": 137, "crash": 139}[rc_kind]
    assert "error" in res["stream_graph_fused_noprog"]  # no JSON from a killed job
    for later in ("stream_graph_fused_fenced", "flat_stream_graph_fused", "xccl", "stream_graph_fused"):
        assert later not in res
    assert int((tmp_path / "ctr").read_text()) == 3  # no launch after the killed one
    assert res["protocol_ab"]["baseline_ms"] is None


def test_c5_leg_force_stream_rehearsal(tmp_path, monkeypatch):
    """--c5-force-stream: the stream-ordered modes ask for
    HICCL_STREAM_ORDERED=force (run stream-ordered even with ranks sharing a
    GPU); host-driven and xccl modes keep 0; refused outside a rehearsal."""
    bench, args = _stub_leg(tmp_path, monkeypatch, ["ok"] * 7)
    res = bench.run_c5(8, args, allow_shared=True, force_stream=True,
                       only=("host", "stream_graph_fused_noprog", "xccl"))
    assert res["forced_stream_ordered"] is True
    assert res["host"]["env_seen"]["HICCL_STREAM_ORDERED"] == "0"
    assert res["stream_graph_fused_noprog"]["env_seen"]["HICCL_STREAM_ORDERED"] == "force"
    assert res["xccl"]["env_seen"]["HICCL_STREAM_ORDERED"] == "0"
    assert "skipped" in bench.run_c5(8, args, allow_shared=False, force_stream=True)


def _c5_leg_raises(port, q):
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import argparse

    import bench

    def boom(*a, **k):
        raise RuntimeError("stub failure")
    bench.run_c5 = boom
    res = bench.c5_leg(argparse.Namespace(c5_log2count=10, c5_iters=1))
    d = bench.Dist(1)
    q.put(res)
    d.close()


def test_c5_leg_error_never_costs_the_headline():
    """An exception inside the config-5 leg becomes a `skipped` record; the
    control plane survives for the replica measurement that follows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_c5_leg_raises, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res == {"skipped": "error: stub failure"}


def test_cpu_placement_one_thread_per_l3_first():
    """The CPU baseline's explicit OMP_PLACES: `l3spread` takes one core per
    L3 domain (CCD) across every NUMA node before a second core of any;
    `node` does the same inside the node holding the most cores."""
    sys.path.insert(0, ROOT)
    import bench
    # 2 nodes x 2 CCDs x 4 cores, CPU c on CCD c // 4, node c // 8
    cores = [{"cpu": c, "pkg": str(c // 8), "node": c // 8, "l3": str(c // 4)} for c in range(16)]
    assert bench.cpu_placement(cores, 4, "l3spread") == [0, 4, 8, 12]
    assert bench.cpu_placement(cores, 6, "l3spread") == [0, 4, 8, 12, 1, 5]
    assert bench.cpu_placement(cores, 4, "node") == [0, 4, 1, 5]
    assert bench.cpu_placement(cores, 99, "l3spread") == sorted(range(16), key=lambda c: (c % 4, c // 4))


def test_cpu_spread_cause_names_what_the_leg_saw():
    """cpu_baseline's spread_cause: quota throttling when it covers most of
    the slow passes' excess; otherwise, with local pages, no migration and
    an idle host, bandwidth taken outside the container, in runs of passes."""
    sys.path.insert(0, ROOT)
    import bench
    loc = {"local_frac": 1.0}
    t = [0.022] * 10 + [0.060] * 5 + [0.022] * 5
    r = bench.spread_cause(t, [0.0] * 20, [0.1] * 20, loc, loc, {}, 16)
    assert r["slow_passes"] == 5 and r["slow_runs"] == 1 and r["cause"].startswith("host memory bandwidth")
    r = bench.spread_cause(t, [0.0] * 10 + [38.0] * 5 + [0.0] * 5, [0.1] * 20, loc, loc, {}, 16)
    assert r["cause"] == "cgroup CPU quota throttling" and r["throttle_covers_frac"] == 1.0
    r = bench.spread_cause(t, None, [0.1] * 20, {"local_frac": 0.5}, loc, {}, 16)
    assert r["cause"].startswith("unnamed") and r["pages_local"] is False


def test_driver_line_stays_compact():
    """bench.py's stdout line carries every contract field and the summaries,
    and stays a few KB even with a full CPU-baseline record and seven
    config-5 modes (the driver keeps a tail of stdout; the full record goes
    to stderr)."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    mode = {"kat": "PASSED", "rc": 0, "collective_ms_median": 31.5, "algorithmic_GBps_median": 34.1,
            "kernel_us_per_step_rank0": 4.1, "mode_used": "stream-ordered+graph+fused+tokens-fenced",
            "host_split_us_per_step": {k: 1.0 for k in "abcdefg"}, "bus_ids": ["0000:05:00.0"] * 8,
            "devices_seen": [8] * 8, "rank_devices": list(range(8)), "pipedepth": 128, "wall_s": 9.1}
    c5 = {"workload": "C5 ...", "env_scrubbed": {}, "devices_counted_unmasked": 8,
          **{k: dict(mode) for k in ("host", "stream_graph", "stream_graph_fused_noprog", "stream_graph_fused_fenced",
                                     "flat_stream_graph_fused", "xccl", "stream_graph_fused")}}
    c5["xccl"] = {"error": "rc 124: " + "x" * 600, "rc": 124, "wall_s": 120.0}
    c5["stopped_after"] = "xccl"
    c5["protocol_ab"] = bench.c5_protocol_ab(c5)
    cpu = {"value": 400.0, "unit": "GB/s", "cores": 16, "kind": "reference", "min": 150.0, "max": 440.0,
           "max_over_min": 2.9, "passes": 50, "pass_ms": [22.123] * 50, "throttled_ms": [0.0] * 50,
           "host_busy_frac": [0.123] * 50, "thread_cpus": list(range(16)), "sample": "s" * 300,
           "placement": {"policy": "l3spread", "cpus": list(range(16)), "numa_nodes": [0, 1], "l3_domains": 16},
           "throttle": {"nr_periods": 10, "nr_throttled": 0, "throttled_usec": 0},
           "spread_cause": {"cause": "host memory bandwidth ...", "slow_passes": 20, "slow_runs": 3,
                            "throttle_covers_frac": 0.0, "pages_local": True, "pages_migrated": 0,
                            "host_busy_others_median": 0.05}}
    line = {"metric": bench.METRIC, "value": 6500.0, "unit": "GB/s", "n_gpus": 8, "steps": 20, "warmup": 5,
            "ms_per_step": 1.48, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic", "config": {"workload": "C2 ..."},
            "roofline": {"bound": "hbm", "achieved": 6530.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.816,
                         "traffic": 9.66e9, "serial_rw_model": {"frac": 0.98, "frac_write_probe": 0.95},
                         "traffic_from_profile": {"file": "profiles/r05b_pmc.json", "box_kernel_ms": 1.4449,
                                                  "fits_this_run": True, "over_algorithmic": 1.00024},
                         "traffic_source": "x" * 200},
            "cpu_baseline": cpu, "parity_full": {"ok": True, "mismatches": 0, "words": 1 << 28, "against": "y" * 100},
            "device_props": {"gcn_arch": "gfx950", "cus": 256, "mem_clock_khz": 2000000},
            "c2_misaligned": {"shifted_over_aligned": 1.007, "shifted_frac": 0.78, "shifted_over_headline": 1.09,
                              "aligned_over_headline": 1.08,
                              "parity_sample_ok": {"aligned": True, "shifted": True}},
            "c2_layout_ab": {"ab": "x" * 80, "bucket_stride_bytes": 1073807360, "bucket_kernel_ms_mean": 1.44,
                             "separate_kernel_ms_mean": 1.52, "separate_over_bucket": 1.0556,
                             "separate_over_headline": 1.05, "bucket_frac": 0.839, "separate_frac": 0.795,
                             "outputs_identical": True}, "c5": c5}
    out = bench.compact_line(line)
    text = json.dumps(out)
    assert len(text) < 3500, len(text)
    assert out["c2_layout_ab"] == {"separate_over_bucket": 1.0556, "separate_over_headline": 1.05, "bucket_frac": 0.839,
                                   "separate_frac": 0.795, "outputs_identical": True}
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert out[k] == line[k]
    r = out["roofline"]
    assert (r["bound"], r["frac"], r["traffic"], r["serial_rw_frac"]) == ("hbm", 0.816, 9.66e9, 0.95)
    c = out["cpu_baseline"]
    assert (c["value"], c["cores"], c["kind"], c["spread_cause"]["slow_runs"]) == (400.0, 16, "reference", 3)
    assert "pass_ms" not in c and out["c2_misaligned"]["parity_ok"] is True
    assert out["c2_misaligned"]["shifted_over_headline"] == 1.09 and out["c2_misaligned"]["aligned_over_headline"] == 1.08
    assert r["traffic_profile"] == {"file": "profiles/r05b_pmc.json", "kernel_ms": 1.4449, "fits_this_run": True,
                                    "x_alg": 1.00024}
    assert out["c5"]["stopped_after"] == "xccl" and out["c5"]["xccl"]["rc"] == 124
    assert out["c5"]["host"]["kat"] == "PASSED" and "host_split_us_per_step" not in out["c5"]["host"]
    assert out["c5"]["protocol_ab"]["baseline_ms"] == 31.5


def test_compact_c5_skipped_leg():
    """A leg skipped as a whole (fewer GPUs than ranks, an error) keeps its
    reason and the mask scrub drops out of the driver's line."""
    sys.path.insert(0, ROOT)
    import bench
    out = bench.compact_c5({"skipped": "2 ranks on 1 GPU(s): config 5 needs one GPU per rank",
                            "env_scrubbed": {"HIP_VISIBLE_DEVICES": "0"}, "devices_counted_unmasked": 1})
    assert out == {"skipped": "2 ranks on 1 GPU(s): config 5 needs one GPU per rank"}
    assert bench.compact_c5({"skipped": "error: boom"}) == {"skipped": "error: boom"}


C5_MODES = ("host", "stream_graph", "stream_graph_fused_noprog", "stream_graph_fused_fenced",
            "flat_stream_graph_fused", "xccl", "stream_graph_fused")
# the compact line's budget: BENCH_r05's stdout_tail held 7,344 characters
# (the 2.9 KB line, then stderr); the worst-case N = 8 line stays near half
DRIVER_TAIL_CHARS = 4000


@pytest.mark.parametrize("failing", [0, 3, 7])
def test_driver_line_keeps_every_c5_mode_at_n8(failing):
    """At N = 8 the driver's one line must let a reader tell, per config-5
    mode, whether the cross-GPU run passed, from SCALE_rNN.json alone: every
    mode's kat, mode_used and rc, the leg's stopped_after and protocol_ab --
    also when modes fail with long errors, all within the stdout tail
    (reference config collectives/main.cpp:151-155)."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    c5 = {"workload": "C5: 8 ranks {1,4,2} {MPI,IPC,IPC} 2^25 floats per rank per chunk, pipedepth 128 " + "w" * 100,
          "env_scrubbed": {"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}, "devices_counted_unmasked": 8}
    for i, m in enumerate(C5_MODES):
        bad = i >= len(C5_MODES) - failing
        r = {"kat": "FAILED" if bad else "PASSED", "rc": 1 if bad else 0,
             "collective_ms_median": 30.0 + i, "algorithmic_GBps_median": 34.1, "kernel_us_per_step_rank0": 4.1,
             "mode_used": f"stream-ordered+graph+fused+program+tokens-fenced+xccl-rccl/{m}",
             "host_split_us_per_step": {k: 1.0 for k in "abcdefgh"}, "bus_ids": ["0000:05:00.0"] * 8,
             "devices_seen": [8] * 8, "rank_devices": list(range(8)), "pipedepth": 128, "wall_s": 9.1}
        if bad:
            r["error"] = f"mode {m}: rc 1: hiccl_signal_wait: timeout after 60 s on flag 0x7f00 " + "e" * 800
        c5[m] = r
    if failing == 7:  # the last mode killed at its limit: the leg stops there
        c5["stream_graph_fused"]["rc"] = 124
        c5["stopped_after"] = "stream_graph_fused"
    c5["protocol_ab"] = bench.c5_protocol_ab(c5)
    line = {"metric": bench.METRIC, "value": 52000.0, "unit": "GB/s", "n_gpus": 8, "steps": 20, "warmup": 5,
            "ms_per_step": 1.48, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic", "config": {"workload": "C2 ..." + "c" * 150, "n_inputs": 8},
            "roofline": {"bound": "hbm", "achieved": 6530.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.816,
                         "traffic": 9.66e9, "serial_rw_model": {"frac": 0.98, "frac_write_probe": 0.95},
                         "traffic_from_profile": {"file": "profiles/r06_pmc.json", "box_kernel_ms": 1.45,
                                                  "fits_this_run": True, "over_algorithmic": 1.00024}},
            "cpu_baseline": None, "parity_full": None, "parity_sample_ok": True,
            "device_props": {"gcn_arch": "gfx950:sramecc+:xnack-", "cus": 256}, "control_plane": "gloo",
            "c2_misaligned": {"shifted_over_aligned": 1.0093, "shifted_frac": 0.7519, "shifted_over_headline": 1.0903,
                              "aligned_over_headline": 1.0796, "parity_sample_ok": {"aligned": True, "shifted": True}},
            "c2_layout_ab": {"separate_over_bucket": 1.0556, "separate_over_headline": 1.05, "bucket_frac": 0.839,
                             "separate_frac": 0.795, "outputs_identical": True},
            "c5": c5}
    out = bench.compact_line(line)
    text = json.dumps(out)
    assert len(text) < DRIVER_TAIL_CHARS, len(text)
    back = json.loads(text)["c5"]
    for i, m in enumerate(C5_MODES):
        assert back[m]["kat"] == c5[m]["kat"] and back[m]["rc"] == c5[m]["rc"], m
        assert back[m]["mode_used"] == c5[m]["mode_used"], m
        if "error" in c5[m]:
            assert back[m]["error"].startswith(f"mode {m}: rc 1: hiccl_signal_wait"), m
    assert back.get("stopped_after") == c5.get("stopped_after")
    ab = back["protocol_ab"]
    assert ab["baseline_ms"] == 32.0
    for k in ("stream_graph_fused_fenced", "stream_graph_fused"):
        assert k in ab


def test_traffic_profile_cited_fits_the_run(tmp_path, monkeypatch):
    """bench.traffic_from_profiles cites the newest PMC profile of the
    headline kernel whose rocprofv3 kernel time is at or below this run's
    kernel mean, and says when none fits."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    (tmp_path / "profiles").mkdir()
    for tag, ns in (("r05b", 1444913.0), ("r05n", 1508727.0), ("r02x_misaligned", 1400000.0)):
        d = {"tag": tag, "n_inputs": 8, "count": 1 << 28, "hbm_bytes_per_launch": 9.666e9,
             "traffic_over_algorithmic": 1.00024, "rocprof_avg_kernel_ns": ns,
             "kernel": "void k_reduce_single<OpF32, 256, 4, 11, 0>(SingleArgs)"}
        if "misaligned" in tag:
            d["variant"] = "misaligned"
        (tmp_path / "profiles" / f"{tag}_pmc.json").write_text(json.dumps(d))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    p = bench.traffic_from_profiles(8, 1 << 28, run_kernel_ms=1.4744)
    assert p["tag"] == "r05b" and p["fits_this_run"] is True and p["profiles_considered"] == 2
    p = bench.traffic_from_profiles(8, 1 << 28, run_kernel_ms=1.52)
    assert p["tag"] == "r05n" and p["fits_this_run"] is True
    p = bench.traffic_from_profiles(8, 1 << 28, run_kernel_ms=1.40)
    assert p["tag"] == "r05n" and p["fits_this_run"] is False
    assert bench.traffic_from_profiles(4, 1 << 28, run_kernel_ms=1.5) is None
