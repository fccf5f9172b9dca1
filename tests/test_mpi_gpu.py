"""GPU tier: the C++ surface end to end on the HIP port.

build/collectives_hip (hiccl_amd/csrc/collectives.cpp, default HIP port)
under MPI with every rank on the box's GPU(s): HiCCL::Comm<T> factorizes,
the transport moves device buffers (IPC put / IPC_get over HIP IPC handles,
MPI with pinned staging), and each step's computes run as ONE batched
gfx950 kernel through the C ABI.  At most 8 ranks touch the GPU.
* the reference's known-answer test for all eight collectives (size_t);
* float all-reduce: every rank's receive buffer equals oracle/schedule.py's
  simulation of the reference schedule bit for bit.
"""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import schedule as S  # noqa: E402

pytestmark = pytest.mark.gpu

MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
HIP = os.path.join(ROOT, "build", "collectives_hip")
HIP_F32 = os.path.join(ROOT, "build", "collectives_hip_f32")


def mpirun(np_, exe, args, timeout=180, streamed=True, fused=False, engine="auto", graph=False, repeat=1,
           stream_env=None, queues=True, extra_env=None):
    """streamed: HICCL_STREAM_ORDERED=force -- every rank here shares the box's
    one GPU, where the library would otherwise fall back to host-driven mode
    (tested by test_shared_device_falls_back_to_host_driven).  Stream-ordered
    runs take the library's default protocol -- fenced tokens, one launch per
    element (test_stream_ordered_default_protocol) -- unless extra_env sets
    HICCL_STEP_PROGRAM / HICCL_PROG_FENCES; extra_env wins, None unsets."""
    assert np_ <= 8
    if stream_env is None:
        stream_env = "force" if streamed else "0"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", HICCL_STREAM_ORDERED=stream_env,
               HICCL_FUSED_GATHER="1" if fused else "0", HICCL_SIGNAL_TIMEOUT="10", HICCL_ENGINE=engine,
               HICCL_GRAPH="1" if graph else "0", HICCL_DRIVER_REPEAT=str(repeat))
    for k in ("HICCL_STEP_PROGRAM", "HICCL_PROG_FENCES"):  # the defaults unless asked
        env.pop(k, None)
    for k, v in (extra_env or {}).items():  # None: unset
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    if np_ > 4 and queues:
        # every rank on the box's one GPU: 8 processes x 4 hardware queues
        # oversubscribe the device's queue slots, and a spinning stream-ordered
        # wait can then outlast its timeout while the peer's queue is not
        # mapped; 2 queues per process keep them all mapped
        env["GPU_MAX_HW_QUEUES"] = "2"
    cmd = ["timeout", "-k", "10", str(timeout), MPIRUN, "-np", str(np_), exe] + [str(a) for a in args]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd="/tmp")
    return p.returncode, p.stdout + p.stderr


@pytest.mark.parametrize("streamed", [True, False], ids=["stream", "host"])
@pytest.mark.parametrize("np_,hier,libs", [(2, "2", "ipc"), (4, "2,2", "mpi,ipc"), (4, "4", "ipc_get"),
                                           (8, "1,4,2", "mpi,ipc,ipc")])
@pytest.mark.parametrize("pattern", [4, 7, 8, 6, 1])
def test_known_answer(np_, hier, libs, pattern, streamed):
    rc, out = mpirun(np_, HIP, [pattern, 4099, 1, 1, 3, 0, 0, hier, libs], streamed=streamed)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out
    assert ("stream-ordered" if streamed else "host-driven") in out


@pytest.mark.parametrize("streamed", [True, False], ids=["stream", "host"])
@pytest.mark.parametrize("np_,hier,libs", [(2, "2", "ipc"), (4, "4", "ipc_get"), (8, "1,4,2", "mpi,ipc,ipc"),
                                           (8, "2,4", "ipc,ipc_get")])
@pytest.mark.parametrize("pattern", [4, 7, 8])
def test_known_answer_fused_gather(np_, hier, libs, pattern, streamed):
    """HICCL_FUSED_GATHER=1: reductions read peers' buffers in place."""
    rc, out = mpirun(np_, HIP, [pattern, 4099, 1, 1, 3, 0, 0, hier, libs], streamed=streamed, fused=True)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out
    assert "fused gather" in out


@pytest.mark.parametrize("np_,count,stripe,ring,depth,hier,libs", [
    (2, 65536, 1, 1, 4, "2", "ipc"),
    (4, 10007, 1, 1, 3, "2,2", "mpi,ipc"),
    (8, 4099, 1, 1, 4, "1,4,2", "mpi,ipc,ipc"),
    (8, 4099, 1, 2, 2, "2,4", "ipc,ipc_get"),
])
@pytest.mark.parametrize("streamed,fused,engine,graph", [
    (True, False, "auto", False), (False, False, "auto", False), (True, True, "auto", False),
    (False, True, "auto", False), (False, False, "phase", False), (True, True, "phase", False),
    (True, False, "auto", True), (True, True, "auto", True)],
    ids=["stream", "host", "stream-fused", "host-fused", "host-phase", "stream-fused-phase", "stream-graph",
         "stream-fused-graph"])
def test_allreduce_float_bits_vs_oracle(tmp_path, oracle, np_, count, stripe, ring, depth, hier, libs, streamed,
                                        fused, engine, graph):
    """HICCL_ENGINE=phase forces the input-phased engine on every step's
    batched plan (these shapes would pick the tile engine).  Graph mode runs
    the pipeline 4 times (eager, capture + replay, 2 replays) and checks the
    last replay's bits."""
    prefix = str(tmp_path / "ar")
    rc, out = mpirun(np_, HIP_F32, [8, count, stripe, ring, depth, 0, 0, hier, libs, prefix], streamed=streamed,
                     fused=fused, engine=engine, graph=graph, repeat=4 if graph else 1)
    assert rc == 0, out[-3000:]
    if graph:
        assert "graph replay" in out
    n = count * np_
    x = {r: oracle.fill(r + 1, n, 1234)[r] for r in range(np_)}
    libmap = {"mpi": S.MPI, "ipc": S.IPC, "ipc_get": S.IPC_GET, "xccl": S.XCCL}
    sch = S.Schedule(np_, [int(h) for h in hier.split(",")], [libmap[lv] for lv in libs.split(",")],
                     numstripe=stripe, ringnodes=ring, pipedepth=depth, ring_reuse_fix=True)
    S.compose("allreduce", np_, count)(sch)
    steps = sch.init()
    user = {}
    for r in range(np_):
        user[(r, ("send",))] = x[r]
        user[(r, ("recv",))] = np.full(n, -1.0, np.float32)
    mem = S.simulate(steps, np_, user)
    for r in range(np_):
        got = np.fromfile(f"{prefix}.rank{r}.bin", dtype=np.float32)
        exp = mem[(r, ("recv",))]
        assert got.tobytes() == exp.tobytes(), f"rank {r}: {int((got != exp).sum())} differ"


@pytest.mark.parametrize("np_,count,depth,hier,libs", [(2, 65536, 4, "2", "ipc"), (8, 4099, 4, "1,4,2", "mpi,ipc,ipc")])
@pytest.mark.parametrize("fused,graph", [(False, False), (True, True)], ids=["stream", "stream-fused-graph"])
@pytest.mark.parametrize("program,tokens", [("0", "full"), ("1", "full"), ("1", "light"), ("0", "light")],
                         ids=["per_element-fenced", "step_program-fenced", "step_program-light", "per_element-light"])
def test_allreduce_bits_step_program_ab(tmp_path, oracle, np_, count, depth, hier, libs, fused, graph, program,
                                        tokens):
    """Stream-ordered mode under every protocol the config-5 leg A/Bs: one
    launch per element or one step program per step (HICCL_STEP_PROGRAM),
    with fenced or light token phases (HICCL_PROG_FENCES, hiccl_token_mode):
    the same bits as oracle/schedule.py every way."""
    prefix = str(tmp_path / "ar")
    rc, out = mpirun(np_, HIP_F32, [8, count, 1, 1, depth, 0, 0, hier, libs, prefix], streamed=True, fused=fused,
                     graph=graph, repeat=4 if graph else 2,
                     extra_env={"HICCL_STEP_PROGRAM": program, "HICCL_PROG_FENCES": tokens})
    assert rc == 0, out[-3000:]
    assert ("step programs: token phases folded" in out) == (program == "1"), out[-2000:]
    assert ("light (relaxed" if tokens == "light" else "fenced (release") in out, out[-2000:]
    n = count * np_
    x = {r: oracle.fill(r + 1, n, 1234)[r] for r in range(np_)}
    libmap = {"mpi": S.MPI, "ipc": S.IPC, "ipc_get": S.IPC_GET}
    sch = S.Schedule(np_, [int(h) for h in hier.split(",")], [libmap[lv] for lv in libs.split(",")],
                     numstripe=1, ringnodes=1, pipedepth=depth, ring_reuse_fix=True)
    S.compose("allreduce", np_, count)(sch)
    steps = sch.init()
    user = {}
    for r in range(np_):
        user[(r, ("send",))] = x[r]
        user[(r, ("recv",))] = np.full(n, -1.0, np.float32)
    mem = S.simulate(steps, np_, user)
    for r in range(np_):
        got = np.fromfile(f"{prefix}.rank{r}.bin", dtype=np.float32)
        exp = mem[(r, ("recv",))]
        assert got.tobytes() == exp.tobytes(), f"rank {r}: {int((got != exp).sum())} differ"


@pytest.mark.parametrize("graph", [False, True], ids=["stream", "stream-graph"])
def test_stream_ordered_default_protocol(graph):
    """Stream-ordered, HICCL_STEP_PROGRAM and HICCL_PROG_FENCES unset: the
    default protocol is fenced tokens and one launch per element of a step
    (the verified one; programs and light tokens are opt-in until a run with
    one GPU per rank decides); init says so and the KAT passes."""
    rc, out = mpirun(2, HIP, [8, 4099, 1, 1, 3, 0, 0, "2", "ipc"], graph=graph)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out and "stream-ordered" in out
    assert "stream-ordered protocol: fenced (release / acquire) tokens, one launch per element" in out, out[-2000:]
    assert "step programs: token phases folded" not in out, out[-2000:]


@pytest.mark.parametrize("np_,hier,libs", [(2, "2", "ipc"), (4, "2,2", "mpi,ipc"), (4, "4", "ipc_get"),
                                           (8, "1,4,2", "mpi,ipc,ipc")])
@pytest.mark.parametrize("pattern", [4, 8])
def test_known_answer_graph_replay(np_, hier, libs, pattern):
    """HICCL_GRAPH=1 with measurement: Comm::measure's eager executions
    advance the transports' epochs, so the next run() re-records the graph;
    HiCCL::measure then replays it, and the reference's KAT validates the
    final replay."""
    rc, out = mpirun(np_, HIP, [pattern, 4099, 1, 1, 3, 1, 3, hier, libs], streamed=True, graph=True)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out
    assert "graph replay" in out


@pytest.mark.parametrize("streamed", [True, False], ids=["stream", "host"])
@pytest.mark.parametrize("np_", [2, 4])
@pytest.mark.parametrize("count", [250000, 1 << 22])
def test_readme_api_example(np_, streamed, count):
    """Three rounds on the same user buffers, each with a fresh communicator
    (its schedule buffers freed and reallocated -- sub-allocated at 1 MB,
    dedicated allocations at 16 MiB -- and every IPC mapping released: the
    user buffers' mappings are revived, the schedule buffers' come back at
    recycled addresses and are opened anew)."""
    rc, out = mpirun(np_, os.path.join(ROOT, "build", "readme_example_hip"), [count, 3, 3], streamed=streamed,
                     extra_env={"HICCL_README_KEEP_BUFFERS": "1"})
    assert rc == 0, out[-3000:]
    assert out.count("README all-reduce: PASSED") == 3, out[-3000:]


@pytest.mark.parametrize("streamed", [True, False], ids=["stream", "host"])
@pytest.mark.parametrize("np_", [2, 4])
def test_recreated_communicators_on_reallocated_buffers(np_, streamed):
    """Five rounds, each with fresh user buffers (the previous round's freed:
    the allocator hands exported addresses back for new allocations) and a
    fresh communicator.  Closing a peer's mapping and opening its new
    allocation at the recycled address reaches other memory on ROCm 7.2
    (DESIGN.md section 6); the transport retires mappings instead, and every
    round must pass."""
    rc, out = mpirun(np_, os.path.join(ROOT, "build", "readme_example_hip"), [250000, 3, 5], streamed=streamed)
    assert rc == 0, out[-3000:]
    assert out.count("README all-reduce: PASSED") == 5, out[-3000:]


def test_recycled_address_never_silently_wrong():
    """With retirement off (HICCL_IPC_RETIRED_MAX=0: every released mapping is
    closed at once) a mapping of a recycled address may miss; the probe at
    init must then stop the job with its error -- a round that completes is
    correct, a FAILED round is never printed."""
    for _ in range(3):
        rc, out = mpirun(4, os.path.join(ROOT, "build", "readme_example_hip"), [250000, 3, 5], streamed=False,
                         extra_env={"HICCL_IPC_RETIRED_MAX": "0"})
        assert "FAILED" not in out, out[-3000:]
        if rc != 0:
            assert "does not reach it" in out, out[-3000:]
            return


@pytest.mark.parametrize("pattern", [8, 7])
def test_shared_device_falls_back_to_host_driven(pattern):
    """8 ranks on one GPU asking for stream-ordered mode (HICCL_STREAM_ORDERED=1)
    at HIP's default hardware-queue count: init() detects the shared device
    (PCI bus id per rank) and runs host-driven, so nothing spins while a
    peer's queue is unmapped -- the known-answer test passes without any
    GPU_MAX_HW_QUEUES override."""
    rc, out = mpirun(8, HIP, [pattern, 4099, 1, 1, 3, 1, 2, "1,4,2", "mpi,ipc,ipc"], stream_env="1", queues=False)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out
    assert "ranks share a GPU" in out and "host-driven" in out


@pytest.mark.parametrize("optin", [False, True], ids=["default", "rccl_requested"])
def test_xccl_level_shared_device_uses_ipc_path(optin):
    """An XCCL level runs on the (tested) IPC path unless HICCL_XCCL=rccl asks
    for RCCL; asked, with ranks sharing the one GPU, RCCL refuses two ranks on
    one device, so the level still runs on the IPC path.  Either way init says
    why and the known-answer test passes."""
    rc, out = mpirun(4, HIP, [8, 4099, 1, 1, 3, 0, 0, "2,2", "ipc,xccl"], streamed=False,
                     extra_env={"HICCL_XCCL": "rccl"} if optin else None)
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out
    assert "XCCL levels run on the IPC path" in out
    assert ("ranks share a GPU" if optin else "RCCL is opt-in") in out


def _ngpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif(_ngpus() < 2, reason="RCCL point-to-point needs one GPU per rank (>= 2 GPUs)")
@pytest.mark.parametrize("streamed", [False, True], ids=["host", "stream"])
def test_xccl_level_on_rccl(streamed):
    """One GPU per rank: the XCCL level moves its bytes with ncclSend/ncclRecv."""
    n = min(_ngpus(), 8)
    rc, out = mpirun(n, HIP, [8, 4099, 1, 1, 3, 0, 0, str(n), "xccl"], streamed=streamed,
                     stream_env="1" if streamed else "0", extra_env={"HICCL_XCCL": "rccl"})
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out and "XCCL on RCCL" in out


@pytest.mark.parametrize("streamed", [False, True], ids=["host", "stream"])
@pytest.mark.parametrize("pattern", [8, 6, 4])
def test_xccl_level_on_rccl_single_rank(pattern, streamed):
    """The form of the RCCL path one GPU can run (RCCL refuses two ranks on
    one device): ONE rank whose XCCL level's self transfers go through RCCL
    (HICCL_XCCL_SELF=rccl) -- the communicator from an MPI-broadcast id, one
    ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd per step on the
    transport stream, host-driven and stream-ordered, destroyed with the last
    communicator; the reference's known-answer test checks the bytes RCCL
    moved.  Cross-GPU RCCL (test_xccl_level_on_rccl) needs >= 2 GPUs."""
    rc, out = mpirun(1, HIP, [pattern, 4099, 1, 1, 3, 0, 0, "1", "xccl"], streamed=streamed,
                     stream_env="1" if streamed else "0",
                     extra_env={"HICCL_XCCL": "rccl", "HICCL_XCCL_SELF": "rccl"})
    assert rc == 0, out[-3000:]
    assert "PASSED!" in out and "XCCL on RCCL" in out, out[-3000:]
    assert ("stream-ordered" if streamed else "host-driven") in out
