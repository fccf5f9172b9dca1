"""CPU tier: the C++ surface end to end under MPI, host port (config 1:
"2-proc MPI loopback on host CPU ... CPU sum path, no GPU").

build/collectives_host is this build's counterpart of collectives/main.cpp
(hiccl_amd/csrc/collectives.cpp) compiled with HICCL_PORT_HOST: HiCCL::Comm<T>
factorizes, the MPI transport moves host buffers, Compute<T> sums on the host.
* every collective passes the reference's own known-answer test
  (HiCCL::validate, bench.h:62-227) with T = size_t, as the reference driver;
* float runs dump every rank's receive buffer and must equal, bit for bit,
  oracle/schedule.py's simulation of the reference's schedule on the same
  inputs (the oracle generator's values).
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
from conftest import make

MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
HOST = os.path.join(ROOT, "build", "collectives_host")
HOST_F32 = os.path.join(ROOT, "build", "collectives_host_f32")

pytestmark = pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")


@pytest.fixture(scope="module", autouse=True)
def built():
    make(ROOT, "build/collectives_host", "build/collectives_host_f32", "build/readme_example_host")


def mpirun(np_, exe, args, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [MPIRUN, "-np", str(np_), exe] + [str(a) for a in args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd="/tmp")
    return p.returncode, p.stdout + p.stderr


def test_config1_two_rank_reduce_float():
    """BASELINE config 1: 2 ranks, Comm<float> reduction of 2 x 1 MiB (host)."""
    rc, out = mpirun(2, HOST_F32, [4, 131072, 1, 1, 1, 1, 3])
    assert rc == 0, out
    assert "VERIFY REDUCE ROOT = 0: PASSED!" in out


@pytest.mark.gpu
def test_config1_two_rank_reduce_float_on_gpu_box_host(tmp_path, oracle):
    """Config 1 exactly as BASELINE.json names it (Comm<float> add_reduction of
    2 x 1 MiB, 2 MPI ranks, CPU sum path) on the GPU box's own host -- the
    box the CPU baseline is timed on.  Marked gpu so the round-end GPU tier
    records it there; no GPU is used.  Besides the reference's KAT, the root's
    float result must equal, bit for bit, the oracle's in-order sum of the two
    ranks' generator inputs (rank 0 + rank 1, the flat order reduce.h:134-169
    emits)."""
    rc, out = mpirun(2, HOST_F32, [4, 131072, 1, 1, 1, 1, 3])
    assert rc == 0, out
    assert "VERIFY REDUCE ROOT = 0: PASSED!" in out
    prefix = str(tmp_path / "c1")
    rc, out = mpirun(2, HOST_F32, [4, 131072, 1, 1, 1, 0, 0, "2", "mpi", prefix])
    assert rc == 0, out
    n = 131072 * 2
    x = [oracle.fill(r + 1, n, 1234)[r] for r in range(2)]  # rank r's input, as the driver generates it
    got = np.fromfile(f"{prefix}.rank0.bin", dtype=np.float32)
    exp = oracle.reduce(x)  # pattern 4: root 0 receives the sum of both 1 MiB send buffers
    assert len(got) == n and got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("np_,hier,libs", [(2, "2", "mpi"), (4, "2,2", "mpi,ipc"), (8, "1,4,2", "mpi,ipc,ipc"),
                                           (6, "3,2", "mpi,mpi")])
@pytest.mark.parametrize("pattern", range(1, 9))
def test_known_answer_all_collectives(np_, hier, libs, pattern):
    rc, out = mpirun(np_, HOST, [pattern, 1000, 1, 1, 3, 0, 0, hier, libs])
    assert rc == 0, out
    assert "PASSED!" in out


@pytest.mark.parametrize("np_,count,stripe,ring,depth,hier,libs", [
    (2, 4096, 1, 1, 4, "2", "mpi"),
    (8, 1000, 1, 1, 3, "1,4,2", "mpi,ipc,ipc"),
    (8, 1000, 1, 1, 1, "8", "mpi"),
    (8, 333, 1, 2, 2, "2,4", "mpi,ipc"),
    (8, 333, 2, 1, 2, "2,4", "mpi,ipc"),
])
def test_allreduce_float_bits_vs_oracle(tmp_path, oracle, np_, count, stripe, ring, depth, hier, libs):
    prefix = str(tmp_path / "ar")
    rc, out = mpirun(np_, HOST_F32, [8, count, stripe, ring, depth, 0, 0, hier, libs, prefix])
    assert rc == 0, out
    n = count * np_
    x = {r: oracle.fill(r + 1, n, 1234)[r] for r in range(np_)}  # row k = rank k's input
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


@pytest.mark.parametrize("np_", [1, 2, 4, 6])
def test_readme_api_example(np_):
    """README.md:12-60 spellings: add_reduction / add_fence / add_multicast /
    init(hierarchy, lib, numstripe, ring, pipeline) / start() / wait(); two
    rounds, each with a fresh communicator (its schedule buffers freed)."""
    rc, out = mpirun(np_, os.path.join(ROOT, "build", "readme_example_host"), [1001, 3, 2])
    assert rc == 0, out
    assert out.count("README all-reduce: PASSED") == 2, out
