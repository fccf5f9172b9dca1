"""The C++ surface's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

The host port (`HICCL_PORT_HOST`: the schedule, factorization, pipeline and
the CPU reduction of compute.h:14-23) and the plan dumper are built with
`tools/sanitize.mk` (g++, CPU only) and run over the reference driver's
patterns (collectives/main.cpp:47-53 argv) and hierarchies; any sanitizer
report aborts the run.  The driver's own known-answer check must pass, and the
sanitized dumper must plan exactly what the plain build plans.
"""
import os
import shutil
import subprocess

import pytest
from conftest import make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
SAN = os.path.join(ROOT, "build", "san")
ENV = dict(os.environ, OMP_NUM_THREADS="1", ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(MPIRUN):
        pytest.skip("no mpirun")
    make(ROOT, "-f", "tools/sanitize.mk", "all")
    make(ROOT, "build/plan_dump")


def _run(cmd, timeout=240):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=ENV, cwd="/tmp")
    out = p.stdout + p.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-3000:]
    assert p.returncode == 0, out[-3000:]
    return out


@pytest.mark.parametrize("np_,args", [
    (2, [4, 131072, 1, 1, 1, 1, 3]),                                   # config 1 (reduce, 2 x 1 MiB)
    (8, [8, 1000, 1, 1, 3, 0, 0, "1,4,2", "mpi,ipc,ipc"]),             # config 5's hierarchy, small
    (8, [5, 1001, 2, 1, 4, 0, 0, "1,4,2", "mpi,ipc,ipc"]),             # stripes, ragged count
    (4, [6, 777, 1, 2, 5, 0, 0, "2,2", "mpi,ipc"]),                    # ring nodes
    (8, [8, 4096, 2, 2, 4, 0, 0, "8", "ipc"]),                         # flat, stripes + ring
])
def test_host_port_clean(np_, args):
    out = _run([MPIRUN, "-np", str(np_), os.path.join(SAN, "collectives_host_f32")] + [str(a) for a in args])
    assert "PASSED" in out and "FAILED" not in out, out[-2000:]


@pytest.mark.parametrize("pattern", range(1, 9))
def test_host_port_every_pattern_clean(pattern):
    out = _run([MPIRUN, "-np", "4", os.path.join(SAN, "collectives_host_f32"), str(pattern), "999", "2", "1", "3",
                "0", "0", "2,2", "mpi,ipc"])
    assert "PASSED" in out and "FAILED" not in out, out[-2000:]


@pytest.mark.parametrize("args", [
    ["8", "8", "1000", "1", "1", "3", "1,4,2", "mpi,ipc,ipc"],
    ["4", "5", "1001", "2", "2", "4", "2,2", "mpi,ipc"],
    ["6", "7", "333", "3", "1", "2", "6", "ipc_get"],
])
def test_plan_dump_clean_and_identical(args):
    san = _run([os.path.join(SAN, "plan_dump")] + args)
    plain = subprocess.run([os.path.join(ROOT, "build", "plan_dump")] + args, capture_output=True, text=True,
                           check=True).stdout
    assert san == plain


def test_driver_json_and_step_timing_clean(tmp_path):
    """bench.py's config-5 JSON path (HICCL_DRIVER_JSON: HiCCL::measure, the
    known-answer run, Comm::set_step_timing's timed runs) under the
    sanitizers, on config 5's hierarchy."""
    import json
    path = tmp_path / "c5.json"
    cmd = [MPIRUN, "-np", "8", os.path.join(SAN, "collectives_host_f32"), "8", "1000", "1", "1", "3", "1", "2",
           "1,4,2", "mpi,ipc,ipc"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(ENV, HICCL_DRIVER_JSON=str(path)),
                       cwd="/tmp")
    out = p.stdout + p.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-3000:]
    assert p.returncode == 0, out[-3000:]
    r = json.loads(path.read_text())
    assert r["kat"] == "PASSED" and r["host_split_us_per_step"]["runs"] == 1
