"""GPU tier: the HIP IPC behaviour the transport's retired mappings rest on.

tests/cpp/ipc_reuse.cpp (2 or 4 MPI processes, all-to-all like a
communicator) runs, per round: every rank exports fresh allocations A, every
peer opens them and then closes its mappings ("close"), keeps them
("keep"), -- "mixed" -- odd ranks keep and even ranks close, or -- "late" --
keeps them until it has opened the next allocation at the same address and
closes them then (what a capped retirement does); every rank
frees A, allocates B of the same sizes (usually at A's addresses) and
exports them; the peers open B and read the owner's nonces through the copy
engine and through a kernel.  Cases: 64 MiB (own allocations) and 1 MiB
(sub-allocated) buffers, one or three per rank.

The design (include/hiccl/transport.h IpcMapping)
retires mappings instead of closing them.  This test asserts that "keep"
always opens and reaches B (the design's premise) and RECORDS what the other
policies do -- whatever the runtime does; on ROCm 7.2 round 3 saw "close"
read stale data through some new mappings and "mixed" fail to open them or
(once) to export the new allocation -- in gpurun_out/ipc_reuse.jsonl
(committed as profiles/r03*_ipc_reuse*.jsonl).  The reproducer records a
failed export or open as an outcome; it runs after the rest of the suite
(marker runtime_probe)."""
import json
import os
import shutil
import subprocess

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.runtime_probe]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
EXE = os.path.join(ROOT, "build", "ipc_reuse")


@pytest.mark.parametrize("ranks", [2, 4])
def test_ipc_close_then_reopen_recycled_address_outcome(ranks):
    rounds = 6
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(["timeout", "-k", "10", "150", MPIRUN, "-np", str(ranks), EXE, str(rounds)],
                       capture_output=True, text=True, env=env, cwd="/tmp")
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    rows = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(rows) == 16, p.stdout
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "ipc_reuse.jsonl"), "a") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    for r in rows:
        if r["variant"] == "keep":
            # the premise of retiring instead of closing: while every earlier
            # mapping stays open, every new allocation -- at a recycled
            # address or not -- opens and is reached, in both views
            assert r["first_export_failed"] == 0 and r["second_export_failed"] == 0, r
            assert r["first_open_failed"] == 0 and r["first_mapping_ok"] == r["first_opens"], r
            assert r["second_open_failed"] == 0, r
            assert r["second_mapping_copy_engine_ok"] == r["reads"], r
            assert r["second_mapping_kernel_ok"] == r["reads"], r
