"""GPU tier: the HIP IPC behaviour the transport's retired mappings rest on.

tests/cpp/ipc_reuse.cpp (two MPI processes) runs, per round: the owner
exports a fresh allocation A, the importer opens it and either closes the
mapping ("close") or keeps it ("keep"); the owner frees A, allocates B of
the same size (usually at A's address) and exports it; the importer opens B
and reads the owner's nonce through the copy engine and through a kernel.

The design (include/hiccl/transport.h IpcMapping)
assumes "keep" always reaches B, and treats "close" as unsafe.  This test
asserts the first and RECORDS the second -- whatever the runtime does -- in
gpurun_out/ipc_reuse.jsonl, so the premise is pinned by a committed outcome
(profiles/r03_ipc_reuse.jsonl) rather than by builder logs.
"""
import json
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
EXE = os.path.join(ROOT, "build", "ipc_reuse")


def test_ipc_close_then_reopen_recycled_address_outcome():
    rounds = 8
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(["timeout", "-k", "10", "120", MPIRUN, "-np", "2", EXE, str(rounds), str(64 << 20)],
                       capture_output=True, text=True, env=env, cwd="/tmp")
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    res = {r["variant"]: r for r in (json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{"))}
    assert set(res) == {"close", "keep"}, p.stdout
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "ipc_reuse.jsonl"), "a") as f:
        for r in res.values():
            f.write(json.dumps(r) + "\n")
    for r in res.values():
        assert r["first_mapping_ok"] == rounds  # a fresh export is always reachable
    keep = res["keep"]
    # the premise of retiring instead of closing: with the old mapping still
    # open, the new allocation at a recycled address is reached in both views
    assert keep["second_mapping_copy_engine_ok"] == rounds and keep["second_mapping_kernel_ok"] == rounds, keep
