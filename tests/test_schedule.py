"""CPU tier: the C++ factorization (include/hiccl/plan.h, Schedule, merge_steps)
against oracle/schedule.py, the restatement of the reference's reduce.h /
broadcast.h / init.h / command.h.

tests/cpp/plan_dump runs the C++ planner for every rank of a virtual machine
and prints the pipeline; this test executes that pipeline with numpy on float
inputs and requires the final receive buffers of every rank to equal the
oracle's bit for bit, and the step structure (per step and library: the
transfers and the computes with their fan-in and counts) to be identical.
The survey's compiled-reference probe is pinned too: a flat
hierarchy sums in rank order, {1,4,2} sums pairs first.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import schedule as S  # noqa: E402
from conftest import make

DUMP = os.path.join(ROOT, "build", "plan_dump")
LIBS = {"mpi": S.MPI, "ipc": S.IPC, "ipc_get": S.IPC_GET, "xccl": S.XCCL}
SEND, RECV, TMP = 1 << 40, 2 << 40, 3 << 40


@pytest.fixture(scope="module", autouse=True)
def built():
    make(ROOT, "build/plan_dump")


def inputs(np_, n):
    rng = np.random.default_rng(np_ * 1000 + n)
    return {r: (rng.uniform(-1, 1, n) * 10.0 ** rng.integers(-3, 4, n)).astype(np.float32) for r in range(np_)}


def run_dump(np_, pattern, count, stripe, ring, depth, hier, libs):
    out = subprocess.run([DUMP, str(np_), str(S.PATTERN_IDS[pattern]), str(count), str(stripe), str(ring),
                          str(depth), ",".join(map(str, hier)), ",".join(libs)],
                         check=True, capture_output=True, text=True).stdout
    return [json.loads(line) for line in out.splitlines()]


def simulate_dump(recs, np_, count, x, fuse=False):
    """fuse=True executes the plan as HICCL_FUSED_GATHER does: transfers
    marked `feeds` are dropped and the compute reads the sender's buffer in
    place (oracle/schedule.py Remote)."""
    allocs = {}
    for r in recs:
        if r["kind"] == "alloc":
            allocs.setdefault(r["rank"], []).append((r["addr"], r["count"]))

    def loc(rank, addr):
        if SEND <= addr < RECV:
            return ("send",), (addr - SEND) // 4
        if RECV <= addr < TMP:
            return ("recv",), (addr - RECV) // 4
        for base, n in allocs.get(rank, []):
            if base <= addr < base + 4 * max(n, 1):
                return ("tmp", rank, base), (addr - base) // 4
        raise AssertionError(f"rank {rank}: address {addr} not allocated")

    meta = {r["rank"]: r for r in recs if r["kind"] == "meta"}
    nsteps = {m["steps"] for m in meta.values()}
    assert len(nsteps) == 1, f"ranks disagree on the number of steps: {nsteps}"
    libs = {tuple(m["libs"]) for m in meta.values()}
    assert len(libs) == 1
    libs = list(libs.pop())
    steps = [{lib: S.Coll(lib) for lib in libs} for _ in range(nsteps.pop())]
    xf = {}
    for r in recs:
        if r["kind"] == "xfer":
            key = (r["step"], r["lib"], r["idx"])
            e = xf.setdefault(key, {"sendid": r["sendid"], "recvid": r["recvid"], "count": r["count"],
                                    "feeds": r["feeds"]})
            assert (e["sendid"], e["recvid"], e["count"], e["feeds"]) == \
                (r["sendid"], r["recvid"], r["count"], r["feeds"]), key  # every rank plans the same
            if r["rank"] == r["sendid"]:
                e["src"] = loc(r["rank"], r["src"])
            if r["rank"] == r["recvid"]:
                e["dst"] = loc(r["rank"], r["dst"])
    fused = {}  # (step, lib, recvid, dst) -> Remote((sendid, src))
    for (s, lib, idx) in sorted(xf):
        e = xf[(s, lib, idx)]
        if fuse and e["feeds"] and e["sendid"] != e["recvid"]:
            fused[(s, lib, e["recvid"], e["dst"])] = S.Remote((e["sendid"], e["src"]))
            continue
        steps[s][lib].add_comm(e["sendid"], e["src"], e["recvid"], e["dst"], e["count"])
    for r in recs:
        if r["kind"] == "comp":
            ins = [loc(r["rank"], a) for a in r["in"]]
            ins = [fused.get((r["step"], r["lib"], r["rank"], i), i) for i in ins]
            steps[r["step"]][r["lib"]].add_compute(r["rank"], ins, loc(r["rank"], r["out"]), r["count"])
    user = {}
    for rank in range(np_):
        user[(rank, ("send",))] = x[rank].copy()
        user[(rank, ("recv",))] = np.full(count * np_, np.nan, np.float32)
    return steps, S.simulate(steps, np_, user)


def oracle_run(np_, pattern, count, stripe, ring, depth, hier, libs, x, fix=True):
    sch = S.Schedule(np_, hier, [LIBS[lib] for lib in libs], numstripe=stripe, ringnodes=ring, pipedepth=depth,
                     ring_reuse_fix=fix)
    S.compose(pattern, np_, count)(sch)
    steps = sch.init()
    user = {}
    for rank in range(np_):
        user[(rank, ("send",))] = x[rank].copy()
        user[(rank, ("recv",))] = np.full(count * np_, np.nan, np.float32)
    return steps, S.simulate(steps, np_, user)


def structure(steps):
    out = []
    for st in steps:
        row = {}
        for lib, c in st.items():
            row[lib] = (sorted((a, b, n) for a, _, b, _, n in c.comms),
                        sorted((r, len(ins), n) for r, ins, _, n in c.computes))
        out.append(row)
    return out


CONFIGS = [
    # numproc, pattern, count, numstripe, ringnodes, pipedepth, hierarchy, libs
    (2, "allreduce", 1000, 1, 1, 4, [2], ["mpi"]),
    (2, "reduce", 513, 1, 1, 3, [2], ["mpi"]),
    (8, "allreduce", 300, 1, 1, 1, [8], ["mpi"]),
    (8, "allreduce", 301, 1, 1, 3, [1, 4, 2], ["mpi", "ipc", "ipc"]),
    (8, "reducescatter", 97, 1, 1, 2, [2, 4], ["mpi", "ipc"]),
    (8, "reduce", 50, 1, 1, 5, [2, 2, 2], ["mpi", "ipc_get", "ipc"]),
    (8, "allreduce", 100, 1, 2, 2, [2, 4], ["mpi", "ipc"]),
    (8, "allreduce", 100, 1, 4, 2, [4, 2], ["mpi", "ipc"]),
    (8, "allreduce", 101, 4, 1, 2, [2, 4], ["mpi", "ipc"]),
    (8, "allreduce", 77, 2, 2, 3, [2, 2, 2], ["mpi", "ipc", "ipc"]),
    (16, "allreduce", 64, 1, 1, 2, [2, 4, 2], ["mpi", "ipc", "ipc"]),
    (12, "allreduce", 40, 1, 1, 2, [2, 6], ["mpi", "ipc"]),
    (12, "allreduce", 40, 1, 3, 2, [3, 4], ["mpi", "ipc"]),
] + [(4, p, 33, 1, 1, 2, [2, 2], ["mpi", "ipc"]) for p in S.PATTERN_IDS] + [
    (8, p, 17, 2, 2, 2, [2, 4], ["mpi", "ipc"]) for p in S.PATTERN_IDS]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: f"P{c[0]}-{c[1]}-s{c[3]}r{c[4]}d{c[5]}-{'x'.join(map(str, c[6]))}")
def test_cpp_plan_matches_oracle(cfg):
    np_, pattern, count, stripe, ring, depth, hier, libs = cfg
    x = inputs(np_, count * np_)
    recs = run_dump(np_, pattern, count, stripe, ring, depth, hier, libs)
    csteps, cmem = simulate_dump(recs, np_, count, x)
    osteps, omem = oracle_run(np_, pattern, count, stripe, ring, depth, hier, libs, x)
    assert len(csteps) == len(osteps)
    assert structure(csteps) == structure(osteps)
    for rank in range(np_):
        a, b = cmem[(rank, ("recv",))], omem[(rank, ("recv",))]
        assert a.tobytes() == b.tobytes(), f"rank {rank}: {int((a != b).sum())} elements differ"
        # user send buffers are never written
        assert cmem[(rank, ("send",))].tobytes() == x[rank].tobytes()


def _seq(x, ranks):
    acc = np.zeros_like(x[0])
    for r in ranks:
        acc = (acc + x[r]).astype(np.float32)
    return acc


def test_probe_orders_flat_and_142():
    """SURVEY.md 8c (compiled reference, mpirun -np 8): flat = sequential
    rank order; {1,4,2} = ((p01 + p23) + p45) + p67 with pairs first."""
    np_, count = 8, 257
    x = inputs(np_, count * np_)
    _, mem = simulate_dump(run_dump(np_, "allreduce", count, 1, 1, 4, [8], ["mpi"]), np_, count, x)
    seq = _seq(x, range(8))
    assert all(mem[(r, ("recv",))].tobytes() == seq.tobytes() for r in range(np_))
    _, mem = simulate_dump(run_dump(np_, "allreduce", count, 1, 1, 4, [1, 4, 2], ["mpi", "ipc", "ipc"]),
                           np_, count, x)
    tree = np.zeros_like(x[0])
    for g in range(4):
        tree = (tree + ((np.float32(0) + x[2 * g]) + x[2 * g + 1]).astype(np.float32)).astype(np.float32)
    assert all(mem[(r, ("recv",))].tobytes() == tree.tobytes() for r in range(np_))
    assert (mem[(0, ("recv",))] != seq).sum() > 0  # the two orders are distinguishable


def test_ring_single_rank_nodes_reference_defect():
    """One rank per ring node, >= 3 nodes: the reference (faithful oracle)
    loses terms and writes into user send buffers; the build sums every rank."""
    np_, count = 4, 16
    x = inputs(np_, count * np_)
    cfg = (np_, "allreduce", count, 1, 4, 1, [4], ["mpi"])
    _, cmem = simulate_dump(run_dump(*cfg), np_, count, x)
    _, ref = oracle_run(*cfg, x, fix=False)
    _, fixed = oracle_run(*cfg, x, fix=True)
    for r in range(np_):
        assert cmem[(r, ("recv",))].tobytes() == fixed[(r, ("recv",))].tobytes()
    exact = sum(x[r].astype(np.float64) for r in range(np_))
    assert np.allclose(cmem[(0, ("recv",))], exact, rtol=1e-5, atol=1e-4)
    assert not np.allclose(ref[(0, ("recv",))], exact, rtol=1e-5, atol=1e-4)
    assert any(ref[(r, ("send",))].tobytes() != x[r].tobytes() for r in range(np_))


def fused_hazards(recs):
    """Static conditions for dropping a `feeds` transfer (comm.h fused
    gather): (1) its receive buffer is an input of exactly one compute of the
    same step and library on the receiver; (2) nothing writes the sender's
    source during that step; (3) no later step reads the receive buffer
    before writing it."""
    problems = []
    feeds = [r for r in recs if r["kind"] == "xfer" and r["feeds"] and r["rank"] == r["recvid"]]
    srcs = {(r["step"], r["lib"], r["idx"]): r for r in recs if r["kind"] == "xfer" and r["rank"] == r["sendid"]}
    comps = [r for r in recs if r["kind"] == "comp"]
    writes = {}  # (step, rank) -> [(addr, nbytes)]
    for r in recs:
        if r["kind"] == "xfer" and r["rank"] == r["recvid"]:
            writes.setdefault((r["step"], r["rank"]), []).append((r["dst"], 4 * r["count"]))
        if r["kind"] == "comp":
            writes.setdefault((r["step"], r["rank"]), []).append((r["out"], 4 * r["count"]))
    ov = lambda a, n, b, m: a < b + m and b < a + n  # noqa: E731
    for f in feeds:
        if f["sendid"] == f["recvid"]:
            continue
        nb = 4 * f["count"]
        uses = sum(i == f["dst"] for c in comps if (c["step"], c["lib"], c["rank"]) == (f["step"], f["lib"], f["recvid"])
                   for i in c["in"])
        if uses != 1:
            problems.append(("uses", f, uses))
        src = srcs[(f["step"], f["lib"], f["idx"])]["src"]
        for (a, n) in writes.get((f["step"], f["sendid"]), []):
            if ov(a, n, src, nb):
                problems.append(("src written", f))
        for t in range(f["step"] + 1, max(r.get("step", 0) for r in recs) + 1):
            rd = [r for r in recs if r.get("step") == t and r["rank"] == f["recvid"]]
            if any(r["kind"] == "xfer" and r["rank"] == r["sendid"] and ov(r["src"], 4 * r["count"], f["dst"], nb)
                   for r in rd):
                problems.append(("read later", f, t))
                break
            if any(r["kind"] == "xfer" and r["rank"] == r["recvid"] and ov(r["dst"], 4 * r["count"], f["dst"], nb)
                   for r in rd):
                break
            if any(r["kind"] == "comp" and any(ov(i, 4 * r["count"], f["dst"], nb) for i in r["in"]) for r in rd):
                problems.append(("read later", f, t))
                break
            if any(r["kind"] == "comp" and ov(r["out"], 4 * r["count"], f["dst"], nb) for r in rd):
                break
    return problems


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: f"P{c[0]}-{c[1]}-s{c[3]}r{c[4]}d{c[5]}-{'x'.join(map(str, c[6]))}")
def test_fused_gather_plan(cfg):
    """SURVEY.md 8 row f: the fused gather + reduce executes the same plan
    minus the `feeds` copies, reading senders' buffers in place; the results
    must equal the unfused oracle bit for bit and the plan must be free of the
    hazards dropping those copies could expose."""
    np_, pattern, count, stripe, ring, depth, hier, libs = cfg
    x = inputs(np_, count * np_)
    recs = run_dump(np_, pattern, count, stripe, ring, depth, hier, libs)
    assert fused_hazards(recs) == []
    _, fmem = simulate_dump(recs, np_, count, x, fuse=True)
    _, omem = oracle_run(np_, pattern, count, stripe, ring, depth, hier, libs, x)
    nfeeds = sum(r["kind"] == "xfer" and r["feeds"] and r["rank"] == r["recvid"] for r in recs)
    if pattern in ("reduce", "allreduce", "reducescatter"):
        assert nfeeds > 0
    for rank in range(np_):
        a, b = fmem[(rank, ("recv",))], omem[(rank, ("recv",))]
        assert a.tobytes() == b.tobytes(), f"rank {rank}: {int((a != b).sum())} elements differ"


def test_consecutive_steps_share_buffers():
    """DESIGN.md section 8 (Next 3): under the reference's buffer recycling a
    pipeline step's copies write the receive buffers the previous step's
    reductions read, so the two cannot share a launch -- tools/step_overlap.py
    over every rank of the C++ factorization (the {1,4,2} all-reduce at
    pipedepth 4 and 16, a flat {8})."""
    if not os.path.exists(DUMP):
        make(ROOT, "build/plan_dump")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import step_overlap
    for args, most in ((["8", "8", "4096", "1", "1", "4", "1,4,2", "mpi,ipc,ipc"], 1),
                       (["8", "8", "65536", "1", "1", "16", "1,4,2", "mpi,ipc,ipc"], 1),
                       (["8", "8", "65536", "1", "1", "16", "8", "ipc"], 0)):
        for r in step_overlap.analyze(args):
            assert r["pairs"] > 0 and r["independent_pairs"] <= most, (args, r)
