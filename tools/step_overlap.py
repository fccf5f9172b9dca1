#!/usr/bin/env python3
"""Could a pipeline step's copies run in the same launch as the previous
step's reductions?  For every rank of a virtual machine (build/plan_dump,
the C++ factorization), count consecutive step pairs (s, s+1) where the
copies of step s+1 neither read what the reductions of step s write nor
write (locally: self copies, peers' puts into this rank) what they read or
write.  DESIGN.md section 8 (Next 3).

    python tools/step_overlap.py [numproc pattern count stripe ring depth hierarchy libs]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def analyze(args):
    out = subprocess.run([os.path.join(ROOT, "build", "plan_dump")] + args, capture_output=True, text=True,
                         check=True).stdout
    rows = [json.loads(line) for line in out.splitlines()]
    comps = [r for r in rows if r["kind"] == "comp"]
    xfers = [r for r in rows if r["kind"] == "xfer"]

    def rg(addr, count):
        return addr, addr + count * 4

    def ov(a, b):
        return a[0] < b[1] and b[0] < a[1]

    res = []
    for me in range(int(args[0])):
        steps = max([r["step"] for r in comps + xfers if r["rank"] == me] + [0]) + 1
        legal = total = 0
        for s in range(steps - 1):
            cs = [r for r in comps if r["rank"] == me and r["step"] == s]
            xs = [r for r in xfers if r["rank"] == me and r["step"] == s + 1]
            writes = [rg(c["out"], c["count"]) for c in cs]
            reads = [rg(i, c["count"]) for c in cs for i in c["in"] if i is not None]
            xr = [rg(x["src"], x["count"]) for x in xs if x["sendid"] == me and x["src"] is not None]
            xw = [rg(x["dst"], x["count"]) for x in xs if x["recvid"] == me and x["dst"] is not None]
            bad = any(ov(a, b) for a in xr for b in writes) or any(ov(a, b) for a in xw for b in writes + reads)
            total += 1
            legal += not bad
        res.append({"rank": me, "independent_pairs": legal, "pairs": total})
    return res


if __name__ == "__main__":
    cases = [sys.argv[1:]] if len(sys.argv) > 1 else [
        ["8", "8", "4096", "1", "1", "4", "1,4,2", "mpi,ipc,ipc"],
        ["8", "8", "65536", "1", "1", "16", "1,4,2", "mpi,ipc,ipc"],
        ["8", "8", "65536", "1", "1", "16", "8", "ipc"]]
    for a in cases:
        print(json.dumps({"args": " ".join(a), "ranks": analyze(a)}))
