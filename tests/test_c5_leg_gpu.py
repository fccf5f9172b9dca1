"""GPU tier: bench.py's config-5 leg (the all-reduce composition run as an
MPI job by rank 0, collectives/main.cpp:151-155) rehearsed on the box's one
GPU: 2 ranks share it, so the stream-ordered mode falls back to host-driven;
both modes must produce the JSON the N > 1 bench line carries and pass the
float-exact known-answer check."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def test_c5_leg_rehearsal_two_ranks_one_gpu():
    import bench
    res = bench.run_c5(2, argparse.Namespace(c5_log2count=16, c5_iters=2), allow_shared=True)
    assert "workload" in res, res
    for mode in ("host", "stream_graph", "stream_graph_fused"):
        r = res[mode]
        assert r.get("kat") == "PASSED", r
        assert r["ranks"] == 2 and r["pipedepth"] == 128
        assert r["collective_ms_median"] > 0 and r["algorithmic_GBps_median"] > 0
        assert r["kernel_steps_rank0"] > 0 and r["kernel_ms_per_run_max_rank"] > 0
