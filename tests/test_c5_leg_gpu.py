"""GPU tier: bench.py's config-5 leg (the all-reduce composition run as an
MPI job by rank 0, collectives/main.cpp:151-155) rehearsed on the box's one
GPU: 2 or 4 ranks share it, so the stream-ordered mode falls back to
host-driven; every mode must produce the JSON the N > 1 bench line carries and pass the
float-exact known-answer check."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ranks", [2, 4])
def test_c5_leg_rehearsal_one_gpu(ranks):
    """4 ranks: hierarchy {1,2,2} {MPI,IPC,IPC}, the same on XCCL levels (RCCL
    refuses shared GPUs: the IPC fallback here), plus the flat {4} {IPC} run."""
    import bench
    res = bench.run_c5(ranks, argparse.Namespace(c5_log2count=14, c5_iters=2), allow_shared=True)
    assert "workload" in res, res
    # the verified default protocol first, the light-token programs last
    modes = (["host", "stream_graph", "stream_graph_fused_noprog", "stream_graph_fused_fenced"]
             + (["flat_stream_graph_fused"] if ranks > 2 else []) + ["xccl", "stream_graph_fused"])
    assert [m for m in res if m.endswith(("host", "fused", "graph", "xccl", "noprog", "fenced"))] == modes
    assert res["devices_counted_unmasked"] >= 1 and isinstance(res["env_scrubbed"], dict)
    for mode in modes:
        r = res[mode]
        assert r.get("kat") == "PASSED", r
        assert r["rc"] == 0 and len(r["devices_seen"]) == ranks and len(r["bus_ids"]) == ranks
        assert len(set(r["bus_ids"])) == 1 and "ranks share a GPU" in r["mode_used"]  # one GPU here
        if mode == "xccl":
            assert "xccl-rccl" not in r["mode_used"]  # RCCL refuses a shared GPU: the IPC path ran
        assert r["ranks"] == ranks and r["pipedepth"] == 128
        assert r["hierarchy"] == (str(ranks) if mode.startswith("flat") or ranks == 2 else f"1,{ranks // 2},2")
        assert r["collective_ms_median"] > 0 and r["algorithmic_GBps_median"] > 0
        assert r["kernel_steps_rank0"] > 0 and r["kernel_ms_per_run_max_rank"] > 0
        hs = r["host_split_us_per_step"]  # shared GPU: host-driven, the transport / compute parts
        assert hs["steps"] > 0 and hs["runs"] == 1 and hs["transport_wait"] + hs["compute_wait"] > 0
    ab = res["protocol_ab"]
    assert ab["baseline_kat"] == "PASSED" and ab["baseline_ms"] > 0
    for name in ("stream_graph_fused_fenced", "stream_graph_fused"):
        assert ab[name]["kat"] == "PASSED" and ab[name]["over_baseline"] > 0


@pytest.mark.parametrize("mode", ["host", "stream_graph_fused_noprog"])
def test_config5_exact_shape_one_gpu(mode):
    """Config 5 at its exact shape and size (collectives/main.cpp:151-155 with
    {1,4,2} {MPI,IPC,IPC}, 2^25 floats per rank per chunk = a 1 GiB send
    buffer per rank, pipedepth 128) with all 8 ranks on the box's one GPU,
    in two protocols: host-driven (the reference's own, comm.h:186-206), and
    the stream-ordered one an 8-GPU run takes by default -- fenced tokens,
    one launch per element, graph replay, fused gather -- forced here
    (HICCL_STREAM_ORDERED=force, 2 hardware queues per rank) where the
    library would otherwise fall back to host-driven on a shared GPU.  The
    all-reduce's float-exact known-answer check passes at full size, every
    step's batched kernel is timed.  Parity only -- one GPU moves the "xGMI"
    bytes through its own HBM, so the times rank nothing (DESIGN.md
    section 6)."""
    import bench
    res = bench.run_c5(8, argparse.Namespace(c5_log2count=25, c5_iters=1), allow_shared=True, only=(mode,),
                       force_stream=True)
    r = res[mode]
    assert r.get("kat") == "PASSED" and r["kat_exact_mismatches"] == 0, r
    assert r["rc"] == 0 and r["ranks"] == 8 and r["hierarchy"] == "1,4,2" and r["libs"] == "MPI,IPC,IPC"
    assert r["pipedepth"] == 128 and r["count_per_rank_chunk"] == 1 << 25
    assert r["sendbuf_bytes_per_rank"] == float(8 << 27)  # 2^25 floats x 8 ranks x 4 B = 1 GiB
    assert r["kernel_steps_rank0"] > 0 and r["kernel_ms_per_run_max_rank"] > 0
    assert len(set(r["bus_ids"])) == 1 and r["mode_used"].endswith("(ranks share a GPU)")
    if mode == "host":
        assert r["mode_used"].startswith("host-driven")
    else:  # the 8-GPU default protocol really ran, not the shared-GPU fallback
        assert r["mode_used"].startswith("stream-ordered+graph+fused+tokens-fenced"), r["mode_used"]
        assert "+program" not in r["mode_used"]
