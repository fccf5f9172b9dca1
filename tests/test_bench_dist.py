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
