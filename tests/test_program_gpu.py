"""GPU tier: programs (include/hiccl_reduce.h hiccl_program_*).

A program is ONE launch of signal/wait phases followed by a batch of
independent computes (exact byte copies from HICCL_BYTES plans, reductions
of the program's dtype); HiCCL::Comm records its stream-ordered pipeline as
a list of them.  The checks: no unit starts before the
last phase is satisfied (the host, as the peer, checks nothing was copied,
writes the source and then the flag while the program waits), consecutive programs see each other's
results, phases store / await their per-launch epochs (and epoch +
*epoch_dev under graph replay), relaunches reuse the gate word, a wait that
is never satisfied times out with the error word set while the grid still
drains, and the reductions give the oracle's bits.
"""
import ctypes

import numpy as np
import pytest
import torch

import hiccl_amd
from hiccl_amd import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _copy_plan(dst, src, nbytes, dst_off=0, src_off=0):
    c = hiccl_amd.Compute(torch.uint8, device=0)
    c.add([(src.view(torch.uint8), src_off)], (dst.view(torch.uint8), dst_off), nbytes, compid=0)
    return c


def _sum_plan(out, ins, count, dtype=torch.float32):
    c = hiccl_amd.Compute(dtype, device=0)
    c.add(list(ins), out, count, compid=0)
    return c


def _inorder(xs):
    acc = torch.zeros_like(xs[0])
    for x in xs:  # T acc = 0; acc += in[k][i] (compute.h:7-9), one rounding per add
        acc = acc + x
    return acc


def _host_coherent(nbytes):
    """Fine-grained (coherent) pinned host memory, mapped for the GPU at the
    same address: the host can play the peer -- its stores reach the waiting
    kernel with no GPU queue involved (hipHostMallocCoherent | Mapped)."""
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x40000000 | 0x2)) == 0
    return p.value, (lambda: hip.hipHostFree(p))


@pytest.mark.parametrize("peer", ["none", "put", "get"])
@pytest.mark.parametrize("count", [(1 << 18) + 3, (1 << 22) + 5], ids=["half_tiles", "full_tiles"])
def test_units_wait_for_the_phases(count, peer):
    """The program waits for a flag; the host plays the peer: while the
    program waits it checks that no copy unit has written yet, rewrites the
    copy's source, then sets the flag -- the copy (and the reduction of the
    same batch) must see the new source: no unit ran before the gate opened.
    Source, copy destination and flag live in coherent pinned host memory,
    so the peer needs no GPU queue (a second stream of this process may share
    the program's hardware queue and then waits behind it).  Three launches
    with new contents each time.  `peer`: the transport's peer policies
    carried into the program (an IPC put's system-scope stores or a get's
    system-scope loads for the copy, the fused gather's system-scope loads
    for the reduction)."""
    import time
    nb = count * 4
    sp, free_s = _host_coherent(nb)
    dp, free_d = _host_coherent(nb)
    fp, free_f = _host_coherent(256)
    src_np = np.ctypeslib.as_array((ctypes.c_float * count).from_address(sp))
    dst_np = np.ctypeslib.as_array((ctypes.c_float * count).from_address(dp))
    flag_np = np.ctypeslib.as_array((ctypes.c_int32 * 64).from_address(fp))
    flag_np[:] = 0
    src = torch.from_numpy(src_np)  # host tensors: the plans only take their addresses
    dst = torch.from_numpy(dst_np)
    b = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(b, 7, 1)
    out = torch.empty(count, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    cp = _copy_plan(dst, src, nb)
    red = _sum_plan(out, [src, b], count)
    if peer != "none":
        cp.set_peer(L.HICCL_PEER_STORES if peer == "put" else L.HICCL_PEER_LOADS)
        red.set_peer(L.HICCL_PEER_LOADS)
    prog = hiccl_amd.Program(torch.float32, device=0)
    prog.add_signal([], [fp])
    prog.add_plan(cp)
    prog.add_plan(red)
    assert prog.units() == 2 and prog.phases() == 1
    rng = np.random.default_rng(count)
    try:
        for it in range(3):
            src_np[:] = rng.standard_normal(count, dtype=np.float32)
            dst_np[:] = np.nan
            prog.launch([it + 1], err=err.data_ptr(), timeout_s=20.0)
            time.sleep(0.05)
            assert np.isnan(dst_np).all(), f"launch {it}: a copy unit ran before the gate opened"
            new = rng.standard_normal(count, dtype=np.float32)
            src_np[:] = new  # the "peer": new data, then the token
            flag_np[0] = it + 1
            torch.cuda.synchronize()
            assert err.item() == 0
            assert np.array_equal(dst_np.view(np.int32), new.view(np.int32)), f"launch {it}: stale source copied"
            exp = torch.from_numpy(new).to(DEV)
            assert torch.equal(out.view(torch.int32), _inorder([exp, b]).view(torch.int32))
    finally:
        torch.cuda.synchronize()
        prog.close()
        cp.close()
        red.close()
        free_s()
        free_d()
        free_f()


def test_chain_of_programs():
    """out_k = out_{k-1} + x_k as 12 programs in a row (each with a phase):
    every program sees the previous one's result (a kernel boundary)."""
    count = (1 << 20) + 7
    xs = [torch.empty(count, device=DEV) for _ in range(12)]
    for k, x in enumerate(xs):
        hiccl_amd.fill_uniform(x, 11, k)
    outs = [torch.empty(count, device=DEV) for _ in range(12)]
    flags = torch.zeros(16, dtype=torch.int32, device=DEV)
    progs, keep = [], []
    for k in range(12):
        c = _sum_plan(outs[k], [xs[k]] if k == 0 else [outs[k - 1], xs[k]], count)
        keep.append(c)
        pr = hiccl_amd.Program(torch.float32, device=0)
        f = flags.data_ptr() + 4 * k
        pr.add_signal([f], [f])
        pr.add_plan(c)
        progs.append(pr)
    for k, pr in enumerate(progs):
        pr.launch([40 + k])
    torch.cuda.synchronize()
    acc = torch.zeros(count, device=DEV)
    for k in range(12):
        acc = acc + xs[k]
        assert torch.equal(outs[k].view(torch.int32), acc.view(torch.int32)), f"program {k}"
    assert flags[:12].tolist() == [40 + k for k in range(12)]
    for pr in progs:
        pr.close()


def test_phases_store_and_await_epochs_and_relaunch():
    count = 1 << 16
    x = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(x, 3, 0)
    out = torch.empty(count, device=DEV)
    flags = torch.zeros(8, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    fa, fb = flags.data_ptr(), flags.data_ptr() + 4
    prog = hiccl_amd.Program(torch.float32, device=0)
    prog.add_signal([fa], [fa])
    prog.add_signal([fb], [fb])
    red = _sum_plan(out, [x, x], count)
    prog.add_plan(red)
    assert prog.phases() == 2 and prog.units() == 1
    with pytest.raises(hiccl_amd.HicclError):
        prog.add_signal([fa], [fa])  # phases precede the units
    for e in (5, 9, 13):
        prog.launch([e, e + 1], err=err.data_ptr(), timeout_s=5.0)
        torch.cuda.synchronize()
        assert flags[:2].tolist() == [e, e + 1]
        assert err.item() == 0
    assert torch.equal(out.view(torch.int32), (torch.zeros_like(x) + x + x).view(torch.int32))
    # a phases-only program (the trailing tokens of a pipeline)
    only = hiccl_amd.Program(torch.float32, device=0)
    only.add_signal([fa], [])
    only.launch([77])
    torch.cuda.synchronize()
    assert flags[0].item() == 77
    only.close()
    prog.close()


def test_unsatisfied_wait_times_out_and_drains():
    """A phase waiting for a flag nobody sets: after timeout_s the error word
    is set and the launch finishes (every later element still runs)."""
    count = 1 << 16
    x = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(x, 5, 0)
    out = torch.zeros(count, device=DEV)
    flags = torch.zeros(4, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    prog = hiccl_amd.Program(torch.float32, device=0)
    prog.add_signal([], [flags.data_ptr()])
    red = _sum_plan(out, [x], count)  # runs once the wait has given up
    prog.add_plan(red)
    prog.launch([1], err=err.data_ptr(), timeout_s=0.2)
    torch.cuda.synchronize()
    assert err.item() != 0
    assert torch.equal(out.view(torch.int32), (torch.zeros_like(x) + x).view(torch.int32))
    prog.close()


def test_graph_replay_reads_epoch_counter():
    """Eager launch first (uploads the tables), then the launch captured into
    a graph with epoch_dev: replay r stores / awaits epoch + r."""
    count = 1 << 16
    x = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(x, 9, 0)
    out = torch.empty(count, device=DEV)
    flags = torch.zeros(4, dtype=torch.int32, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int32, device=DEV)
    f = flags.data_ptr()
    prog = hiccl_amd.Program(torch.float32, device=0)
    prog.add_signal([f], [f])
    red = _sum_plan(out, [x, x, x], count)
    prog.add_plan(red)
    prog.launch([100])
    torch.cuda.synchronize()
    assert flags[0].item() == 100
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            cs = torch.cuda.current_stream()
            L.check(L.lib().hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1, ctypes.c_void_p(cs.cuda_stream)),
                    "counter_add")
            prog.launch([100], epoch_dev=ctr.data_ptr(), stream=cs)
    for r in range(1, 4):
        g.replay()
        torch.cuda.synchronize()
        assert ctr.item() == r and flags[0].item() == 100 + r
    exp = torch.zeros_like(x) + x + x + x
    assert torch.equal(out.view(torch.int32), exp.view(torch.int32))
    del g
    prog.close()


def test_gate_values_never_reused_across_captures():
    """The gate word a replay leaves behind never opens a later capture's gate
    early.  Graph A is replayed with its epoch counter far ahead (as after
    2^24 + 11 replays), so its gate value is high; graph B, captured next
    from the same program with a fresh counter, must still keep its units
    back until its phase is satisfied (the host plays the peer, as in
    test_units_wait_for_the_phases).  With 32-bit gate values reserved 2^24
    per capture and a >= test, B's workgroups passed the gate at once."""
    import time
    count = (1 << 18) + 3
    nb = count * 4
    sp, free_s = _host_coherent(nb)
    dp, free_d = _host_coherent(nb)
    fp, free_f = _host_coherent(256)
    src_np = np.ctypeslib.as_array((ctypes.c_float * count).from_address(sp))
    dst_np = np.ctypeslib.as_array((ctypes.c_float * count).from_address(dp))
    flag_np = np.ctypeslib.as_array((ctypes.c_int32 * 64).from_address(fp))
    flag_np[:] = 0
    src, dst = torch.from_numpy(src_np), torch.from_numpy(dst_np)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    cp = _copy_plan(dst, src, nb)
    prog = hiccl_amd.Program(torch.float32, device=0)
    prog.add_signal([], [fp])
    prog.add_plan(cp)
    ctr_a = torch.zeros(1, dtype=torch.int32, device=DEV)
    ctr_b = torch.zeros(1, dtype=torch.int32, device=DEV)
    s = torch.cuda.Stream()

    def capture(ctr, epoch):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                cs = torch.cuda.current_stream()
                L.check(L.lib().hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 1,
                                                  ctypes.c_void_p(cs.cuda_stream)), "counter_add")
                prog.launch([epoch], epoch_dev=ctr.data_ptr(), err=err.data_ptr(), timeout_s=20.0, stream=cs)
        return g

    try:
        flag_np[0] = 1
        prog.launch([1], err=err.data_ptr(), timeout_s=20.0)  # eager: uploads
        torch.cuda.synchronize()
        ga = capture(ctr_a, 10)
        ctr_a.fill_((1 << 24) + 10)  # replay A as its (2^24 + 11)-th
        flag_np[0] = 10 + (1 << 24) + 11
        ga.replay()
        torch.cuda.synchronize()
        assert err.item() == 0
        base = 1 << 25  # B's token epochs: above every flag value so far
        gb = capture(ctr_b, base)
        rng = np.random.default_rng(5)
        for r in range(1, 3):
            src_np[:] = rng.standard_normal(count, dtype=np.float32)
            dst_np[:] = np.nan
            gb.replay()
            time.sleep(0.05)
            assert np.isnan(dst_np).all(), f"replay {r} of B: a unit ran before its gate opened"
            new = rng.standard_normal(count, dtype=np.float32)
            src_np[:] = new
            flag_np[0] = base + r
            torch.cuda.synchronize()
            assert err.item() == 0
            assert np.array_equal(dst_np.view(np.int32), new.view(np.int32)), f"replay {r} of B: stale source"
        del ga, gb
    finally:
        torch.cuda.synchronize()
        prog.close()
        cp.close()
        free_s()
        free_d()
        free_f()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float64, torch.int64], ids=["bf16", "f64", "u64"])
def test_program_dtypes_match_oracle(oracle, dtype):
    count = (1 << 17) + 9
    n = 5
    fill_as = torch.float64 if dtype == torch.int64 else dtype
    ins = [torch.empty(count, dtype=fill_as, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, 21, k)
    ins = [t.view(dtype) for t in ins]
    out = torch.empty(count, dtype=dtype, device=DEV)
    prog = hiccl_amd.Program(dtype, device=0)
    red = _sum_plan(out, ins, count, dtype)
    prog.add_plan(red)
    prog.launch()
    ref = torch.empty_like(out)
    hiccl_amd.reduce(ref, ins)
    torch.cuda.synchronize()
    iv = {torch.bfloat16: torch.int16, torch.float64: torch.int64, torch.int64: torch.int64}[dtype]
    assert torch.equal(out.view(iv), ref.view(iv))
    if dtype == torch.float64:
        host = np.stack([t.cpu().numpy() for t in ins])
        exp = oracle.reduce(host)
        assert np.array_equal(out.cpu().numpy().view(np.uint64), exp.view(np.uint64))
    prog.close()


def test_batch_of_plans_and_refusals():
    count = 1 << 18
    a = torch.empty(count, device=DEV)
    b = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(a, 1, 0)
    hiccl_amd.fill_uniform(b, 1, 1)
    o1 = torch.empty(count, device=DEV)
    o2 = torch.empty(count, device=DEV)
    prog = hiccl_amd.Program(torch.float32, device=0)
    p1, p2 = _sum_plan(o1, [a, b], count), _sum_plan(o2, [b, a], count)
    prog.add_plan(p1)
    prog.add_plan(p2)
    assert prog.units() == 2
    prog.launch()
    torch.cuda.synchronize()
    assert torch.equal(o1.view(torch.int32), _inorder([a, b]).view(torch.int32))
    assert torch.equal(o2.view(torch.int32), _inorder([b, a]).view(torch.int32))
    # a plan of another reduction dtype is refused (bytes plans are accepted)
    bad = _sum_plan(torch.empty(count, dtype=torch.float64, device=DEV),
                    [torch.zeros(count, dtype=torch.float64, device=DEV)], count, torch.float64)
    with pytest.raises(hiccl_amd.HicclError):
        prog.add_plan(bad)
    prog.close()
