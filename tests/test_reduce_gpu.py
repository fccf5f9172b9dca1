"""GPU tier: the HIP kernels through the C ABI vs the oracle and the golden
fixtures (bit-exact; NaN outputs compared by NaN-ness).

Covers the edge cases SURVEY.md sections 4 and 8a list: n = 0, 1, 2, 3, 4, 7,
8, 9, 16, 64 and > 64 (device pointer table), counts around the packet/tile
boundaries, signed zeros / Inf / NaN / denormals / overflow, mutually
misaligned inputs (partition() element offsets), in-place outputs, bf16 in
both accumulation modes, size_t known-answer, the batched plan vs the
reference's one-launch-per-compute structure, and a full-size sampled check.
"""
import ctypes

import numpy as np
import pytest
import torch

import auto_table as A
import hiccl_amd
from conftest import bits_equal, first_mismatch, load_golden
from hiccl_amd import _lib as L

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
# Both kernel engines compute the same bits; every edge-case test runs under
# the default (auto: tile for these small sizes) and the forced phased engine.
PHASE = dict(engine=hiccl_amd.HICCL_ENGINE_PHASE)
ENGINES = pytest.mark.parametrize("eng", [None, PHASE], ids=["auto", "phase"])
TORCH_OF = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
            np.dtype(np.uint64): torch.int64, np.dtype(np.uint16): torch.bfloat16, np.dtype(np.int32): torch.int32}


def to_dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).to(DEV)
    if a.dtype == np.uint64:
        return torch.from_numpy(a.view(np.int64).copy()).to(DEV)
    return torch.from_numpy(a.copy()).to(DEV)


def to_host(t, np_dtype):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).cpu().numpy().view(np.uint16)
    if np.dtype(np_dtype) == np.uint64:
        return t.cpu().numpy().view(np.uint64)
    return t.cpu().numpy()


def gpu_reduce(x, count, dtype, offsets=None, out_offset=0, config=None):
    """Place each input row at an element offset inside its own buffer and
    reduce; returns the host result."""
    n = x.shape[0]
    tdt = TORCH_OF[np.dtype(dtype)]
    offsets = offsets or [0] * n
    bufs = []
    ins = []
    for k in range(n):
        b = torch.empty(count + offsets[k] + 8, dtype=tdt, device=DEV)
        b.view(torch.uint8).fill_(0x5A)
        seg = b[offsets[k]:offsets[k] + count]
        seg.copy_(to_dev(x[k]).view(tdt) if count else seg)
        bufs.append(b)
        ins.append(seg)
    ob = torch.empty(count + out_offset + 8, dtype=tdt, device=DEV)
    ob.view(torch.uint8).fill_(0xA5)
    out = ob[out_offset:out_offset + count]
    hiccl_amd.reduce(out, ins, count=count, config=config)
    torch.cuda.synchronize()
    # guard bytes around the output must be untouched
    guard = to_host(ob, dtype)
    assert (guard[:out_offset].view(np.uint8) == 0xA5).all()
    assert (guard[out_offset + count:].view(np.uint8) == 0xA5).all()
    return to_host(out, dtype)


@pytest.mark.parametrize("name,dtype", [("reduce_f32", np.float32), ("reduce_f64", np.float64),
                                        ("reduce_u64", np.uint64), ("reduce_bf16", np.uint16),
                                        ("reduce_i32", np.int32)])
@ENGINES
def test_golden_fixtures(name, dtype, eng):
    for case, d in load_golden(name).items():
        x, y = d["in"], d["out"]
        got = gpu_reduce(x, len(y), dtype, config=eng)
        assert bits_equal(got, y), f"{name}/{case}: {first_mismatch(got, y)}"


@pytest.mark.parametrize("offs", [[1, 0], [0, 3], [1, 2, 3, 0], [3, 3, 3], [2, 1, 0, 3, 2, 1, 0, 3, 1]])
@pytest.mark.parametrize("out_off", [0, 1, 3])
@ENGINES
def test_misaligned_inputs_f32(oracle, offs, out_off, eng):
    n = len(offs)
    for count in (1, 5, 4099, 70001):
        x = oracle.fill(n, count, seed=11 + count)
        got = gpu_reduce(x, count, np.float32, offsets=offs, out_offset=out_off, config=eng)
        exp = oracle.reduce(list(x))
        assert bits_equal(got, exp), f"offs={offs} out={out_off} count={count}: {first_mismatch(got, exp)}"


@pytest.mark.parametrize("offs", [[1, 0, 5], [7, 3], [0, 0, 1, 2, 3, 4, 5, 6]])
@ENGINES
def test_misaligned_inputs_bf16(oracle, offs, eng):
    n = len(offs)
    for count in (3, 9, 4099, 33333):
        x = oracle.fill(n, count, seed=5, dtype=np.uint16)
        got = gpu_reduce(x, count, np.uint16, offsets=offs, out_offset=1, config=eng)
        exp = oracle.reduce(list(x), dtype=np.uint16)
        assert bits_equal(got, exp), f"offs={offs} count={count}: {first_mismatch(got, exp)}"


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 6, 7, 8, 9, 15, 16, 17, 31, 64, 65, 100, 200])
@ENGINES
def test_input_counts(oracle, n, eng):
    count = 3 * 4096 + 77
    x = oracle.fill(n, count, seed=n) if n else np.zeros((0, count), np.float32)
    got = gpu_reduce(x, count, np.float32, config=eng)
    exp = oracle.reduce(list(x), count=count, dtype=np.float32)
    assert bits_equal(got, exp), f"n={n}: {first_mismatch(got, exp)}"


@pytest.mark.parametrize("count", [1, 2, 3, 4, 5, 511, 512, 513, 2047, 2048, 2049, 8191, 8192, 8193,
                                   131072 * 4 + 3])
@ENGINES
def test_tile_boundaries(oracle, count, eng):
    x = oracle.fill(4, count, seed=3)
    got = gpu_reduce(x, count, np.float32, config=eng)
    assert bits_equal(got, oracle.reduce(list(x)))


@pytest.mark.parametrize("count", [8192 * 4 - 1, 8192 * 4, 8192 * 4 + 1, 8192 * 4 * 3 + 5,
                                   65536 - 1, 65536 + 1, 32768 * 4 * 2 + 4 * 1000 + 3])
@pytest.mark.parametrize("n", [1, 2, 7, 8])
def test_phase_chunk_boundaries(oracle, count, n):
    """Phased chunks are 512 x 16 packets (f32: 32768 elements; bf16:
    65536 elements): partial last chunks, odd/even n."""
    x = oracle.fill(n, count, seed=count + n)
    got = gpu_reduce(x, count, np.float32, offsets=[1] + [0] * (n - 1), config=PHASE)
    assert bits_equal(got, oracle.reduce(list(x)))
    xb = oracle.fill(n, count, seed=count, dtype=np.uint16)
    gotb = gpu_reduce(xb, count, np.uint16, config=PHASE)
    assert bits_equal(gotb, oracle.reduce(list(xb), dtype=np.uint16))


@pytest.mark.parametrize("config", [
    dict(engine=2), dict(engine=2, block=1024, unroll=4), dict(engine=2, block=512, unroll=8),
    dict(engine=2, block=1024, unroll=8), dict(engine=2, block=256, unroll=16),
    dict(engine=2, nontemporal=1, store_policy=1), dict(engine=2, nontemporal=2, store_policy=3),
    dict(engine=2, nontemporal=1), dict(engine=2, grid=5), dict(engine=2, blocks_per_cu=2)])
def test_phase_variants_same_bits(oracle, config):
    """Every instantiated phased shape / cache policy gives the reference bits
    (f32; bf16 where the shape exists for bf16)."""
    bf16_ok = True  # bf16 (packed accumulator) has the f32 shape table
    for n, count in ((8, (1 << 20) + 3), (3, 123457), (1, 77777)):
        x = oracle.fill(n, count, seed=n)
        got = gpu_reduce(x, count, np.float32, offsets=[0, 1, 2][:n] + [0] * (n - 3), config=config)
        assert bits_equal(got, oracle.reduce(list(x))), config
        if bf16_ok:
            xb = oracle.fill(n, count, seed=n, dtype=np.uint16)
            gotb = gpu_reduce(xb, count, np.uint16, config=config)
            assert bits_equal(gotb, oracle.reduce(list(xb), dtype=np.uint16)), config


@pytest.mark.parametrize("engine", [1, 2], ids=["tile", "phase"])
@pytest.mark.parametrize("grid", [1, 2])
def test_dynamic_schedule_same_bits(oracle, engine, grid):
    """Dynamic unit scheduling (device ticket counter, reset by the launch
    itself) against static, repeated launches on one stream (the counter
    must come back to zero each time: a stale counter would skip units and
    leave the NaN prefill), and a second stream (its own counter)."""
    S = hiccl_amd._lib
    # >= 32 tickets per workgroup (the dynamic threshold): 64+ phased chunks
    for n, count in ((8, (1 << 21) + 5), (3, (1 << 21) + 33333)):
        x = oracle.fill(n, count, seed=n + grid)
        exp = oracle.reduce(list(x))
        ins = [to_dev(r) for r in x]
        out = torch.empty(count, device=DEV)
        side = torch.cuda.Stream()
        for sched in (S.HICCL_SCHED_STATIC, S.HICCL_SCHED_DYNAMIC):
            cfg = dict(engine=engine, grid=grid, schedule=sched, grab=1)
            for rep in range(5):
                out.fill_(float("nan"))
                hiccl_amd.reduce(out, ins, config=cfg)
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                assert bits_equal(got, exp), (sched, rep, first_mismatch(got, exp))
            side.wait_stream(torch.cuda.current_stream())
            out.fill_(float("nan"))
            torch.cuda.current_stream().synchronize()
            hiccl_amd.reduce(out, ins, config=cfg, stream=side)
            side.synchronize()
            got = out.cpu().numpy()
            assert bits_equal(got, exp), (sched, "side stream", first_mismatch(got, exp))


def test_dynamic_schedule_plan_many_computes(oracle):
    """An AUTO plan big enough for the dynamic schedule (tile engine, mean n
    >= 5, >= 32 tickets per workgroup of 256), many computes of ragged
    sizes, launched 3 times."""
    rng = np.random.default_rng(11)
    comp = hiccl_amd.Compute(torch.float32, device=0)
    outs, exps, keep = [], [], []
    for c in range(300):
        n = int(rng.integers(5, 10))
        count = int(rng.integers(1, 600000))  # ~11,000 two-tile tickets
        x = oracle.fill(n, count, seed=500 + c)
        ins = [to_dev(r) for r in x]
        keep += ins
        out = torch.empty(count, device=DEV)
        comp.add(ins, out, count, compid=0)
        outs.append(out)
        exps.append(oracle.reduce(list(x)))
    for _ in range(3):
        for o in outs:
            o.fill_(float("nan"))
        comp.start()
        comp.wait()
        for o, e in zip(outs, exps):
            got = o.cpu().numpy()
            assert bits_equal(got, e), first_mismatch(got, e)
    comp.close()


@pytest.mark.parametrize("eng", [None, PHASE], ids=["auto", "phase"])
def test_graph_capture_replay(oracle, eng):
    """hiccl_reduce captured into a HIP graph (torch.cuda.graph) and
    replayed with new input values: during capture the library takes the
    static schedule (a replayed graph must not share a stream's ticket
    counter), and every replay gives the reference bits."""
    n, count = 8, (1 << 24) + 3  # big enough that AUTO would go dynamic uncaptured
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    out = torch.empty(count, device=DEV)
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, 1, k)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hiccl_amd.reduce(out, ins, config=eng)  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        hiccl_amd.reduce(out, ins, config=eng)
    rng = np.random.default_rng(5)
    for seed in (11, 12, 13):
        for k, t in enumerate(ins):
            hiccl_amd.fill_uniform(t, seed, k)
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        idx = np.concatenate([np.arange(16), count - 16 + np.arange(16),
                              rng.integers(0, count, 2048)]).astype(np.int64)
        got = out[torch.from_numpy(idx).to(DEV)].cpu().numpy()
        exp = oracle.sample_sum(idx.astype(np.uint64), seed, n)
        assert bits_equal(got, exp), (seed, first_mismatch(got, exp))


def test_phase_unsupported_shape_is_an_error():
    x = torch.zeros(100, device=DEV)
    with pytest.raises(hiccl_amd.HicclError):
        hiccl_amd.reduce(x, [x, x], config=dict(engine=2, block=128, unroll=16))
    with pytest.raises(hiccl_amd.HicclError):
        hiccl_amd.reduce(x, [x, x], config=dict(engine=7))
    with pytest.raises(hiccl_amd.HicclError):
        hiccl_amd.reduce(x, [x, x], config=dict(schedule=9))


def test_python_reduce_argument_checks():
    x = torch.zeros(100, device=DEV)
    with pytest.raises(ValueError, match="count"):
        hiccl_amd.reduce(x, [x], count=-1)
    with pytest.raises(ValueError, match="device tensor"):
        hiccl_amd.reduce(x, [x.cpu()])
    with pytest.raises(ValueError, match="< count"):
        hiccl_amd.reduce(x, [x[:50]], count=100)


@pytest.mark.parametrize("config", [
    dict(block=256, unroll=1), dict(block=256, unroll=2), dict(block=256, unroll=4),
    dict(block=512, unroll=1), dict(block=512, unroll=2), dict(block=512, unroll=4),
    dict(block=256, unroll=2, nontemporal=1), dict(block=256, unroll=2, nontemporal=2, store_policy=2),
    dict(block=256, unroll=4, nontemporal=1, store_policy=3, grid=192),
    dict(block=512, unroll=4, nontemporal=2, store_policy=2, blocks_per_cu=2),
    dict(block=256, unroll=1, grid=7), dict(block=256, unroll=8), dict(block=256, unroll=16),
    dict(block=256, unroll=8, schedule=2, grab=1, grid=3), dict(block=256, unroll=16, grid=5),
    # tile order interleaved over 2^L stretches (a bijection for any tile count; static and dynamic)
    dict(order=2), dict(order=8, grid=3), dict(order=64, schedule=2, grab=1, grid=5), dict(order=4096, unroll=1),
    dict(order=16, engine=2)])
def test_tuning_variants_same_bits(oracle, config):
    for n, count in ((8, 1 << 20), (3, 123457)):
        x = oracle.fill(n, count, seed=n)
        got = gpu_reduce(x, count, np.float32, offsets=[0, 1] + [0] * (n - 2), config=config)
        assert bits_equal(got, oracle.reduce(list(x))), config
        xb = oracle.fill(n, count, seed=n, dtype=np.uint16)
        gotb = gpu_reduce(xb, count, np.uint16, config=config)
        assert bits_equal(gotb, oracle.reduce(list(xb), dtype=np.uint16)), config


@ENGINES
def test_in_place_output(oracle, eng):
    n, count = 4, 100003
    x = oracle.fill(n, count, seed=9)
    ins = [to_dev(r) for r in x]
    for k in range(n):  # out aliases input k exactly
        t = [i.clone() for i in ins]
        hiccl_amd.reduce(t[k], t, count=count, config=eng)
        torch.cuda.synchronize()
        assert bits_equal(t[k].cpu().numpy(), oracle.reduce(list(x))), k


@ENGINES
def test_in_place_large_n_table_path(oracle, eng):
    n, count = 80, 20011
    x = oracle.fill(n, count, seed=1)
    t = [to_dev(r) for r in x]
    hiccl_amd.reduce(t[70], t, count=count, config=eng)
    torch.cuda.synchronize()
    assert bits_equal(t[70].cpu().numpy(), oracle.reduce(list(x)))


@ENGINES
def test_bf16_wide_accumulation(oracle, eng):
    n, count = 8, 50001
    x = oracle.fill(n, count, seed=2, dtype=np.uint16)
    got = gpu_reduce(x, count, np.uint16, config=dict(acc=hiccl_amd.HICCL_ACC_WIDE, **(eng or {})))
    exp = oracle.reduce(list(x), dtype=np.uint16, wide=True)
    assert bits_equal(got, exp), first_mismatch(got, exp)


@ENGINES
def test_int32_wraparound(oracle, eng):
    rng = np.random.default_rng(0)
    x = rng.integers(-2**31, 2**31 - 1, size=(5, 10007), dtype=np.int64).astype(np.int32)
    ins = [torch.from_numpy(r.copy()).to(DEV) for r in x]
    out = torch.empty(10007, dtype=torch.int32, device=DEV)
    hiccl_amd.reduce(out, ins, config=eng)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.reduce(list(x)))


def test_generator_matches_oracle(oracle):
    for dtype, tdt in ((np.float32, torch.float32), (np.uint16, torch.bfloat16), (np.float64, torch.float64)):
        t = torch.empty(100003, dtype=tdt, device=DEV)
        hiccl_amd.fill_uniform(t, seed=1234, k=5, first=17)
        torch.cuda.synchronize()
        exp = oracle.fill(6, 100003, 1234, dtype=dtype, first=17)[5]
        assert bits_equal(to_host(t, dtype), exp), dtype


def _plan_case(oracle, each, engine=hiccl_amd.HICCL_ENGINE_AUTO):
    rng = np.random.default_rng(4)
    comp = hiccl_amd.Compute(torch.float32, device=0, engine=engine)
    expected = []
    outs = []
    keep = []
    for c in range(37):
        n = int(rng.integers(1, 12))
        count = int(rng.integers(1, 70000))
        offs = [int(o) for o in rng.integers(0, 4, size=n)]
        x = oracle.fill(n, count, seed=100 + c)
        ins = []
        for k in range(n):
            b = torch.empty(count + offs[k], device=DEV)
            b[offs[k]:].copy_(torch.from_numpy(x[k]))
            ins.append((b, offs[k]))
            keep.append(b)
        ob = torch.full((count + 2,), float("nan"), device=DEV)
        comp.add(ins, (ob, 1), count, compid=0)
        outs.append((ob, count))
        expected.append(oracle.reduce(list(x)))
    comp.add([(keep[0], 0)], (keep[0], 0), 1, compid=3)  # not mine: ignored (compute.h:66)
    assert comp.numcomp == 37
    comp.start(each=each)
    comp.wait()
    if not each:  # launch_each runs one-shot launches and leaves the plan's table alone
        assert comp.engine() == (hiccl_amd.HICCL_ENGINE_TILE if engine == hiccl_amd.HICCL_ENGINE_AUTO else engine)
    for (ob, count), exp in zip(outs, expected):
        got = ob[1:1 + count].cpu().numpy()
        assert bits_equal(got, exp), first_mismatch(got, exp)
        assert np.isnan(ob[0].item()) and np.isnan(ob[count + 1].item())
    # a second launch of the same plan gives the same bits
    comp.start()
    comp.wait()
    assert bits_equal(outs[0][0][1:1 + outs[0][1]].cpu().numpy(), expected[0])
    comp.close()


def test_plan_batched(oracle):
    _plan_case(oracle, each=False)


def test_plan_launch_each(oracle):
    _plan_case(oracle, each=True)


@pytest.mark.parametrize("each", [False, True])
def test_plan_phase_engine(oracle, each):
    _plan_case(oracle, each=each, engine=hiccl_amd.HICCL_ENGINE_PHASE)


def test_plan_auto_engine_picks_phase_for_large_buckets(oracle):
    """f32 AUTO (round 3, profiles/r03n_midsize.jsonl): TILE with >= 5 inputs
    from 64 tickets per workgroup (n = 6: two tiles per ticket, 2^27 f32 per
    input on 256 CUs); below that, with >= 5 inputs, PHASE once every CU gets
    a 128 KiB chunk (2^23 f32 per input) and the last round of chunks keeps
    >= 70 % of the CUs busy (n = 8 at 1.25 chunks per CU: TILE); with 3-4
    inputs PHASE from 4 chunks per CU in whole-enough rounds (~90 %),
    with 2 inputs from 16; TILE otherwise.  Round 5: three f32 inputs take
    static tiles when the launch stores write-through (its store form left
    to size, <= 256 MiB written); with nt stores asked for, the table above."""
    a = torch.empty(1 << 27, device=DEV)
    hiccl_amd.fill_uniform(a, 77, 0)
    out = torch.empty(1 << 27, device=DEV)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for (dt, cnt, n, cfg), expect in A.GPU_PLAN_ENGINE_F32:  # one table with the CPU tier's check
        comp = hiccl_amd.Compute(torch.float32, device=0, config=cfg)
        comp.add([a] * n, out, cnt, compid=0)
        comp.start()
        comp.wait()
        assert comp.engine() == hiccl_amd.auto_choice(dt, cnt, n, config=cfg, cus=cus)["engine"]
        if cus == 256:
            assert comp.engine() == expect
        idx = np.array([0, 1, cnt // 2, cnt - 1], np.int64)
        exp = oracle.sample_sum(idx.astype(np.uint64), 77, 1)
        got = out[torch.from_numpy(idx).to(DEV)].cpu().numpy()
        ref = np.zeros_like(exp)
        for _ in range(n):
            ref = (ref + exp).astype(np.float32)
        assert bits_equal(got, ref)
        comp.close()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("n", [2, 3, 4])
def test_auto_wide_tiles_large_few_inputs(oracle, dtype, n):
    """AUTO at 1 GiB per input with 2-4 inputs: TILE with 32 KiB-per-input
    tiles on the dynamic schedule (plan and one-shot), bit-exact vs the
    in-order sum (sampled) and vs the forced phased engine."""
    esz = 2 if dtype == torch.bfloat16 else 4
    count = (1 << 30) // esz
    base = torch.empty(count + 8, dtype=dtype, device=DEV)
    hiccl_amd.fill_uniform(base, 55 + n, 0)
    ins = [(base, k) for k in range(n)]  # mutually misaligned views of one buffer
    outs = {}
    for name, eng in (("auto", hiccl_amd.HICCL_ENGINE_AUTO), ("phase", hiccl_amd.HICCL_ENGINE_PHASE)):
        out = torch.empty(count, dtype=dtype, device=DEV)
        comp = hiccl_amd.Compute(dtype, device=0, engine=eng)
        comp.add(ins, out, count, compid=0)
        comp.start()
        comp.wait()
        if name == "auto" and torch.cuda.get_device_properties(0).multi_processor_count == 256:
            want = dict(((dt, c, nn), w) for (dt, c, nn, _), w in A.GPU_WIDE_TILES)[
                (L.DTYPE_OF_TORCH[dtype], count, n)]
            assert comp.engine() == want
        comp.close()
        outs[name] = out
    one = torch.empty(count, dtype=dtype, device=DEV)
    hiccl_amd.reduce(one, [base[k:k + count] for k in range(n)])
    torch.cuda.synchronize()
    iv = lambda t: t.view(torch.int16 if dtype == torch.bfloat16 else torch.int32)  # noqa: E731
    assert torch.equal(iv(outs["auto"]), iv(outs["phase"]))
    assert torch.equal(iv(outs["auto"]), iv(one))
    idx = torch.randint(0, count, (4096,), generator=torch.Generator().manual_seed(n))
    idx[:2] = torch.tensor([0, count - 1])
    host = base.cpu()
    acc = torch.zeros(idx.numel(), dtype=dtype)
    for k in range(n):  # T acc = 0; acc += in[k][i] (compute.h:7-9)
        acc = (acc.float() + host[idx + k].float()).to(dtype)
    assert torch.equal(iv(outs["auto"][idx.to(DEV)].cpu()), iv(acc))


@pytest.mark.parametrize("config", [dict(block=512), dict(nontemporal=1), dict(store_policy=1),
                                    dict(block=256, nontemporal=1)],
                         ids=["block512", "nt_off", "store_plain", "block256_nt_off"])
def test_wide_tile_size_with_caller_shape_runs(oracle, config):
    """1 GiB per input x 2 inputs is where AUTO picks wide tiles (U = 16), a
    shape that exists only at block 256 with nt loads and stores.  A caller
    asking for another block or cache policy at that size must still run
    (u4 / PHASE, not 'unsupported config'), bit-exact vs the default call."""
    count = 1 << 28
    a = torch.empty(count, device=DEV)
    b = torch.empty(count, device=DEV)
    hiccl_amd.fill_uniform(a, 91, 0)
    hiccl_amd.fill_uniform(b, 91, 1)
    ref = torch.empty(count, device=DEV)
    hiccl_amd.reduce(ref, [a, b])
    out = torch.empty(count, device=DEV)
    hiccl_amd.reduce(out, [a, b], config=config)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    idx = torch.tensor([0, 1, count // 2, count - 1], device=DEV)
    exp = ((torch.zeros(4, device=DEV) + a[idx]) + b[idx])
    assert torch.equal(out[idx].view(torch.int32), exp.view(torch.int32))


def test_plan_auto_engine_bf16():
    """bf16 with >= 5 inputs: AUTO takes TILE only from 64 tickets per
    workgroup (n = 8: 2^27 elements per input on 256 CUs) and above the
    write-through cap (round 5: at 2^27 a launch writes 256 MiB and stores
    write-through, where PHASE leads), PHASE below; either engine gives the
    other's bits, and the result matches an in-order bf16 sum on the host
    (sampled)."""
    P, T = hiccl_amd.HICCL_ENGINE_PHASE, hiccl_amd.HICCL_ENGINE_TILE
    big = 1 << 28
    base = torch.empty(big + 64, dtype=torch.bfloat16, device=DEV)
    hiccl_amd.fill_uniform(base, 91, 0)
    offs = (0, 0, 1, 3, 0, 2, 7, 5)
    full = 256 == torch.cuda.get_device_properties(0).multi_processor_count
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for (dt, cnt, n, cfg), expect in A.GPU_PLAN_ENGINE_BF16:  # one table with the CPU tier's check
        assert n == len(offs) and cfg is None
        other = T if expect == P else P
        ins = [(base, o) for o in offs]
        outs = []
        for eng in (hiccl_amd.HICCL_ENGINE_AUTO, other):
            out = torch.empty(cnt, dtype=torch.bfloat16, device=DEV)
            comp = hiccl_amd.Compute(torch.bfloat16, device=0, engine=eng)
            comp.add(ins, out, cnt, compid=0)
            comp.start()
            comp.wait()
            if eng == hiccl_amd.HICCL_ENGINE_AUTO:
                assert comp.engine() == hiccl_amd.auto_choice(dt, cnt, n, cus=cus)["engine"]
                if full:
                    assert comp.engine() == expect
            comp.close()
            outs.append(out)
        assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
        idx = torch.randint(0, cnt, (4096,), generator=torch.Generator().manual_seed(cnt % 97))
        host = base.cpu()
        acc = torch.zeros(idx.numel(), dtype=torch.bfloat16)
        for o in offs:  # reduce_kernel<T>: T acc = 0; acc += in[k][i] (compute.h:2-12)
            acc = (acc.float() + host[idx + o].float()).to(torch.bfloat16)
        got = outs[0][idx.to(DEV)].cpu()
        assert torch.equal(got.view(torch.int16), acc.view(torch.int16))
        del outs


def test_plan_launch_from_other_thread(oracle):
    """Comm::start runs compute->start() on a pthread (comm.h:214-224)."""
    import threading
    x = oracle.fill(3, 4099, seed=8)
    ins = [to_dev(r) for r in x]
    out = torch.empty(4099, device=DEV)
    comp = hiccl_amd.Compute(torch.float32, device=0)
    comp.add(ins, out, 4099, compid=0)
    th = threading.Thread(target=lambda: (comp.start(), comp.wait()))
    th.start()
    th.join()
    assert bits_equal(out.cpu().numpy(), oracle.reduce(list(x)))


@pytest.mark.parametrize("count", [1 << 28, 250_000_000], ids=["2^28", "readme_2.5e8"])
@pytest.mark.parametrize("eng", [None, dict(engine=hiccl_amd.HICCL_ENGINE_TILE)], ids=["auto", "tile"])
def test_full_size_sampled(oracle, count, eng):
    """Config 2 shape (8 x 2^28 f32, and the README's 1e9/sizeof(float)
    count for tail handling) checked at 4096 random indices plus the ends: a
    size-independent property check against the oracle's generator."""
    n, seed = 8, 1234
    free, _ = torch.cuda.mem_get_info()
    if free < (n + 2) * count * 4:
        pytest.skip("not enough device memory")
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, device=DEV)
    hiccl_amd.reduce(out, ins, config=eng)
    torch.cuda.synchronize()
    rng = np.random.default_rng(0)
    idx = np.concatenate([np.arange(64), count - 64 + np.arange(64),
                          rng.integers(0, count, 4096)]).astype(np.int64)
    got = out[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    exp = oracle.sample_sum(idx.astype(np.uint64), seed, n)
    assert bits_equal(got, exp), first_mismatch(got, exp)
    # checksum-of-checksums: the sum of the output equals the sum of the oracle
    # partial sums over a strided sample (catches whole-tile drops)
    stride = 997
    idx2 = np.arange(0, count, stride * 1024, dtype=np.int64)
    got2 = out[torch.from_numpy(idx2).to(DEV)].cpu().numpy()
    assert bits_equal(got2, oracle.sample_sum(idx2.astype(np.uint64), seed, n))


@pytest.mark.parametrize("n,log2count", [(2, 24), (5, 24), (16, 23), (64, 22)])
@pytest.mark.parametrize("eng", [None, PHASE, dict(engine=hiccl_amd.HICCL_ENGINE_TILE)],
                         ids=["auto", "phase", "tile"])
def test_nway_sampled(oracle, n, log2count, eng):
    """Config-3 shapes (N-way sweep) at 16-64 MiB per input: 4096 sampled
    indices + both ends against the oracle generator, every engine."""
    count, seed = (1 << log2count) + 7, 99
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, device=DEV)
    hiccl_amd.reduce(out, ins, config=eng)
    torch.cuda.synchronize()
    rng = np.random.default_rng(n)
    idx = np.concatenate([np.arange(40), count - 40 + np.arange(40),
                          rng.integers(0, count, 4096)]).astype(np.int64)
    got = out[torch.from_numpy(idx).to(DEV)].cpu().numpy()
    exp = oracle.sample_sum(idx.astype(np.uint64), seed, n)
    assert bits_equal(got, exp), first_mismatch(got, exp)


@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
@pytest.mark.parametrize("engine", [hiccl_amd.HICCL_ENGINE_AUTO, hiccl_amd.HICCL_ENGINE_PHASE])
def test_plan_partitioned_on_default_stream(oracle, dtype, engine):
    """Config-4 layout: one bucket split into pipedepth computes with the
    partition() formula (reduce.h:401-415: count/numbatch + (b < count%numbatch)),
    launched as ONE batched kernel on torch's (NULL) default stream."""
    n, count, depth = 8, 3 * 65536 + 1234, 7
    tdt = TORCH_OF[np.dtype(dtype)]
    x = oracle.fill(n, count, seed=21, dtype=dtype)
    ins = [to_dev(r).view(tdt) for r in x]
    out = torch.full((count,), 7.0, dtype=tdt, device=DEV)
    comp = hiccl_amd.Compute(tdt, device=0, engine=engine)
    off = 0
    for b in range(depth):
        c = count // depth + (1 if b < count % depth else 0)
        comp.add([(t, off) for t in ins], (out, off), c, compid=0)
        off += c
    assert off == count
    for each in (False, True):
        out.fill_(7.0)
        comp.start(stream=torch.cuda.current_stream(), each=each)
        torch.cuda.synchronize()
        got = to_host(out, dtype)
        exp = oracle.reduce(list(x), dtype=dtype)
        assert bits_equal(got, exp), (each, first_mismatch(got, exp))
    comp.close()


@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 4099, 1 << 20, (1 << 22) + 7])
def test_byte_copy_exact(nbytes):
    """HICCL_BYTES: an exact copy (NaN payloads and -0 preserved), any byte
    offsets, one launch for a batch of copies (the transport's data path)."""
    rng = np.random.default_rng(nbytes)
    src = torch.from_numpy(rng.integers(0, 256, nbytes + 64, dtype=np.uint8)).to(DEV)
    import ctypes
    from hiccl_amd import _lib as L
    lib = L.lib()
    plan = ctypes.c_void_p()
    assert lib.hiccl_reduce_plan_create(ctypes.byref(plan), L.HICCL_BYTES, 0) == 0
    outs = []
    for so, do in ((0, 0), (1, 3), (5, 0), (13, 11)):
        dst = torch.zeros(nbytes + 64, dtype=torch.uint8, device=DEV)
        tab = (ctypes.c_void_p * 1)(src.data_ptr() + so)
        assert lib.hiccl_reduce_plan_add(plan, ctypes.c_void_p(dst.data_ptr() + do), tab, 1, nbytes) == 0, L.last_error()
        outs.append((dst, so, do))
    assert lib.hiccl_reduce_plan_launch(plan, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    s = src.cpu().numpy()
    for dst, so, do in outs:
        d = dst.cpu().numpy()
        assert np.array_equal(d[do:do + nbytes], s[so:so + nbytes])
        assert not d[:do].any() and not d[do + nbytes:].any()
    lib.hiccl_reduce_plan_destroy(plan)
    # float payloads survive a byte copy bit for bit (no 0 + x)
    f = torch.tensor([-0.0, float("nan"), 1.5, -2.25], device=DEV)
    f.view(torch.int32)[1] = 0x7FA00001
    g = torch.empty_like(f)
    hiccl_amd.reduce_ptrs(L.HICCL_BYTES, g.data_ptr(), [f.data_ptr()], 16)
    torch.cuda.synchronize()
    assert g.view(torch.int32).tolist() == f.view(torch.int32).tolist()


def test_plain_c_client_on_gpu():
    """build/abi_c (tests/cpp/abi_c.c, built by make): a C99 program using
    only include/hiccl_reduce.h reduces 3 device buffers, bit-exact with a
    host loop in the reference's order, then the same sum in a bucket from
    hiccl_bucket_alloc, bit-identical."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "abi_c")
    assert os.path.exists(exe), "run make"
    p = subprocess.run(["timeout", "-k", "5", "60", exe, "gpu"], capture_output=True, text=True)
    assert p.returncode == 0 and "abi_c: PASSED" in p.stdout, p.stdout + p.stderr


# ---------------------------------------------------------------------------
# Config sizes exactly as BASELINE.json names them (sampled bitwise checks
# against the oracle generator: a size-independent property at full size).

def _sampled(out, n, count, seed, bf16=False, extra=()):
    rng = np.random.default_rng(count % 1000003 + n)
    idx = np.concatenate([np.arange(64), count - 64 + np.arange(64), rng.integers(0, count, 4096),
                          np.asarray(extra, np.int64)]).astype(np.int64)
    idx = idx[(idx >= 0) & (idx < count)]
    got = out[torch.from_numpy(idx).to(DEV)]
    got = got.view(torch.int16).cpu().numpy().view(np.uint16) if bf16 else got.cpu().numpy()
    from conftest import Oracle
    exp = Oracle().sample_sum(idx.astype(np.uint64), seed, n, bf16=bf16)
    return bits_equal(got, exp), first_mismatch(got, exp)


@pytest.mark.parametrize("n", [2, 3, 4, 8, 16, 32, 64])
def test_config3_exact_sizes(oracle, n):
    """Config 3: n inputs x 2^26 fp32 (256 MiB each), the one-shot launch."""
    count, seed = 1 << 26, 3000 + n
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, device=DEV)
    hiccl_amd.reduce(out, ins)
    torch.cuda.synchronize()
    ok, msg = _sampled(out, n, count, seed)
    assert ok, msg


def _config4_bucket(oracle, dtype, per_input, each=False):
    """Config 4: n = 8, `per_input` bytes per input split into 1 MiB computes
    with the partition() formula (reduce.h:401-415; pipedepth = bytes / 1 MiB,
    as SURVEY.md 8d C4), ONE batched plan launch; checked at a random sample,
    at every compute's first and last element against the oracle generator,
    and for no element left unwritten (the output starts as NaN)."""
    n, esz = 8, (2 if dtype == torch.bfloat16 else 4)
    count, seed, depth = per_input // esz, 4000 + esz + (per_input >> 28), per_input >> 20
    free, _ = torch.cuda.mem_get_info()
    if free < (n + 1) * per_input + (1 << 30):
        pytest.skip("not enough device memory")
    ins = [torch.empty(count, dtype=dtype, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.full((count,), float("nan"), dtype=dtype, device=DEV)
    comp = hiccl_amd.Compute(dtype, device=0)
    off = 0
    for b in range(depth):
        c = count // depth + (1 if b < count % depth else 0)
        comp.add([(t, off) for t in ins], (out, off), c, compid=0)
        off += c
    assert off == count and comp.numcomp == depth
    comp.start(stream=torch.cuda.current_stream(), each=each)
    torch.cuda.synchronize()
    bounds = [b * (count // depth) + min(b, count % depth) for b in range(depth)]
    ok, msg = _sampled(out, n, count, seed, bf16=(dtype == torch.bfloat16),
                       extra=bounds + [x - 1 for x in bounds[1:]] + [count - 1])
    assert ok, msg
    assert not torch.isnan(out).any().item()  # no compute left unwritten
    comp.close()
    del ins, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_config4_exact_256MiB_in_1MiB_computes(oracle, dtype):
    """Config 4 at 256 MiB per input: 256 computes of 1 MiB in one launch."""
    _config4_bucket(oracle, dtype, 256 << 20)


@pytest.mark.parametrize("each", [False, True], ids=["batched", "launch_per_compute"])
@pytest.mark.parametrize("per_input", [16 << 20, 64 << 20], ids=["16MiB", "64MiB"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_config4_small_in_1MiB_computes(oracle, dtype, per_input, each):
    """Config 4's smallest sizes (16 and 64 computes of 1 MiB), both ways
    SURVEY.md 8d reports them: one batched plan launch, and the reference's
    structure of one launch per compute (compute.h:88-91;
    hiccl_reduce_plan_launch_each)."""
    _config4_bucket(oracle, dtype, per_input, each=each)


@pytest.mark.parametrize("per_input", [1 << 30, 4 << 30], ids=["1GiB", "4GiB"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_config4_large_in_1MiB_computes(oracle, dtype, per_input):
    """Config 4's largest sizes: 1 GiB and 4 GiB per input = 1,024 and 4,096
    computes of 1 MiB in ONE plan launch -- at 4 GiB the computes' byte
    offsets pass 2^32 inside the batched plan (bf16: 2^31 elements per
    input)."""
    _config4_bucket(oracle, dtype, per_input)


def test_bf16_2pow31_elements_64bit_offsets(oracle):
    """bf16 at 2^31 elements per input (4 GiB, n = 2): every byte offset past
    2^32 -- checked around 2^31 elements and at the end, under both engines."""
    n, count, seed = 2, 1 << 31, 77
    free, _ = torch.cuda.mem_get_info()
    if free < (n + 1) * count * 2 + (1 << 30):
        pytest.skip("not enough device memory")
    ins = [torch.empty(count, dtype=torch.bfloat16, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, dtype=torch.bfloat16, device=DEV)
    edge = [(1 << 30) - 1, 1 << 30, (1 << 31) - 8 + np.arange(8)]
    extra = [int(x) for e in edge for x in np.atleast_1d(e)]
    for eng in (None, PHASE, dict(engine=hiccl_amd.HICCL_ENGINE_TILE)):
        out.view(torch.int16).fill_(-1)
        hiccl_amd.reduce(out, ins, config=eng)
        torch.cuda.synchronize()
        ok, msg = _sampled(out, n, count, seed, bf16=True, extra=extra)
        assert ok, (eng, msg)


# ---------------------------------------------------------------------------
# Plan configuration and capture rules

@pytest.mark.parametrize("cfg", [
    dict(engine=1, unroll=1, blocks_per_cu=4), dict(engine=1, unroll=2, blocks_per_cu=3),
    dict(engine=1, unroll=4, schedule=2, grab=1), dict(engine=2), dict(engine=2, schedule=2),
    dict(engine=1, grid=7), dict(blocks_per_cu=2)])
@pytest.mark.parametrize("dtype", [np.float32, np.uint16], ids=["f32", "bf16"])
def test_plan_config_same_bits(oracle, cfg, dtype):
    """hiccl_reduce_plan_set_config: every honoured field gives the reference
    bits on a ragged, misaligned batch."""
    rng = np.random.default_rng(9)
    tdt = TORCH_OF[np.dtype(dtype)]
    comp = hiccl_amd.Compute(tdt, device=0, config=cfg)
    outs, exps, keep = [], [], []
    for c in range(9):
        n = int(rng.integers(1, 10))
        count = int(rng.integers(1, 300000))
        x = oracle.fill(n, count, seed=70 + c, dtype=dtype)
        ins = [to_dev(r).view(tdt) for r in x]
        keep += ins
        ob = torch.empty(count + 1, dtype=tdt, device=DEV)
        comp.add(ins, (ob, 1), count, compid=0)
        outs.append((ob, count))
        exps.append(oracle.reduce(list(x), dtype=dtype))
    for _ in range(2):
        comp.start()
        comp.wait()
        for (ob, count), e in zip(outs, exps):
            got = to_host(ob[1:1 + count], dtype)
            assert bits_equal(got, e), (cfg, first_mismatch(got, e))
    comp.close()


@pytest.mark.parametrize("peer", [1, 2, 3], ids=["stores", "loads", "both"])
@pytest.mark.parametrize("dtype,cfg", [(np.float32, None), (np.float32, dict(engine=2)),
                                       (np.float32, dict(engine=1, unroll=2)), (np.uint16, None),
                                       (np.float64, None), (np.uint64, dict(engine=2))],
                         ids=["f32", "f32-phase", "f32-u2", "bf16", "f64", "u64-phase"])
def test_plan_peer_policy_same_bits(oracle, peer, dtype, cfg):
    """hiccl_reduce_plan_set_peer (system-scope stores / loads for buffers in
    another GPU's memory, the transport's puts and gets and the fused
    gather): the same bits as the oracle on a ragged, misaligned batch (the
    scalar head/tail path with its fences included), relaunched."""
    rng = np.random.default_rng(11)
    tdt = TORCH_OF[np.dtype(dtype)]
    comp = hiccl_amd.Compute(tdt, device=0, config=cfg)
    comp.set_peer(peer)
    assert comp.peer() == peer
    outs, exps, keep = [], [], []
    for c in range(7):
        n = int(rng.integers(1, 10))
        count = int(rng.integers(1, 200000))
        if np.dtype(dtype) == np.uint64:
            x = rng.integers(0, 1 << 63, (n, count), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
        else:
            x = oracle.fill(n, count, seed=90 + c, dtype=dtype)
        ins = [to_dev(r).view(tdt) for r in x]
        keep += ins
        ob = torch.empty(count + 1, dtype=tdt, device=DEV)
        comp.add(ins, (ob, 1), count, compid=0)
        outs.append((ob, count))
        exps.append(oracle.reduce(list(x), dtype=dtype))
    for _ in range(2):
        for ob, _c in outs:
            ob.fill_(0)
        comp.start()
        comp.wait()
        for (ob, count), e in zip(outs, exps):
            got = to_host(ob[1:1 + count], dtype)
            assert bits_equal(got, e), (peer, cfg, first_mismatch(got, e))
    comp.close()


@pytest.mark.parametrize("peer", [1, 2])
def test_byte_copy_plan_peer_policy_exact(peer):
    """The transport's batched copies with the peer policy it uses (IPC put:
    system-scope stores; IPC get: system-scope loads): exact at odd sizes and
    byte offsets."""
    import ctypes
    from hiccl_amd import _lib as L
    lib = L.lib()
    plan = ctypes.c_void_p()
    assert lib.hiccl_reduce_plan_create(ctypes.byref(plan), L.HICCL_BYTES, 0) == 0
    assert lib.hiccl_reduce_plan_set_peer(plan, 7) == 1  # unknown bits refused
    assert lib.hiccl_reduce_plan_set_peer(plan, peer) == 0
    rng = np.random.default_rng(peer)
    src = torch.from_numpy(rng.integers(0, 256, (1 << 21) + 64, dtype=np.uint8)).to(DEV)
    outs = []
    for so, do, nb in ((0, 0, 1 << 20), (1, 3, 4099), (5, 0, 17), (13, 11, (1 << 21) - 5)):
        dst = torch.zeros(nb + 64, dtype=torch.uint8, device=DEV)
        tab = (ctypes.c_void_p * 1)(src.data_ptr() + so)
        assert lib.hiccl_reduce_plan_add(plan, ctypes.c_void_p(dst.data_ptr() + do), tab, 1, nb) == 0, L.last_error()
        outs.append((dst, so, do, nb))
    assert lib.hiccl_reduce_plan_launch(plan, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    s = src.cpu().numpy()
    for dst, so, do, nb in outs:
        d = dst.cpu().numpy()
        assert np.array_equal(d[do:do + nb], s[so:so + nb])
        assert not d[:do].any() and not d[do + nb:].any()
    lib.hiccl_reduce_plan_destroy(plan)


def test_plan_peer_policy_replaces_wide_tiles(oracle):
    """Two f32 inputs of 1 GiB would take wide tiles (unroll 16), which the
    peer kernels lack: with a peer policy the plan runs TILE at unroll 4,
    sampled-exact."""
    n, count, seed = 2, 1 << 28, 515
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, device=DEV)
    comp = hiccl_amd.Compute(torch.float32, device=0)
    comp.set_peer(2)
    comp.add(ins, out, count, compid=0)
    comp.start()
    comp.wait()
    assert comp.engine() == hiccl_amd.HICCL_ENGINE_TILE
    ok, msg = _sampled(out, n, count, seed)
    assert ok, msg
    comp.close()


@pytest.mark.parametrize("case", list(A.GPU_STORE_SMALL_STEP))
def test_plan_store_form_small_step(oracle, case):
    """A pipeline step's plan (the C5 step: 4 computes of n = 2 and one of
    n = 4, 2^18 f32, 5 MiB written) stores write-through by default -- nt
    lines left dirty in the L2s would cost the kernel boundary their
    write-back -- unless its config asks for nt or a shape only the nt
    kernels have; every form gives the oracle's bits, relaunched."""
    (dt, total, mean_n, cfg), want = A.GPU_STORE_SMALL_STEP[case]  # one table with the CPU tier's check
    c = 1 << 18
    assert total == 5 * c and mean_n == 2.4
    x = oracle.fill(12, c, seed=1212)
    ins = [to_dev(r) for r in x]
    outs = [torch.full((c,), float("nan"), device=DEV) for _ in range(5)]
    comp = hiccl_amd.Compute(torch.float32, device=0, config=cfg)
    for j in range(4):
        comp.add([ins[2 * j], ins[2 * j + 1]], outs[j], c, compid=0)
    comp.add(ins[8:12], outs[4], c, compid=0)
    assert comp.store_policy() == want
    exps = [oracle.reduce([x[2 * j], x[2 * j + 1]]) for j in range(4)] + [oracle.reduce(list(x[8:12]))]
    for _ in range(2):
        comp.start()
        comp.wait()
        for o, e in zip(outs, exps):
            assert bits_equal(o.cpu().numpy(), e)
    comp.close()


@pytest.mark.parametrize("case", list(A.GPU_STORE_LARGE))
def test_plan_store_form_large(oracle, case):
    """A reduction plan writing up to 256 MiB per launch stores write-through
    by default (config 3 / 4 sizes: 1.6-9 % faster), above it nt (512 MiB
    and 1 GiB: no gain); write-through on request; sampled-exact at 8 inputs
    in 1 MiB computes."""
    (dt, count, n, cfg), want = A.GPU_STORE_LARGE[case]  # one table with the CPU tier's check
    seed = 808
    ins = [torch.empty(count, device=DEV) for _ in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, seed, k)
    out = torch.empty(count, device=DEV)
    comp = hiccl_amd.Compute(torch.float32, device=0, config=cfg)
    step = 1 << 18
    for off in range(0, count, step):
        comp.add([(t, off) for t in ins], (out, off), step, compid=0)
    assert comp.store_policy() == want
    comp.start()
    comp.wait()
    ok, msg = _sampled(out, n, count, seed)
    assert ok, msg
    comp.close()


def test_byte_copy_plan_store_forms():
    """Byte copies (the transport's, HICCL_BYTES plans) store write-through
    up to 32 MiB per launch and nt above (they lose from 48 MiB written),
    exact."""
    big = hiccl_amd.Compute(torch.uint8, device=0)
    src = torch.randint(0, 256, (48 << 20,), dtype=torch.uint8, device=DEV)
    dst = torch.zeros(48 << 20, dtype=torch.uint8, device=DEV)
    big.add([src], dst, 48 << 20, compid=0)
    assert big.store_policy() == dict(((c, n), w) for (dt, c, n, _), w in A.GPU_STORE_BYTES)[(48 << 20, 1)]
    big.start()
    big.wait()
    assert torch.equal(src, dst)
    big.close()
    _byte_copy_plan_small()


def _byte_copy_plan_small():
    """The transport's per-step copies (HICCL_BYTES plans, 1 MiB each) take
    the write-through form, exact."""
    comp = hiccl_amd.Compute(torch.uint8, device=0)
    src = [torch.randint(0, 256, ((1 << 20) + 3,), dtype=torch.uint8, device=DEV) for _ in range(5)]
    dst = [torch.zeros((1 << 20) + 3, dtype=torch.uint8, device=DEV) for _ in range(5)]
    for a, b in zip(src, dst):
        comp.add([a], b, (1 << 20) + 3, compid=0)
    assert comp.store_policy() == dict(((c, n), w) for (dt, c, n, _), w in A.GPU_STORE_BYTES)[(5 * ((1 << 20) + 3), 1)]
    comp.start()
    comp.wait()
    assert all(torch.equal(a, b) for a, b in zip(src, dst))
    comp.close()


@pytest.mark.parametrize("dtype", [np.float32, np.uint16, np.float64, np.int32], ids=["f32", "bf16", "f64", "i32"])
@pytest.mark.parametrize("cfg", [None, dict(store_policy=4), dict(store_policy=4, engine=2),
                                 dict(store_policy=4, engine=1, unroll=2), dict(store_policy=2)],
                         ids=["auto", "wt", "wt-phase", "wt-u2", "nt"])
def test_oneshot_store_forms_same_bits(oracle, dtype, cfg):
    """One-shot calls take the write-through store form by size too (the
    default below 32 MiB written) or on request; misaligned output, same
    bits as the oracle in every form the type has."""
    if cfg and cfg.get("unroll") == 2 and np.dtype(dtype) not in (np.dtype(np.float32), np.dtype(np.uint16)):
        pytest.skip("unroll 2 exists for f32 / bf16 only")
    n, count = 5, 300007
    if np.dtype(dtype) == np.dtype(np.int32):  # wrap-around sums
        x = np.random.default_rng(4242).integers(-2**31, 2**31, (n, count), dtype=np.int32)
    else:
        x = oracle.fill(n, count, seed=4242, dtype=dtype)
    tdt = TORCH_OF[np.dtype(dtype)]
    ins = [to_dev(r).view(tdt) for r in x]
    ob = torch.empty(count + 1, dtype=tdt, device=DEV)
    hiccl_amd.reduce(ob[1:], ins, config=cfg)
    torch.cuda.synchronize()
    got = to_host(ob[1:], dtype)
    e = oracle.reduce(list(x), dtype=dtype)
    assert bits_equal(got, e), first_mismatch(got, e)


def test_oneshot_write_through_needs_its_shape():
    """Explicit write-through with a shape only the nt kernels have (wide
    tiles) is refused, never silently replaced."""
    x = [torch.zeros(1 << 16, device=DEV) for _ in range(2)]
    with pytest.raises(hiccl_amd.HicclError):
        hiccl_amd.reduce(torch.empty(1 << 16, device=DEV), x, config=dict(store_policy=4, engine=1, unroll=8))


def test_plan_config_refuses_unsupported_fields():
    for bad in (dict(order=2), dict(order=-1), dict(engine=1, unroll=32), dict(engine=1, unroll=3), dict(engine=2, unroll=4), dict(engine=1, block=512),
                dict(nontemporal=1), dict(store_policy=3), dict(store_policy=1), dict(drain=1), dict(schedule=7),
                # write-through has no TILE unroll 1 / 8 / 16 plan kernel (refused here, not at launch)
                dict(store_policy=4, engine=1, unroll=8), dict(store_policy=4, engine=1, unroll=16),
                dict(store_policy=4, engine=1, unroll=1)):
        with pytest.raises(hiccl_amd.HicclError):
            hiccl_amd.Compute(torch.float32, device=0, config=bad)
    with pytest.raises(hiccl_amd.HicclError):  # unroll 2 exists for f32/bf16 only
        hiccl_amd.Compute(torch.float64, device=0, config=dict(engine=1, unroll=2))


def test_large_n_refuses_unsupported_shape():
    """n > 64 runs on the plan kernel: a one-shot shape it lacks is an error,
    not silently replaced -- refused before any
    allocation, so nothing leaks (write-through wide tiles at
    n = 65 used to fail only at launch, after the pointer table's
    hipMallocAsync)."""
    x = torch.zeros(1000, device=DEV)
    for _ in range(3):
        with pytest.raises(hiccl_amd.HicclError, match="n > 64"):
            hiccl_amd.reduce(x, [x] * 65, config=dict(store_policy=4, engine=1, unroll=8))
    with pytest.raises(hiccl_amd.HicclError, match="n > 64"):
        hiccl_amd.reduce(x, [x] * 70, config=dict(block=512, unroll=4))
    with pytest.raises(hiccl_amd.HicclError, match="n > 64"):
        hiccl_amd.reduce(x, [x] * 70, config=dict(engine=2, nontemporal=1))


@pytest.mark.parametrize("n", [65, 100])
def test_large_n_capture_is_refused(n):
    """A > 64-input one-shot call uploads its pointer table from host memory
    per call: captured, the graph would replay a copy from a freed buffer --
    the library refuses the capture with a clear error."""
    count = 4099
    ins = [torch.ones(count, device=DEV) for _ in range(n)]
    out = torch.empty(count, device=DEV)
    hiccl_amd.reduce(out, ins)  # eager: fine
    torch.cuda.synchronize()
    assert out[0].item() == float(n)
    g = torch.cuda.CUDAGraph()
    with pytest.raises(hiccl_amd.HicclError, match="cannot be captured"):
        with torch.cuda.graph(g):
            hiccl_amd.reduce(out, ins)


def test_plan_capture_after_eager_upload(oracle):
    """A plan's first launch after an add uploads its table (synchronous):
    refused inside a capture; after one eager launch the plan captures and
    every replay gives the reference bits."""
    n, count = 6, 300001
    x = oracle.fill(n, count, seed=41)
    ins = [to_dev(r) for r in x]
    out = torch.empty(count, device=DEV)
    comp = hiccl_amd.Compute(torch.float32, device=0)
    for b in range(3):
        c = count // 3 + (1 if b < count % 3 else 0)
        comp.add([(t, b * (count // 3) + min(b, count % 3)) for t in ins],
                 (out, b * (count // 3) + min(b, count % 3)), c, compid=0)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(hiccl_amd.HicclError, match="cannot be captured"):
        with torch.cuda.graph(g, stream=s):
            comp.start(stream=s)
    comp.start(stream=s)  # eager: uploads
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        comp.start(stream=s)
    for _ in range(3):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        exp = oracle.reduce(list(x))
        assert bits_equal(got, exp), first_mismatch(got, exp)
    comp.close()


def test_dynamic_schedule_per_thread_stream_two_threads(oracle):
    """hipStreamPerThread is one handle value for a different stream on each
    host thread: two threads launching dynamic-schedule reductions on it at
    once must not share a ticket counter (the library takes the static
    schedule there) -- both results bit-exact."""
    import threading
    n, count = 8, (1 << 22) + 5  # >= 32 tickets per workgroup: dynamic if allowed
    xs = [oracle.fill(n, count, seed=s) for s in (1, 2)]
    exps = [oracle.reduce(list(x)) for x in xs]
    bufs = [([to_dev(r) for r in x], torch.empty(count, device=DEV)) for x in xs]
    torch.cuda.synchronize()
    PER_THREAD = 2  # hipStreamPerThread
    errs = []

    def work(i):
        try:
            torch.cuda.set_device(0)
            ins, out = bufs[i]
            for _ in range(20):
                hiccl_amd.reduce(out, ins, stream=PER_THREAD,
                                 config=dict(engine=hiccl_amd.HICCL_ENGINE_TILE,
                                             schedule=hiccl_amd._lib.HICCL_SCHED_DYNAMIC))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for (ins, out), e in zip(bufs, exps):
        got = out.cpu().numpy()
        assert bits_equal(got, e), first_mismatch(got, e)


@pytest.mark.parametrize("offs,out_off", [([1, 0], 0), ([0, 3], 1), ([1, 2, 3, 0], 0), ([3, 3, 3], 3),
                                          ([2, 1, 0, 3, 2, 1, 0, 3, 1], 0), ([1, 2, 3, 1, 2, 3, 1, 2], 0),
                                          ([1, 2, 3, 1, 2, 3, 1, 2], 1)])
@pytest.mark.parametrize("dtype", [np.float32, np.uint16])
def test_misaligned_full_tiles(oracle, offs, out_off, dtype):
    """Inputs off a 16-B boundary on the full 256 x 4 tile shape (the C2
    shape; the small-count tests above run on half tiles): bit-exact
    against the oracle across tile boundaries and partial last tiles."""
    n = len(offs)
    cfg = dict(engine=hiccl_amd.HICCL_ENGINE_TILE, block=256, unroll=4)
    for count in (1, 5, 4099, 70001, (1 << 20) + 3, 3 * 4096 * 64 + 7):
        x = oracle.fill(n, count, seed=17 + count, dtype=dtype)
        got = gpu_reduce(x, count, dtype, offsets=offs, out_offset=out_off, config=cfg)
        exp = oracle.reduce(list(x), dtype=dtype)
        assert bits_equal(got, exp), f"offs={offs} out={out_off} count={count}: {first_mismatch(got, exp)}"


def test_bucket_layout_alloc_and_reduce(oracle):
    """hiccl_bucket_alloc (C ABI) and hiccl_amd.bucket (Python): n inputs and
    the output in one allocation at hiccl_bucket_stride; the reduction over
    them gives the oracle's bits (the layout only moves where the bytes
    live)."""
    lib = hiccl_amd.lib()
    n, count = 8, (1 << 20) + 5
    stride = lib.hiccl_bucket_stride(L.HICCL_FLOAT32, count)
    base, out = ctypes.c_void_p(), ctypes.c_void_p()
    ins = (ctypes.c_void_p * n)()
    L.check(lib.hiccl_bucket_alloc(L.HICCL_FLOAT32, n, count, 0, ctypes.byref(base), ins, ctypes.byref(out)),
            "bucket_alloc")
    try:
        assert [ins[k] - base.value for k in range(n)] == [k * stride for k in range(n)]
        assert out.value - base.value == n * stride
        x = oracle.fill(n, count, seed=606)
        for k in range(n):
            t = torch.from_numpy(x[k]).to(DEV)
            L.check(lib.hiccl_stream_copy(ctypes.c_void_p(ins[k]), ctypes.c_void_p(t.data_ptr()), count * 4, None),
                    "copy")
        torch.cuda.synchronize()
        hiccl_amd.reduce_ptrs(L.HICCL_FLOAT32, out.value, [ins[k] for k in range(n)], count)
        got = torch.empty(count, device=DEV)
        L.check(lib.hiccl_stream_copy(ctypes.c_void_p(got.data_ptr()), out, count * 4, None), "copy")
        torch.cuda.synchronize()
        assert bits_equal(got.cpu().numpy(), oracle.reduce(list(x)))
    finally:
        L.check(lib.hiccl_bucket_free(base), "bucket_free")
    # the Python views: same layout, bf16 too
    for dt, npdt in ((torch.float32, np.float32), (torch.bfloat16, np.uint16)):
        vi, vo = hiccl_amd.bucket(5, count, dt)
        st = lib.hiccl_bucket_stride(L.DTYPE_OF_TORCH[dt], count)
        assert [v.data_ptr() - vi[0].data_ptr() for v in vi + [vo]] == [j * st for j in range(6)]
        x = oracle.fill(5, count, seed=707, dtype=npdt)
        for k in range(5):
            vi[k].copy_(to_dev(x[k]))
        hiccl_amd.reduce(vo, vi)
        torch.cuda.synchronize()
        assert bits_equal(to_host(vo, npdt), oracle.reduce(list(x), dtype=npdt))


@pytest.mark.parametrize("dtype,n", [(np.float64, 3), (np.float32, 70), (np.int32, 9)], ids=["f64-3", "f32-70", "i32-9"])
def test_bucket_layout_more_shapes(oracle, dtype, n):
    """hiccl_amd.bucket for other types and for n > 64 (the plan kernel via
    the device pointer table), with a ragged count: the oracle's bits."""
    count = 300007
    tdt = TORCH_OF[np.dtype(dtype)]
    if np.dtype(dtype) == np.dtype(np.int32):
        x = np.random.default_rng(n).integers(-2**31, 2**31, (n, count), dtype=np.int32)
    else:
        x = oracle.fill(n, count, seed=900 + n, dtype=dtype)
    ins, out = hiccl_amd.bucket(n, count, tdt)
    st = hiccl_amd.lib().hiccl_bucket_stride(L.DTYPE_OF_TORCH[tdt], count)
    assert ins[1].data_ptr() - ins[0].data_ptr() == st and out.data_ptr() - ins[0].data_ptr() == n * st
    for k in range(n):
        ins[k].copy_(to_dev(x[k]).view(tdt))
    hiccl_amd.reduce(out, ins)
    torch.cuda.synchronize()
    e = oracle.reduce(list(x), dtype=dtype)
    got = to_host(out, dtype)
    assert bits_equal(got, e), first_mismatch(got, e)
