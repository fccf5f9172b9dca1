"""CPU tier: the C-ABI library loads, exports every declared symbol, and its
host-side argument checking behaves (no compute calls without a GPU)."""
import ctypes
import os

import pytest

import hiccl_amd
from hiccl_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_built_in_tree():
    assert os.path.exists(L.LIB_PATH), "run make / __graft_entry__.build()"
    assert os.path.dirname(L.LIB_PATH) == os.path.join(ROOT, "hiccl_amd")


def test_exports_every_header_symbol():
    names = L.header_functions()
    assert "hiccl_reduce" in names and "hiccl_reduce_plan_launch" in names
    raw = ctypes.CDLL(L.LIB_PATH)
    missing = [n for n in names if not hasattr(raw, n)]
    assert not missing, f"declared in include/hiccl_reduce.h but not exported: {missing}"
    # and every declared symbol has a Python signature
    assert not [n for n in names if n not in L._SIGS]


def test_gfx950_code_object_embedded():
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_dtype_sizes_and_version():
    lib = L.lib()
    assert [lib.hiccl_dtype_size(d) for d in range(6)] == [4, 8, 2, 8, 4, 1]
    assert lib.hiccl_dtype_size(99) == 0
    assert lib.hiccl_version() >= 100


def _tab(ptrs):
    return (ctypes.c_void_p * max(1, len(ptrs)))(*ptrs)


def test_invalid_arguments_rejected_on_host():
    lib = L.lib()
    # unknown dtype
    assert lib.hiccl_reduce(42, ctypes.c_void_p(0x1000), _tab([0x2000]), 1, 4, None) == 1
    assert "dtype" in L.last_error()
    # count == 0 is a no-op (no device access)
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0), _tab([]), 0, 0, None) == 0
    # NULL out
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0), _tab([0x2000]), 1, 4, None) == 1
    assert "out is NULL" in L.last_error()
    # misaligned out for f32
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0x1002), _tab([0x2000]), 1, 4, None) == 1
    assert "element-aligned" in L.last_error()
    # NULL input pointer
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0x1000), _tab([0]), 1, 4, None) == 1
    # partial overlap of an input with the output (exact aliasing is allowed)
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0x1000), _tab([0x1004]), 1, 4, None) == 1
    assert "overlaps" in L.last_error()
    # negative n
    assert lib.hiccl_reduce(0, ctypes.c_void_p(0x1000), _tab([]), -1, 4, None) == 1
    # byte copies take exactly one input
    assert lib.hiccl_reduce(5, ctypes.c_void_p(0x1000), _tab([0x2000, 0x3000]), 2, 4, None) == 1
    assert "n == 1" in L.last_error()
    # unsupported tuning config
    cfg = L.ReduceConfig(block=128)
    assert lib.hiccl_reduce_ex(0, ctypes.c_void_p(0x1000), _tab([0x2000]), 1, 4, None, ctypes.byref(cfg)) == 1
    # unknown engine / schedule, bad grab
    for bad, word in ((dict(engine=7), "engine"), (dict(schedule=5), "schedule"), (dict(grab=-1), "grab"),
                      (dict(grab=100000), "grab")):
        cfg = L.ReduceConfig(**bad)
        assert lib.hiccl_reduce_ex(0, ctypes.c_void_p(0x1000), _tab([0x2000]), 1, 4, None, ctypes.byref(cfg)) == 1
        assert word in L.last_error()
    # plan NULL handling
    assert lib.hiccl_reduce_plan_launch(None, None) == 1
    assert lib.hiccl_reduce_plan_set_engine(None, L.HICCL_ENGINE_PHASE) == 1
    assert lib.hiccl_reduce_plan_engine(None) == -1
    assert lib.hiccl_reduce_plan_set_peer(None, L.HICCL_PEER_STORES) == 1
    assert "plan is NULL" in L.last_error()
    assert lib.hiccl_reduce_plan_peer(None) == -1
    assert lib.hiccl_reduce_plan_store_policy(None) == -1
    assert lib.hiccl_reduce_plan_numcomp(None) == 0
    lib.hiccl_reduce_plan_destroy(None)
    # host pipe: argument checks come before any HIP call
    h = ctypes.c_void_p()
    assert lib.hiccl_host_pipe_create(None, 0, 0, 0, 0) == 1
    assert lib.hiccl_host_pipe_create(ctypes.byref(h), 42, 0, 0, 0) == 1 and not h.value
    assert "dtype" in L.last_error()
    assert lib.hiccl_host_pipe_create(ctypes.byref(h), 0, 0, 0, 9) == 1
    assert "depth" in L.last_error()
    assert lib.hiccl_host_pipe_create(ctypes.byref(h), 1, 0, 4, 0) == 1  # f64 chunk < 1 element
    assert lib.hiccl_host_pipe_reduce(None, ctypes.c_void_p(0x1000), _tab([0x2000]), 1, 4) == 1
    lib.hiccl_host_pipe_destroy(None)


def test_python_layer_refuses_cpu_tensors():
    import torch
    x = torch.zeros(4)
    with pytest.raises(ValueError, match="device tensor"):
        hiccl_amd.reduce(x, [x])


def test_header_is_c_and_plain_c_client_runs():
    """include/hiccl_reduce.h compiles as C99 (-pedantic -Werror) and a C
    client linked against the library passes its host-side checks."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "abi_c")
        subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cpp", "abi_c.c"),
                        "-o", exe, "-L", os.path.join(ROOT, "hiccl_amd"), "-lhiccl_reduce",
                        "-Wl,-rpath," + os.path.join(ROOT, "hiccl_amd"), "-L/opt/rocm/lib", "-lamdhip64",
                        "-Wl,-rpath,/opt/rocm/lib"], check=True)
        p = subprocess.run([exe], capture_output=True, text=True)
        assert p.returncode == 0 and "abi_c: PASSED" in p.stdout, p.stdout + p.stderr


def test_program_argument_checks_on_host():
    """hiccl_program_*: NULL handles and unknown dtypes are refused before any
    device work (no GPU here)."""
    lib = L.lib()
    h = ctypes.c_void_p()
    assert lib.hiccl_program_create(None, L.HICCL_FLOAT32, 0) != 0
    assert lib.hiccl_program_create(ctypes.byref(h), 99, 0) != 0 and not h.value
    assert lib.hiccl_program_add_signal(None, None, 0, None, 0) != 0
    assert lib.hiccl_program_add_plan(None, None) != 0
    assert lib.hiccl_program_launch(None, None, None, None, 1.0, None) != 0
    assert lib.hiccl_program_num_units(None) == 0 and lib.hiccl_program_num_phases(None) == 0
    lib.hiccl_program_destroy(None)


def _auto(dtype, count, n, cus=256, acc=0):
    import ctypes
    lib = L.lib()
    e, u, b, d = (ctypes.c_int() for _ in range(4))
    rc = lib.hiccl_reduce_auto_choice(dtype, acc, count, float(n), cus, ctypes.byref(e), ctypes.byref(u),
                                      ctypes.byref(b), ctypes.byref(d))
    assert rc == 0, L.last_error()
    return e.value, u.value, b.value, d.value


def test_auto_choice_rule_table_on_host():
    """hiccl_reduce_auto_choice (no device queried): AUTO's engine / shape /
    schedule for the BASELINE configs and the round-3 mid-size rule
    (profiles/r03n_midsize.jsonl, r03q_sweep_manyn.jsonl)."""
    from auto_table import RULE_CASES as cases
    T, P = L.HICCL_ENGINE_TILE, L.HICCL_ENGINE_PHASE
    f32, bf16 = L.HICCL_FLOAT32, L.HICCL_BFLOAT16
    MiB = 1 << 20
    for (dt, count, n), want in cases:
        assert _auto(dt, count, n) == want, (dt, count, n, _auto(dt, count, n), want)
    # 64 KiB phased chunks (bf16 with the f32 accumulator, int32): the same rule
    # in chunks, PHASE for many inputs only when 80 % of the last round is busy
    # (profiles/r03ze_midsize_i32.jsonl, r03ze_midsize_bf16wide.jsonl)
    assert _auto(bf16, 40 * MiB // 2, 3, acc=L.HICCL_ACC_WIDE)[0] == T   # 2.5 chunks per CU
    assert _auto(bf16, 72 * MiB // 2, 4, acc=L.HICCL_ACC_WIDE)[0] == P   # 4.5, 90 % busy
    assert _auto(L.HICCL_INT32, 24 * MiB // 4, 8)[0] == T                # 1.5, 75 % busy
    assert _auto(L.HICCL_INT32, 40 * MiB // 4, 8)[0] == P                # 2.5, 83 % busy
    # another CU count: the thresholds scale with it
    assert _auto(f32, 1 << 28, 8, cus=304)[0] == T
    lib = L.lib()
    import ctypes
    assert lib.hiccl_reduce_auto_choice(42, 0, 1024, 2.0, 256, None, None, None, None) == 1
    assert lib.hiccl_reduce_auto_choice(f32, 0, 1024, 2.0, 0, None, None, None, None) == 1


def test_gpu_tier_auto_expectations_follow_the_rule():
    """The GPU tier's AUTO expectations (tests/auto_table.py, read by
    test_reduce_gpu.py) agree with the rule the library implements: every
    engine row and every store-form row, answered on the host for 256 CUs.
    A rule change not carried into the table fails HERE, in the CPU tier."""
    import auto_table as A
    for (dt, count, n, cfg), want in A.all_engine_rows():
        got = hiccl_amd.auto_choice(dt, count, n, config=cfg)
        assert got["engine"] == want, (dt, count, n, cfg, got, want)
    for (dt, count, n, cfg), want in A.all_store_rows():
        got = hiccl_amd.auto_choice(dt, count, n, config=cfg)
        assert got["store_policy"] == want, (dt, count, n, cfg, got, want)
    # the plain entry point is the _ex one with a default config
    for (dt, count, n), want in A.RULE_CASES:
        got = hiccl_amd.auto_choice(dt, count, n)
        assert (got["engine"], got["unroll"], got["blocks_per_cu"], got["dynamic"]) == want


def test_auto_choice_ex_store_form_and_refusals():
    """hiccl_reduce_auto_choice_ex: the store form is decided before the
    engine, on the shapes that have a write-through kernel (the
    engine must not follow write-through measurements for a launch that
    stays nt), and a config no kernel has is refused as hiccl_reduce_ex
    refuses it."""
    T, P = L.HICCL_ENGINE_TILE, L.HICCL_ENGINE_PHASE
    f32 = L.HICCL_FLOAT32
    c3 = (f32, 1 << 26, 3)  # 3 x 256 MiB: write-through by size -> static tiles
    assert hiccl_amd.auto_choice(*c3) == dict(engine=T, unroll=4, blocks_per_cu=1, dynamic=0, store_policy=4)
    # plain loads (nontemporal 1): no write-through kernel, so nt stores AND the nt engine table
    got = hiccl_amd.auto_choice(*c3, config=dict(nontemporal=1))
    assert (got["engine"], got["store_policy"]) == (P, 2), got
    assert hiccl_amd.auto_choice(*c3, config=dict(store_policy=2))["engine"] == P
    # explicit unroll 1 stays nt by size (one rule for one-shot calls and plans), write-through on request
    assert hiccl_amd.auto_choice(*c3, config=dict(engine=T, unroll=1))["store_policy"] == 2
    assert hiccl_amd.auto_choice(*c3, config=dict(engine=T, unroll=1, store_policy=4))["store_policy"] == 4
    # above the cap: nt whatever the engine
    assert hiccl_amd.auto_choice(f32, 1 << 28, 8)["store_policy"] == 2
    # byte copies: 32 MiB cap
    assert hiccl_amd.auto_choice(L.HICCL_BYTES, 32 << 20, 1)["store_policy"] == 4
    assert hiccl_amd.auto_choice(L.HICCL_BYTES, (32 << 20) + 16, 1)["store_policy"] == 2
    # refusals: write-through wide tiles (one-shot), and n > 64 on the plan kernel
    for cfg, n in ((dict(store_policy=4, engine=T, unroll=8), 2), (dict(store_policy=4, engine=T, unroll=8), 65),
                   (dict(store_policy=4, engine=T, unroll=1), 65), (dict(block=512, unroll=4), 70),
                   (dict(engine=7), 2), (dict(acc=5), 2), (dict(schedule=9), 2),
                   (dict(order=3), 2), (dict(order=8192), 2), (dict(order=-2), 2), (dict(order=2), 65),
                   (dict(blocks_per_cu=65), 2), (dict(grid=-1), 2)):
        with pytest.raises(hiccl_amd.HicclError):
            hiccl_amd.auto_choice(f32, 1 << 16, n, config=cfg)
    # n > 64 with unroll 8 and nt: the plan kernel has it
    assert hiccl_amd.auto_choice(f32, 1 << 16, 65, config=dict(engine=T, unroll=8))["unroll"] == 8


def test_stream_ordered_defaults_resolve_as_stated(monkeypatch):
    """The stream-ordered protocol defaults: fenced
    token phases unless HICCL_PROG_FENCES=light, one launch per element
    unless HICCL_STEP_PROGRAM=1 -- resolved from the environment at each call,
    as every launch resolves them (hiccl_token_mode,
    hiccl_step_program_default; HiCCL::Comm::want_programs uses the latter)."""
    lib = L.lib()
    for k in ("HICCL_PROG_FENCES", "HICCL_STEP_PROGRAM"):
        monkeypatch.delenv(k, raising=False)
    assert lib.hiccl_token_mode() == L.HICCL_TOKENS_FENCED
    assert lib.hiccl_step_program_default() == 0
    for v, want in (("full", L.HICCL_TOKENS_FENCED), ("light", L.HICCL_TOKENS_LIGHT), ("", L.HICCL_TOKENS_FENCED),
                    ("LIGHT", L.HICCL_TOKENS_FENCED), ("0", L.HICCL_TOKENS_FENCED)):
        monkeypatch.setenv("HICCL_PROG_FENCES", v)
        assert lib.hiccl_token_mode() == want, v
    # round 3's truthy spellings keep working; anything else reads as off
    for v, want in (("1", 1), ("0", 0), ("", 0), ("yes", 1), ("ON", 1), ("True", 1), ("off", 0), ("no", 0),
                    ("2", 0), ("bogus", 0)):
        monkeypatch.setenv("HICCL_STEP_PROGRAM", v)
        assert lib.hiccl_step_program_default() == want, v


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: with the HIP library absent every entry point raises
    (the product never computes on the host instead)."""
    import torch
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "libhiccl_reduce.so"))
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(ImportError, match="HIP extension missing"):
        L.lib()
    with pytest.raises(ImportError, match="HIP extension missing"):
        hiccl_amd.Compute(torch.float32, device=0)


def test_bucket_layout_on_host():
    """hiccl_bucket_stride: the buffer rounded up to 64 KiB plus 64 KiB
    (config 2: 1 GiB + 64 KiB); hiccl_bucket_alloc refuses bad arguments
    before any HIP call."""
    lib = L.lib()
    K = 64 << 10
    assert lib.hiccl_bucket_stride(L.HICCL_FLOAT32, 1 << 28) == (1 << 30) + K
    assert lib.hiccl_bucket_stride(L.HICCL_FLOAT32, 1) == 2 * K
    assert lib.hiccl_bucket_stride(L.HICCL_BFLOAT16, K // 2) == 2 * K
    assert lib.hiccl_bucket_stride(L.HICCL_BFLOAT16, K // 2 + 1) == 3 * K
    assert lib.hiccl_bucket_stride(99, 10) == 0 and lib.hiccl_bucket_stride(L.HICCL_FLOAT32, 0) == 0
    base, out = ctypes.c_void_p(), ctypes.c_void_p()
    ins = (ctypes.c_void_p * 8)()
    for args, word in (((99, 8, 16, 0), "dtype"), ((0, -1, 16, 0), "n out of range"), ((0, 8, 0, 0), "count"),
                       ((0, 8, 16, 0, None, ins, ctypes.byref(out)), "NULL"),
                       ((0, 8, 16, 0, ctypes.byref(base), None, ctypes.byref(out)), "NULL")):
        full = args if len(args) == 7 else args + (ctypes.byref(base), ins, ctypes.byref(out))
        assert lib.hiccl_bucket_alloc(*full) == 1
        assert word in L.last_error()
    assert lib.hiccl_bucket_free(None) == 0
