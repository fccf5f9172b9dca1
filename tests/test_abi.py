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
