"""ctypes binding of the C ABI in include/hiccl_reduce.h.

The product path is hiccl_amd/libhiccl_reduce.so (HIP kernels for gfx950).
There is deliberately NO fallback: if the shared library is missing this
module raises, so a GPU run can never silently compute on the CPU.

torch is imported before the library is opened so that the process holds a
single HIP runtime (torch's libamdhip64.so.7 satisfies the library's NEEDED
entry by SONAME).
"""
import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL: one HIP runtime per process)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhiccl_reduce.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hiccl_reduce.h")

HICCL_FLOAT32 = 0
HICCL_FLOAT64 = 1
HICCL_BFLOAT16 = 2
HICCL_UINT64 = 3
HICCL_INT32 = 4
HICCL_BYTES = 5

HICCL_ACC_NATIVE = 0
HICCL_ACC_WIDE = 1

HICCL_ENGINE_AUTO = 0
HICCL_ENGINE_TILE = 1
HICCL_ENGINE_PHASE = 2

HICCL_PEER_STORES = 1
HICCL_PEER_LOADS = 2
HICCL_TOKENS_FENCED = 0  # hiccl_token_mode()
HICCL_TOKENS_LIGHT = 1

HICCL_SCHED_AUTO = 0
HICCL_SCHED_STATIC = 1
HICCL_SCHED_DYNAMIC = 2

DTYPE_OF_TORCH = {
    torch.float32: HICCL_FLOAT32,
    torch.float64: HICCL_FLOAT64,
    torch.bfloat16: HICCL_BFLOAT16,
    torch.int64: HICCL_UINT64,  # two's-complement add == size_t add bit for bit
    torch.uint64: HICCL_UINT64,
    torch.int32: HICCL_INT32,
    torch.uint8: HICCL_BYTES,  # exact byte copies (one input)
}


class HicclError(RuntimeError):
    """A non-zero hipError_t returned through the C ABI."""

    def __init__(self, code, where, msg):
        super().__init__(f"{where}: hipError {code}: {msg}")
        self.code = code


class ReduceConfig(ctypes.Structure):
    _fields_ = [("block", ctypes.c_int), ("unroll", ctypes.c_int),
                ("blocks_per_cu", ctypes.c_int), ("nontemporal", ctypes.c_int),
                ("acc", ctypes.c_int), ("grid", ctypes.c_int), ("store_policy", ctypes.c_int),
                ("engine", ctypes.c_int), ("schedule", ctypes.c_int), ("grab", ctypes.c_int),
                ("drain", ctypes.c_int), ("order", ctypes.c_int)]


_lib = None

_vp = ctypes.c_void_p
_SIGS = {
    "hiccl_dtype_size": (ctypes.c_size_t, [ctypes.c_int]),
    "hiccl_last_error": (ctypes.c_char_p, []),
    "hiccl_version": (ctypes.c_int, []),
    "hiccl_reduce": (ctypes.c_int, [ctypes.c_int, _vp, _vp, ctypes.c_int, ctypes.c_size_t, _vp]),
    "hiccl_reduce_f32": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, _vp]),
    "hiccl_reduce_bf16": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_size_t, _vp]),
    "hiccl_reduce_ex": (ctypes.c_int, [ctypes.c_int, _vp, _vp, ctypes.c_int, ctypes.c_size_t, _vp,
                                       ctypes.POINTER(ReduceConfig)]),
    "hiccl_reduce_auto_choice": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_double,
                                                ctypes.c_int, _vp, _vp, _vp, _vp]),
    "hiccl_reduce_auto_choice_ex": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ReduceConfig), ctypes.c_size_t,
                                                   ctypes.c_double, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "hiccl_reduce_plan_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int]),
    "hiccl_reduce_plan_set_acc": (ctypes.c_int, [_vp, ctypes.c_int]),
    "hiccl_reduce_plan_set_engine": (ctypes.c_int, [_vp, ctypes.c_int]),
    "hiccl_reduce_plan_set_config": (ctypes.c_int, [_vp, ctypes.POINTER(ReduceConfig)]),
    "hiccl_reduce_plan_engine": (ctypes.c_int, [_vp]),
    "hiccl_reduce_plan_set_peer": (ctypes.c_int, [_vp, ctypes.c_int]),
    "hiccl_reduce_plan_peer": (ctypes.c_int, [_vp]),
    "hiccl_reduce_plan_store_policy": (ctypes.c_int, [_vp]),
    "hiccl_reduce_plan_add": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_size_t]),
    "hiccl_reduce_plan_launch": (ctypes.c_int, [_vp, _vp]),
    "hiccl_reduce_plan_enqueue": (ctypes.c_int, [_vp, _vp]),
    "hiccl_reduce_plan_launch_each": (ctypes.c_int, [_vp, _vp]),
    "hiccl_reduce_plan_sync": (ctypes.c_int, [_vp]),
    "hiccl_reduce_plan_numcomp": (ctypes.c_int, [_vp]),
    "hiccl_reduce_plan_stream": (_vp, [_vp]),
    "hiccl_reduce_plan_bytes": (ctypes.c_size_t, [_vp]),
    "hiccl_reduce_plan_destroy": (None, [_vp]),
    "hiccl_host_pipe_create": (ctypes.c_int, [ctypes.POINTER(_vp), ctypes.c_int, ctypes.c_int,
                                              ctypes.c_size_t, ctypes.c_int]),
    "hiccl_host_pipe_reduce": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_size_t]),
    "hiccl_host_pipe_destroy": (None, [_vp]),
    "hiccl_fill_uniform": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.c_size_t, ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.c_size_t, _vp]),
    "hiccl_stream_copy": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "hiccl_device_info": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp]),
    "hiccl_bucket_stride": (ctypes.c_size_t, [ctypes.c_int, ctypes.c_size_t]),
    "hiccl_bucket_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, _vp, _vp, _vp]),
    "hiccl_bucket_free": (ctypes.c_int, [_vp]),
    "hiccl_signal_wait": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_uint32, _vp,
                                         ctypes.c_double, _vp]),
    "hiccl_signal_wait_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_uint32, _vp, _vp,
                                             ctypes.c_double, _vp]),
    "hiccl_counter_add": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp]),
    "hiccl_signal_wait_phases": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, ctypes.c_double, _vp]),
    "hiccl_program_create": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "hiccl_program_add_signal": (ctypes.c_int, [_vp, _vp, ctypes.c_int, _vp, ctypes.c_int]),
    "hiccl_program_add_plan": (ctypes.c_int, [_vp, _vp]),
    "hiccl_program_set_max_workgroups": (ctypes.c_int, [_vp, ctypes.c_int]),
    "hiccl_program_num_units": (ctypes.c_int, [_vp]),
    "hiccl_program_num_phases": (ctypes.c_int, [_vp]),
    "hiccl_program_launch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_double, _vp]),
    "hiccl_program_destroy": (None, [_vp]),
    "hiccl_token_mode": (ctypes.c_int, []),
    "hiccl_step_program_default": (ctypes.c_int, []),
}


def lib():
    """Open libhiccl_reduce.so (once).  Raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"HIP extension missing: {LIB_PATH} not built. "
                "Run `python -c 'import __graft_entry__ as g; g.build()'` (or `make`).")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def header_functions(path=HEADER_PATH):
    """Names of every function declared in include/hiccl_reduce.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(hiccl_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def check(code, where):
    if code != 0:
        msg = lib().hiccl_last_error().decode(errors="replace")
        raise HicclError(code, where, msg)


def last_error():
    return lib().hiccl_last_error().decode(errors="replace")
