"""hiccl_amd -- HiCCL's local bucket-reduction stage, MI355X-native.

The compute is a hand-written HIP kernel for gfx950 in libhiccl_reduce.so
behind the C ABI of include/hiccl_reduce.h; the C++ drop-in surface
(HiCCL::Comm<T> / HiCCL::Compute<T>) is include/hiccl.h.  This Python
package is the binding used by the tests and bench.py.
"""
from ._lib import (HICCL_ACC_NATIVE, HICCL_ACC_WIDE, HICCL_BFLOAT16, HICCL_ENGINE_AUTO,  # noqa: F401
                   HICCL_ENGINE_PHASE, HICCL_ENGINE_TILE, HICCL_FLOAT32, HICCL_FLOAT64, HICCL_INT32, HICCL_UINT64, HicclError, LIB_PATH, header_functions,
                   lib)
from .compute import (Compute, HostPipe, Program, auto_choice, bucket, fill_uniform, reduce, reduce_ptrs,  # noqa: F401
                      stream_copy)

__version__ = "0.1.0"
