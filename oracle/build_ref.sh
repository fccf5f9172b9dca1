#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
#
# Compiles the reference's OWN CPU reduction, reduce_kernel<T>
# (/root/reference/source/compute.h:14-23, the branch taken when no PORT_*
# macro is defined), into oracle/_ref/libhiccl_ref.so.  The function is
# read straight out of the reference header (the lines between the first
# `#else` and `#endif` of compute.h) and piped to g++ on stdin, so no
# reference source is ever written into this repository.  The fragment
# needs nothing but <cstddef> (size_t) -- no CommBench, no MPI, no stand-in
# headers: the rest of HiCCL (whose CommBench submodule is not vendored,
# .gitmodules:1-3) is NOT built.  It is wrapped in `namespace HiCCL` exactly
# as hiccl.h:29,43 includes it, and explicitly instantiated for the types the
# reference drivers use (float: main.cu:10; size_t: collectives/main.cpp:24)
# plus double and int32.
#
# usage: build_ref.sh <reference-root> <output.so>
set -euo pipefail
REF=${1:-/root/reference}
OUT=${2:-$(dirname "$0")/_ref/libhiccl_ref.so}
SRC="$REF/source/compute.h"
[ -f "$SRC" ] || { echo "build_ref: $SRC not found (reference absent) -- skipping" >&2; exit 0; }
mkdir -p "$(dirname "$OUT")"
FRAG=$(awk '/^#else/{f=1;next} /^#endif/{if(f)exit} f' "$SRC")
grep -q 'void reduce_kernel' <<<"$FRAG" || { echo "build_ref: reduce_kernel not found in $SRC" >&2; exit 1; }
{
  echo '#include <cstddef>'
  echo '#include <cstdint>'
  echo 'namespace HiCCL {'
  echo "#line 14 \"$SRC\""
  echo "$FRAG"
  echo '}'
  echo '#line 1 "oracle/build_ref.sh:wrapper"'
  echo 'extern "C" void ref_reduce_f32(float *o, size_t c, float **in, int n) { HiCCL::reduce_kernel<float>(o, c, in, n); }'
  echo 'extern "C" void ref_reduce_f64(double *o, size_t c, double **in, int n) { HiCCL::reduce_kernel<double>(o, c, in, n); }'
  echo 'extern "C" void ref_reduce_u64(size_t *o, size_t c, size_t **in, int n) { HiCCL::reduce_kernel<size_t>(o, c, in, n); }'
  echo 'extern "C" void ref_reduce_i32(int32_t *o, size_t c, int32_t **in, int n) { HiCCL::reduce_kernel<int32_t>(o, c, in, n); }'
} | g++ -x c++ -std=c++17 -O3 -fopenmp -fwrapv -fPIC -shared -o "$OUT" -
# (-fwrapv: a signed int32 sum that overflows wraps in two's complement, as
# the GPU's integer adds do, instead of being undefined in C++)
echo "build_ref: built $OUT from $SRC"

# The same fragment instantiated for bf16 with ROCm's own host bf16 type,
# __hip_bfloat16 (<hip/hip_bf16.h>: `T acc = 0` and `acc += x` are the
# compiler's __bf16 add, rounded to bf16 after every add) -- the type a HIP
# user of reduce_kernel<T> would instantiate.  clang++ (ROCm's) is needed for
# __bf16 on the host; no OpenMP runtime is linked (the pragma is ignored, the
# loop's result does not depend on it).
OUT16="$(dirname "$OUT")/libhiccl_ref_bf16.so"
CLANG=/opt/rocm/llvm/bin/clang++
if [ -x "$CLANG" ] && [ -f /opt/rocm/include/hip/hip_bf16.h ]; then
  {
    echo '#include <cstddef>'
    echo '#include <cstdint>'
    echo '#include <hip/hip_bf16.h>'
    echo 'namespace HiCCL {'
    echo "#line 14 \"$SRC\""
    echo "$FRAG"
    echo '}'
    echo '#line 1 "oracle/build_ref.sh:wrapper_bf16"'
    echo 'static_assert(sizeof(__hip_bfloat16) == 2, "bf16 storage");'
    echo 'extern "C" void ref_reduce_bf16(uint16_t *o, size_t c, uint16_t **in, int n) {'
    echo '  HiCCL::reduce_kernel<__hip_bfloat16>(reinterpret_cast<__hip_bfloat16 *>(o), c, reinterpret_cast<__hip_bfloat16 **>(in), n); }'
  } | "$CLANG" -x c++ -std=c++17 -O2 -Wno-unknown-pragmas -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -fPIC -shared -o "$OUT16" -
  echo "build_ref: built $OUT16 from $SRC (reduce_kernel<__hip_bfloat16>)"
fi

# ---------------------------------------------------------------------------
# The reference's own GPU kernel (compute.h:2-12, the PORT_CUDA / PORT_HIP
# branch: the lines between `#if defined PORT_CUDA || defined PORT_HIP` and
# the first `#else`), compiled for gfx950 by hipcc into
# oracle/_ref/libhiccl_ref_hip.so, with launchers that launch it exactly as
# Compute<T>::start does (compute.h:88-91: block 256, ceil(count / 256)
# workgroups, the caller's stream, a device array of input pointers).  The
# GPU tier compares this build's kernels with it on the same device (bits and
# time, tests/test_ref_hip_gpu.py); nothing in the product calls it.
OUTHIP="$(dirname "$OUT")/libhiccl_ref_hip.so"
GFRAG=$(awk '/^#if defined PORT_CUDA \|\| defined PORT_HIP/{f=1;next} /^#else/{if(f)exit} f' "$SRC")
if [ -x /opt/rocm/bin/hipcc ] && grep -q '__global__ void reduce_kernel' <<<"$GFRAG"; then
  TMPD=$(mktemp -d)
  {
    echo '#include <hip/hip_runtime.h>'
    echo '#include <hip/hip_bf16.h>'
    echo '#include <cstddef>'
    echo '#include <cstdint>'
    echo 'namespace HiCCL {'
    echo "#line 3 \"$SRC\""
    echo "$GFRAG"
    echo '}'
    echo '#line 1 "oracle/build_ref.sh:wrapper_hip"'
    echo 'template <typename T> static int launch(T *o, size_t c, T **in_d, int n, hipStream_t s) {'
    echo '  int blocksize = 256;'
    echo '  if (c) HiCCL::reduce_kernel<T><<<(c + blocksize - 1) / blocksize, blocksize, 0, s>>>(o, c, in_d, n);'
    echo '  return (int)hipGetLastError(); }'
    echo 'extern "C" int ref_hip_reduce_f32(float *o, size_t c, float **in_d, int n, hipStream_t s) { return launch(o, c, in_d, n, s); }'
    echo 'extern "C" int ref_hip_reduce_f64(double *o, size_t c, double **in_d, int n, hipStream_t s) { return launch(o, c, in_d, n, s); }'
    echo 'extern "C" int ref_hip_reduce_u64(size_t *o, size_t c, size_t **in_d, int n, hipStream_t s) { return launch(o, c, in_d, n, s); }'
    echo 'extern "C" int ref_hip_reduce_i32(int32_t *o, size_t c, int32_t **in_d, int n, hipStream_t s) { return launch(o, c, in_d, n, s); }'
    echo 'extern "C" int ref_hip_reduce_bf16(__hip_bfloat16 *o, size_t c, __hip_bfloat16 **in_d, int n, hipStream_t s) { return launch(o, c, in_d, n, s); }'
  } > "$TMPD/ref_gpu.hip"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$OUTHIP" "$TMPD/ref_gpu.hip"
  rm -rf "$TMPD"
  echo "build_ref: built $OUTHIP from $SRC (reduce_kernel<T> GPU branch, gfx950)"
fi

# ---------------------------------------------------------------------------
# Drop-in check: the reference's OWN driver, collectives/main.cpp, compiled
# unmodified against THIS build's include/hiccl.h.  The source is fed on
# stdin from inside include/hiccl/, so its `#include "../hiccl.h"`
# (collectives/main.cpp:17) resolves to include/hiccl.h; nothing is edited or
# copied.  Host port (no GPU) and HIP port (gfx950 reduction library).
DRV="$REF/collectives/main.cpp"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUTDIR=$(cd "$(dirname "$OUT")" && pwd)
MPI_INC=${MPI_INC:-/opt/conda/include}
MPI_LIB=${MPI_LIB:-/opt/conda/lib}
if [ -f "$DRV" ] && [ -f "$MPI_INC/mpi.h" ]; then
  MPI_LINK="$MPI_LIB/libmpi.so -Wl,-rpath,/usr/lib/x86_64-linux-gnu:$MPI_LIB"
  ( cd "$ROOT/include/hiccl" && g++ -std=c++17 -O2 -fopenmp -DHICCL_PORT_HOST -I"$MPI_INC" \
      -x c++ - -x none -o "$OUTDIR/collectives_main_host" $MPI_LINK < "$DRV" )
  echo "build_ref: built $OUTDIR/collectives_main_host from $DRV against include/hiccl.h"
  # the HIP port needs the product library: a missing one is a build-order
  # error, never a silent skip (tests/test_reference_driver.py fails when the
  # stamp below exists and a driver does not)
  [ -f "$ROOT/hiccl_amd/libhiccl_reduce.so" ] || {
    echo "build_ref: hiccl_amd/libhiccl_reduce.so missing -- build it first (make)" >&2; exit 1; }
  ( cd "$ROOT/include/hiccl" && g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -DHICCL_WITH_RCCL -I/opt/rocm/include -I"$MPI_INC" \
      -x c++ - -x none -o "$OUTDIR/collectives_main_hip" \
      -L"$ROOT/hiccl_amd" -lhiccl_reduce -Wl,-rpath,'$ORIGIN/../../hiccl_amd' \
      -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib $MPI_LINK < "$DRV" )
  echo "build_ref: built $OUTDIR/collectives_main_hip from $DRV against include/hiccl.h"
  # stamp: this tree was built where the reference was present, so every
  # reference-built artefact must exist wherever the tree is tested
  echo "reference: $REF" > "$OUTDIR/BUILT_FROM_REFERENCE"
fi
