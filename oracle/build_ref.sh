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
