// include/hiccl.h -- HiCCL C++ surface, MI355X-native build.
//
// Drop-in for the reference's hiccl.h (hiccl.h:16-54): namespace HiCCL with
// Comm<T> (add_reduce / add_bcast / add_fence / set_* / init / run / start /
// wait / measure, plus the README spellings add_reduction / add_multicast /
// init(hierarchy, lib, numstripe, ring, pipeline)), Compute<T>, measure(),
// validate(), the pattern / collective enums, and the transport names the
// reference and collectives/main.cpp take from CommBench.
//
// Port selection (the reference's PORT_* macros, hiccl.h:19-22):
//   default            HIP on gfx950: the reduction is libhiccl_reduce.so
//                      (hand-written CDNA4 kernels behind include/hiccl_reduce.h);
//                      link -lhiccl_reduce -lamdhip64 and compile this header
//                      with hipcc, or g++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include.
//   HICCL_PORT_HOST    host-only build for machines without a GPU (config 1):
//                      host buffers, MPI transport, OpenMP reduction.
// MPI (mpi.h) is required in both, as in the reference.
#ifndef HICCL_H
#define HICCL_H

#include "hiccl/transport.h"
#include "hiccl/compute.h"
#include "hiccl/plan.h"
#include "hiccl/command.h"
#include "hiccl/comm.h"
#include "hiccl/bench.h"

namespace HiCCL {

// hiccl.h:31-38
inline const MPI_Comm &comm_mpi = CommBench::comm_mpi;
inline const int &numproc = CommBench::numproc;
inline const int &myid = CommBench::myid;
inline int printid = 0;

// README.md:31-48 uses the library names unqualified under `using namespace HiCCL`.
using CommBench::library;
inline constexpr CommBench::library IPC = CommBench::IPC;
inline constexpr CommBench::library IPC_get = CommBench::IPC_get;
inline constexpr CommBench::library MPI = CommBench::MPI;
inline constexpr CommBench::library XCCL = CommBench::XCCL;
using CommBench::allocate;
using CommBench::free;

}  // namespace HiCCL

#endif  // HICCL_H
