// hiccl_amd/csrc/readme_example.cpp -- the reference README's API example
// (README.md:12-60: in-place all-reduce composed from add_reduction +
// add_fence + add_multicast, init(hierarchy, lib, numstripe, ring, pipeline),
// repeated start()/wait()) against this build's HiCCL surface, with a check.
//
//   mpirun -np P build/readme_example_{hip,host} [count] [iterations] [rounds]
//
// Inputs are small integers so the float sums are exact in any order: every
// rank must end with recvbuf[i] == sum_p (p + 1) * ((i % 7) + 1).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hiccl.h"

#define T float

using namespace HiCCL;

int main(int argc, char **argv) {
  CommBench::init();
  const size_t count = argc > 1 ? std::atol(argv[1]) : (size_t)(1e6 / sizeof(T));
  const int numiter = argc > 2 ? std::atoi(argv[2]) : 3;

  // rounds > 1: a fresh communicator and fresh user buffers per round (the
  // previous round's are freed: a peer's new buffer may get the same address)
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 1;
  unsigned long failed = 0;
  // HICCL_README_KEEP_BUFFERS: one pair of user buffers for all rounds
  const bool keep = std::getenv("HICCL_README_KEEP_BUFFERS") != nullptr;
  T *sendbuf = nullptr;
  T *recvbuf = nullptr;
  for (int round = 0; round < rounds; round++) {
    if (!keep || round == 0) {
      allocate(sendbuf, count * numproc);
      allocate(recvbuf, count * numproc);
    }

    // the communicator goes before its buffers (its teardown is collective:
    // every peer releases its mappings of them first)
    {
      Comm<T> allreduce;

      // partial reductions (each GPU gathers count elements from all GPUs for reduction)
      for (int i = 0; i < numproc; i++) allreduce.add_reduction(sendbuf + i * count, recvbuf + i * count, count, HiCCL::all, i);
      // express ordering of the primitives
      allreduce.add_fence();
      // multicast partial results (each GPU sends count elements to all GPUs except itself)
      for (int i = 0; i < numproc; i++)
        allreduce.add_multicast(recvbuf + i * count, recvbuf + i * count, count, i, HiCCL::others);

      // optimization parameters: two-level hierarchy when the rank count allows
      std::vector<int> hierarchy = {numproc};
      std::vector<library> lib = {IPC};
      if (numproc % 2 == 0 && numproc > 2) {
        hierarchy = {numproc / 2, 2};
        lib = {MPI, IPC};
      }
      int numstripe(1);  // multi-rail striping (off)
      int ring(1);       // number of virtual ring nodes (off)
      int pipeline(4);   // pipeline depth
      allreduce.init(hierarchy, lib, numstripe, ring, pipeline);

      std::vector<T> host(count * numproc);
      for (size_t i = 0; i < host.size(); i++) host[i] = (T)((myid + 1 + round) * ((i % 7) + 1));
      CommBench::memcpyH2D(sendbuf, host.data(), host.size());

      for (int iter = 0; iter < numiter; iter++) {
        allreduce.start();  // nonblocking start
        allreduce.wait();   // blocking wait
      }

      std::vector<T> out(count * numproc);
      CommBench::memcpyD2H(out.data(), recvbuf, out.size());
      const double ranks = (double)numproc * (numproc + 1) / 2 + (double)round * numproc;
      size_t errors = 0;
      for (size_t i = 0; i < out.size(); i++)
        if (out[i] != (T)(ranks * ((i % 7) + 1))) {
          if (!errors)
            std::printf("rank %d round %d: first wrong element %zu (chunk %zu): %g, want %g\n", myid, round, i, i / count,
                        (double)out[i], ranks * ((i % 7) + 1));
          errors++;
        }
      unsigned long total = errors;
      MPI_Allreduce(MPI_IN_PLACE, &total, 1, MPI_UNSIGNED_LONG, MPI_SUM, comm_mpi);
      if (myid == 0) std::printf("README all-reduce: %s (%lu errors, %d ranks, count %zu, round %d)\n", total ? "FAILED" : "PASSED", total, numproc, count, round);
      failed += total;
#ifndef HICCL_PORT_HOST
      if (total) CommBench::ipc_log_dump();  // HICCL_DEBUG_IPC=2
#endif
    }
    if (!keep || round == rounds - 1) {
      free(sendbuf);
      free(recvbuf);
    }
  }
  MPI_Finalize();
  return failed ? 1 : 0;
}
