// include/hiccl/bench.h -- HiCCL::measure and HiCCL::validate
// (reference: source/bench.h:1-227).
#ifndef HICCL_BENCH_H
#define HICCL_BENCH_H

#include <algorithm>
#include <cstdio>
#include <vector>

#include "comm.h"

namespace HiCCL {

enum collective { dummy, gather, scatter, broadcast, reduce, alltoall, allgather, reducescatter, allreduce };

// Sorted per-iteration times (seconds, MAX over ranks) of measure().
struct Times {
  std::vector<double> t;
  double min() const { return t.empty() ? 0 : t.front(); }
  double median() const { return t.empty() ? 0 : t[t.size() / 2]; }
  double max() const { return t.empty() ? 0 : t.back(); }
};

// bench.h:1-60: whole-collective time per iteration (barrier, run, MAX over
// ranks); GB/s priced on count * sizeof(T) (the user buffer).  Also returns
// the sorted times (the reference returns nothing).
template <typename T>
Times measure(int warmup, int numiter, size_t count, Comm<T> &comm) {
  std::vector<double> times;
  if (CommBench::myid == CommBench::printid) std::printf("%d warmup iterations (in order):\n", warmup);
  for (int it = -warmup; it < numiter; it++) {
#ifndef HICCL_PORT_HOST
    CommBench::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
#endif
    MPI_Barrier(CommBench::comm_mpi);
    double t = MPI_Wtime();
    comm.run();
    t = MPI_Wtime() - t;
    MPI_Allreduce(MPI_IN_PLACE, &t, 1, MPI_DOUBLE, MPI_MAX, CommBench::comm_mpi);
    if (it < 0) {
      if (CommBench::myid == CommBench::printid) std::printf("warmup: %e\n", t);
    } else {
      times.push_back(t);
    }
  }
  if (CommBench::myid == CommBench::printid) std::printf("Total ");
  Compute<T>::print_times(times, (double)count * sizeof(T));
  std::sort(times.begin(), times.end());
  return Times{times};
}

// bench.h:62-227: known-answer test.  sendbuf[i] = i on every rank, recv
// filled with 0xFF bytes, start()/wait(), exact check per collective.
// Returns true on every rank when all ranks pass.
template <typename T>
bool validate(T *sendbuf_d, T *recvbuf_d, size_t count, int patternid, int root, Comm<T> &comm) {
  const int np = CommBench::numproc, me = CommBench::myid;
  const size_t n = count * np;
  std::vector<T> sendbuf(n), recvbuf(n);
  for (size_t i = 0; i < n; i++) sendbuf[i] = (T)i;
#ifndef HICCL_PORT_HOST
  CommBench::hip_check(hipMemset(recvbuf_d, -1, n * sizeof(T)), "hipMemset");
#else
  std::memset((void *)recvbuf_d, -1, n * sizeof(T));  // the reference has no CPU branch (bench.h:65-79)
#endif
  CommBench::memcpyH2D(sendbuf_d, sendbuf.data(), n);
  MPI_Barrier(CommBench::comm_mpi);
  comm.start();
  comm.wait();
  CommBench::memcpyD2H(recvbuf.data(), recvbuf_d, n);
  MPI_Barrier(CommBench::comm_mpi);
  size_t errors = 0;
  auto expect = [&](size_t i, T v) {
    if (recvbuf[i] != v) errors++;
  };
  const char *name = "";
  switch (patternid) {
    case gather:
      name = "GATHER";
      if (me == root)
        for (int p = 0; p < np; p++)
          for (size_t i = 0; i < count; i++) expect(p * count + i, (T)i);
      break;
    case scatter:
      name = "SCATTER";
      for (size_t i = 0; i < count; i++) expect(i, (T)(me * count + i));
      break;
    case broadcast:
      name = "BCAST";
      for (size_t i = 0; i < n; i++) expect(i, (T)i);
      break;
    case reduce:
      name = "REDUCE";
      if (me == root)
        for (size_t i = 0; i < n; i++) expect(i, (T)(i * np));
      break;
    case alltoall:
      name = "ALL-TO-ALL";
      for (int p = 0; p < np; p++)
        for (size_t i = 0; i < count; i++) expect(p * count + i, (T)(me * count + i));
      break;
    case allgather:
      name = "ALL-GATHER";
      for (int p = 0; p < np; p++)
        for (size_t i = 0; i < count; i++) expect(p * count + i, (T)i);
      break;
    case reducescatter:
      name = "REDUCE-SCATTER";
      for (size_t i = 0; i < count; i++) expect(i, (T)((me * count + i) * np));
      break;
    case allreduce:
      name = "ALL-REDUCE";
      for (size_t i = 0; i < n; i++) expect(i, (T)(i * np));
      break;
    default:
      errors = 1;
  }
  int pass = errors == 0;
  MPI_Allreduce(MPI_IN_PLACE, &pass, 1, MPI_INT, MPI_LAND, CommBench::comm_mpi);
  unsigned long total = errors;
  MPI_Allreduce(MPI_IN_PLACE, &total, 1, MPI_UNSIGNED_LONG, MPI_SUM, CommBench::comm_mpi);
  if (me == CommBench::printid) {
    std::printf("VERIFY %s ROOT = %d: %s\n", name, root, pass ? "PASSED!" : "FAILED!!!");
    if (!pass) std::printf("count %zu total errorcount %lu\n", count, total);
  }
  return pass != 0;
}

}  // namespace HiCCL

#endif  // HICCL_BENCH_H
