// tests/cpp/ipc_reuse.cpp -- HIP IPC across buffer reuse (2 ranks, any GPUs).
//
// Each round rank 0 allocates a buffer of the same size (the allocator hands
// back the freed address), fills it with the round number and exports it;
// rank 1 opens the handle, reads it with a KERNEL (hiccl_stream_copy into a
// local buffer) and writes a pattern into it with a kernel; rank 0 checks the
// pattern landed, then frees.  Rank 1 closes the previous round's mapping
// only right before it opens the next one, i.e. AFTER rank 0 allocated the
// next buffer -- so that buffer gets new physical memory at the old virtual
// address, and rank 1 typically maps it at its old virtual address too: a
// stale translation or cache line on either side shows up as wrong bytes.
//   mpirun -np 2 build/ipc_reuse [rounds] [bytes]
#include <hip/hip_runtime.h>
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hiccl_reduce.h"

#define CHECK(x)                                                                                     \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      MPI_Abort(MPI_COMM_WORLD, 1);                                                                  \
    }                                                                                                \
  } while (0)

static size_t count_not(const std::vector<unsigned char> &h, unsigned char v) {
  size_t n = 0;
  for (unsigned char c : h) n += c != v;
  return n;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int me = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &me);
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
  const size_t bytes = argc > 2 ? (size_t)std::atoll(argv[2]) : (size_t)1 << 22;
  int ndev = 0;
  CHECK(hipGetDeviceCount(&ndev));
  CHECK(hipSetDevice(me % ndev));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *local = nullptr;
  CHECK(hipMalloc(&local, bytes));
  std::vector<unsigned char> h(bytes);
  int bad = 0;
  void *q = nullptr;  // rank 1: the current mapping
  for (int r = 0; r < rounds; r++) {
    struct {
      hipIpcMemHandle_t h;
      unsigned long long va;
    } msg;
    void *p = nullptr;
    const unsigned char mine = (unsigned char)(r + 1), theirs = (unsigned char)(101 + r);
    if (me == 0) {
      CHECK(hipMalloc(&p, bytes));
      CHECK(hipMemset(p, mine, bytes));
      CHECK(hipDeviceSynchronize());
      CHECK(hipIpcGetMemHandle(&msg.h, p));
      msg.va = (unsigned long long)(uintptr_t)p;
      MPI_Send(&msg, sizeof(msg), MPI_BYTE, 1, r, MPI_COMM_WORLD);
    } else if (me == 1) {
      MPI_Recv(&msg, sizeof(msg), MPI_BYTE, 0, r, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
      if (q) CHECK(hipIpcCloseMemHandle(q));  // the previous round's, only now
      CHECK(hipIpcOpenMemHandle(&q, msg.h, hipIpcMemLazyEnablePeerAccess));
      // kernel read through the mapping
      if (hiccl_stream_copy(local, q, bytes, s)) MPI_Abort(MPI_COMM_WORLD, 2);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(h.data(), local, bytes, hipMemcpyDeviceToHost));
      const size_t rd = count_not(h, mine);
      // kernel write through the mapping
      CHECK(hipMemset(local, theirs, bytes));
      CHECK(hipDeviceSynchronize());
      if (hiccl_stream_copy(q, local, bytes, s)) MPI_Abort(MPI_COMM_WORLD, 2);
      CHECK(hipStreamSynchronize(s));
      std::printf("round %d: exporter va %#llx, mapped at %p, kernel read %zu wrong bytes\n", r, msg.va, q, rd);
      bad += rd != 0;
    }
    MPI_Barrier(MPI_COMM_WORLD);
    if (me == 0) {
      CHECK(hipMemcpy(h.data(), p, bytes, hipMemcpyDeviceToHost));
      const size_t wr = count_not(h, theirs);
      std::printf("round %d: peer kernel write %zu wrong bytes\n", r, wr);
      bad += wr != 0;
      CHECK(hipFree(p));
    }
    MPI_Barrier(MPI_COMM_WORLD);
  }
  if (q) CHECK(hipIpcCloseMemHandle(q));
  MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  if (me == 0) std::printf("ipc_reuse: %s (%d bad checks over %d rounds)\n", bad ? "FAILED" : "PASSED", bad, rounds);
  MPI_Finalize();
  return bad ? 1 : 0;
}
