// tests/cpp/ipc_reuse.cpp -- HIP IPC across buffer reuse (2 ranks, any GPUs).
//
// The pattern of a re-created communicator (tests/test_mpi_gpu.py
// test_readme_api_example): every round rank 0 allocates two buffers S and R
// (the allocator hands the freed addresses back, swapped), exports R
// `exports` times (one hipIpcGetMemHandle per transfer into it), rank 1 opens
// the first handle, writes the second half of R through it with a kernel
// (hiccl_stream_copy), rank 0 writes the first half itself with a kernel and
// checks both halves; then rank 1 closes its mapping, a barrier, and rank 0
// frees S and R.  Prints whether the handle bytes repeat across rounds.
//   mpirun -np 2 build/ipc_reuse [rounds] [bytes] [exports]
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

static size_t count_not(const unsigned char *h, size_t n, unsigned char v) {
  size_t k = 0;
  for (size_t i = 0; i < n; i++) k += h[i] != v;
  return k;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int me = 0;
  MPI_Comm_rank(MPI_COMM_WORLD, &me);
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
  const size_t bytes = argc > 2 ? (size_t)std::atoll(argv[2]) : (size_t)2000000;
  const int exports = argc > 3 ? std::atoi(argv[3]) : 4;
  const size_t half = bytes / 2;
  int ndev = 0;
  CHECK(hipGetDeviceCount(&ndev));
  CHECK(hipSetDevice(me % ndev));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *local = nullptr;
  CHECK(hipMalloc(&local, bytes));
  std::vector<unsigned char> h(bytes);
  std::vector<unsigned char> prev(sizeof(hipIpcMemHandle_t), 0);
  int bad = 0;
  const int peer = 1 - me;
  for (int r = 0; r < rounds; r++) {
    // both ranks: S and R, R exported `exports` times; rank k owns half k of
    // every R, writes it in its own R with its own kernel and in the peer's R
    // through the peer's mapping
    const unsigned char val[2] = {(unsigned char)(r + 1), (unsigned char)(101 + r)};
    void *S = nullptr, *R = nullptr, *q = nullptr;
    std::vector<hipIpcMemHandle_t> hs(exports), peer_hs(exports);
    CHECK(hipMalloc(&S, bytes));
    CHECK(hipMalloc(&R, bytes));
    for (int k = 0; k < exports; k++) CHECK(hipIpcGetMemHandle(&hs[k], R));
    MPI_Sendrecv(hs.data(), (int)(exports * sizeof(hipIpcMemHandle_t)), MPI_BYTE, peer, r, peer_hs.data(),
                 (int)(exports * sizeof(hipIpcMemHandle_t)), MPI_BYTE, peer, r, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    const bool same = std::memcmp(prev.data(), &hs[0], sizeof(hs[0])) == 0;
    std::memcpy(prev.data(), &hs[0], sizeof(hs[0]));
    CHECK(hipIpcOpenMemHandle(&q, peer_hs[0], hipIpcMemLazyEnablePeerAccess));
    char *mine_half = (char *)R + (me ? half : 0);
    char *theirs_half = (char *)q + (me ? half : 0);
    const size_t n_mine = me ? bytes - half : half;
    CHECK(hipMemset(local, val[me], bytes));
    CHECK(hipDeviceSynchronize());
    if (hiccl_stream_copy(mine_half, local, n_mine, s)) MPI_Abort(MPI_COMM_WORLD, 2);
    if (hiccl_stream_copy(theirs_half, local, n_mine, s)) MPI_Abort(MPI_COMM_WORLD, 2);
    CHECK(hipStreamSynchronize(s));
    MPI_Barrier(MPI_COMM_WORLD);
    CHECK(hipMemcpy(h.data(), R, bytes, hipMemcpyDeviceToHost));
    const size_t w0 = count_not(h.data(), half, val[0]), w1 = count_not(h.data() + half, bytes - half, val[1]);
    std::printf("round %d rank %d: S %p R %p mapped %p, handle %s, half0 %zu wrong, half1 %zu wrong\n", r, me, S, R, q,
                same ? "REPEATED" : "new", w0, w1);
    bad += (w0 || w1);
    CHECK(hipIpcCloseMemHandle(q));
    MPI_Barrier(MPI_COMM_WORLD);
    CHECK(hipFree(S));
    CHECK(hipFree(R));
  }
  MPI_Allreduce(MPI_IN_PLACE, &bad, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
  if (me == 0) std::printf("ipc_reuse: %s (%d bad rounds of %d)\n", bad ? "FAILED" : "PASSED", bad, rounds);
  MPI_Finalize();
  return bad ? 1 : 0;
}
