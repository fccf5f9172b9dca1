// tests/cpp/ipc_reuse.cpp -- standalone two-process reproducer of the HIP IPC
// behaviour the transport works around (include/hiccl/transport.h,
// IpcMapping: released mappings are retired, not closed).
//
// Rank 0 (owner) and rank 1 (importer), one device each (or both on device 0
// of a one-GPU box).  Per round:
//   1. owner: hipMalloc A, write nonce a, export A's handle
//   2. importer: open A, read a (copy engine and a kernel), then, in variant
//      "close", hipIpcCloseMemHandle(A) -- in variant "keep", leave it open
//   3. owner: hipFree A, hipMalloc B of the same size (the allocator usually
//      hands A's address back), write nonce b, export B
//   4. importer: open B, read b through the new mapping (copy engine and a
//      kernel: hiccl_stream_copy), record whether each view saw b
// The reference exchanges hipIpcMemHandle_t across processes the same way
// (/root/reference/misc/test.md:85); the transport's CommBench layer opens
// one mapping per peer allocation (tests/test_ipc_reuse_gpu.py runs this).
//
//   mpirun -np 2 build/ipc_reuse <rounds> <bytes>   -> one JSON line per variant
#include <hip/hip_runtime_api.h>
#include <mpi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hiccl_reduce.h"

static void check(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "ipc_reuse: %s: %s\n", what, hipGetErrorString(e));
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
}

struct Export {
  hipIpcMemHandle_t h;
  uint64_t addr;
  uint64_t nonce;
};

// importer: read the first 8 bytes of `p` with the copy engine and with a
// kernel; bit 0 = copy engine saw `want`, bit 1 = kernel saw `want`
static int read_views(const void *p, uint64_t want, uint64_t *scratch) {
  uint64_t got = 0, got_k = 0;
  check(hipMemcpy(&got, p, 8, hipMemcpyDeviceToHost), "read (copy engine)");
  if (hiccl_stream_copy(scratch, p, 8, nullptr)) {
    std::fprintf(stderr, "ipc_reuse: hiccl_stream_copy: %s\n", hiccl_last_error());
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  check(hipDeviceSynchronize(), "sync");
  check(hipMemcpy(&got_k, scratch, 8, hipMemcpyDeviceToHost), "read (kernel)");
  return (got == want ? 1 : 0) | (got_k == want ? 2 : 0);
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int me = 0, np = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &me);
  MPI_Comm_size(MPI_COMM_WORLD, &np);
  if (np != 2) {
    if (me == 0) std::fprintf(stderr, "ipc_reuse: run with 2 ranks\n");
    MPI_Finalize();
    return 2;
  }
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 8;
  const size_t bytes = argc > 2 ? (size_t)std::atoll(argv[2]) : ((size_t)64 << 20);
  int ndev = 0;
  check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  check(hipSetDevice(me % ndev), "hipSetDevice");
  uint64_t *scratch = nullptr;
  check(hipMalloc((void **)&scratch, 64), "hipMalloc(scratch)");
  uint64_t seq = 0x9e3779b97f4a7c15ull;
  for (const char *variant : {"close", "keep"}) {
    const bool close_first = std::string(variant) == "close";
    int same_addr = 0, first_ok = 0, copy_ok = 0, kernel_ok = 0;
    std::vector<void *> kept;  // importer: mappings left open ("keep")
    for (int r = 0; r < rounds; r++) {
      Export e{};
      void *a = nullptr;
      if (me == 0) {  // 1.
        check(hipMalloc(&a, bytes), "hipMalloc(A)");
        seq = seq * 6364136223846793005ull + 1442695040888963407ull;
        e.nonce = seq;
        check(hipMemcpy(a, &e.nonce, 8, hipMemcpyHostToDevice), "write a");
        check(hipIpcGetMemHandle(&e.h, a), "export A");
        e.addr = (uint64_t)(uintptr_t)a;
        MPI_Send(&e, sizeof(e), MPI_BYTE, 1, 0, MPI_COMM_WORLD);
      } else {  // 2.
        MPI_Recv(&e, sizeof(e), MPI_BYTE, 0, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
        void *m = nullptr;
        check(hipIpcOpenMemHandle(&m, e.h, hipIpcMemLazyEnablePeerAccess), "open A");
        if (read_views(m, e.nonce, scratch) == 3) first_ok++;
        if (close_first) check(hipIpcCloseMemHandle(m), "close A");
        else kept.push_back(m);
      }
      MPI_Barrier(MPI_COMM_WORLD);
      Export f{};
      if (me == 0) {  // 3.
        check(hipFree(a), "free A");
        void *b = nullptr;
        check(hipMalloc(&b, bytes), "hipMalloc(B)");
        seq = seq * 6364136223846793005ull + 1442695040888963407ull;
        f.nonce = seq;
        check(hipMemcpy(b, &f.nonce, 8, hipMemcpyHostToDevice), "write b");
        check(hipIpcGetMemHandle(&f.h, b), "export B");
        f.addr = (uint64_t)(uintptr_t)b;
        MPI_Send(&f, sizeof(f), MPI_BYTE, 1, 1, MPI_COMM_WORLD);
        MPI_Barrier(MPI_COMM_WORLD);  // the importer has read B
        check(hipFree(b), "free B");
      } else {  // 4.
        MPI_Recv(&f, sizeof(f), MPI_BYTE, 0, 1, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
        if (f.addr == e.addr) same_addr++;
        void *m = nullptr;
        check(hipIpcOpenMemHandle(&m, f.h, hipIpcMemLazyEnablePeerAccess), "open B");
        const int v = read_views(m, f.nonce, scratch);
        copy_ok += v & 1;
        kernel_ok += (v >> 1) & 1;
        check(hipIpcCloseMemHandle(m), "close B");
        MPI_Barrier(MPI_COMM_WORLD);
      }
      MPI_Barrier(MPI_COMM_WORLD);
    }
    for (void *m : kept) check(hipIpcCloseMemHandle(m), "close kept");
    if (me == 1)
      std::printf("{\"variant\": \"%s\", \"rounds\": %d, \"bytes\": %zu, \"devices\": %d, \"first_mapping_ok\": %d, "
                  "\"recycled_address\": %d, \"second_mapping_copy_engine_ok\": %d, "
                  "\"second_mapping_kernel_ok\": %d}\n",
                  variant, rounds, bytes, ndev, first_ok, same_addr, copy_ok, kernel_ok);
    std::fflush(stdout);
    MPI_Barrier(MPI_COMM_WORLD);
  }
  check(hipFree(scratch), "free scratch");
  MPI_Finalize();
  return 0;
}
