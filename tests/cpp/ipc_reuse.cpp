// tests/cpp/ipc_reuse.cpp -- standalone two-process reproducer of the HIP IPC
// behaviour the transport works around (include/hiccl/transport.h,
// IpcMapping: released mappings are retired, not closed).
//
// Rank 0 (owner) and rank 1 (importer), one device each (or both on device 0
// of a one-GPU box).  Per round, with `nbuf` buffers of `bytes` each:
//   1. owner: hipMalloc A[0..nbuf), write nonce a_j into each, export each
//   2. importer: open each, read a_j (copy engine and a kernel), then, in
//      variant "close", hipIpcCloseMemHandle each -- in "keep", leave them open
//   3. owner: hipFree A[*], hipMalloc B[0..nbuf) of the same sizes (the
//      allocator usually hands A's addresses back), write nonces b_j, export
//   4. importer: open B[*], read b_j through the new mappings (copy engine
//      and a kernel: hiccl_stream_copy), record whether each view saw b_j
// Small buffers (1 MiB) are sub-allocated by HIP from larger chunks, large
// ones (64 MiB) are allocations of their own; the transport sees both (user
// buffers, schedule buffers).  The reference exchanges hipIpcMemHandle_t
// across processes the same way (/root/reference/misc/test.md:85).
//
//   mpirun -np 2 build/ipc_reuse <rounds>   -> one JSON line per case
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

static uint64_t next_nonce() {
  static uint64_t seq = 0x9e3779b97f4a7c15ull;
  seq = seq * 6364136223846793005ull + 1442695040888963407ull;
  return seq;
}

// owner: nbuf fresh allocations with nonces, exported to rank 1
static std::vector<void *> owner_round(size_t bytes, int nbuf, int tag) {
  std::vector<void *> a(nbuf);
  std::vector<Export> e(nbuf);
  for (int j = 0; j < nbuf; j++) {
    check(hipMalloc(&a[j], bytes), "hipMalloc");
    e[j].nonce = next_nonce();
    check(hipMemcpy(a[j], &e[j].nonce, 8, hipMemcpyHostToDevice), "write nonce");
    check(hipIpcGetMemHandle(&e[j].h, a[j]), "export");
    e[j].addr = (uint64_t)(uintptr_t)a[j];
  }
  MPI_Send(e.data(), (int)(nbuf * sizeof(Export)), MPI_BYTE, 1, tag, MPI_COMM_WORLD);
  return a;
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
  int ndev = 0;
  check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  check(hipSetDevice(me % ndev), "hipSetDevice");
  uint64_t *scratch = nullptr;
  check(hipMalloc((void **)&scratch, 64), "hipMalloc(scratch)");
  const size_t sizes[2] = {(size_t)64 << 20, (size_t)1 << 20};
  const int nbufs[2] = {1, 3};
  for (size_t bytes : sizes)
    for (int nbuf : nbufs)
      for (const char *variant : {"close", "keep"}) {
        const bool close_first = std::string(variant) == "close";
        int same_addr = 0, first_ok = 0, copy_ok = 0, kernel_ok = 0, reads = 0;
        std::vector<void *> kept;  // importer: mappings left open ("keep")
        for (int r = 0; r < rounds; r++) {
          std::vector<void *> a;
          std::vector<Export> e(nbuf), f(nbuf);
          if (me == 0) {
            a = owner_round(bytes, nbuf, 0);  // 1.
          } else {  // 2.
            MPI_Recv(e.data(), (int)(nbuf * sizeof(Export)), MPI_BYTE, 0, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
            std::vector<void *> m(nbuf);
            for (int j = 0; j < nbuf; j++) {
              check(hipIpcOpenMemHandle(&m[j], e[j].h, hipIpcMemLazyEnablePeerAccess), "open A");
              if (read_views(m[j], e[j].nonce, scratch) == 3) first_ok++;
            }
            for (int j = 0; j < nbuf; j++) {
              if (close_first) check(hipIpcCloseMemHandle(m[j]), "close A");
              else kept.push_back(m[j]);
            }
          }
          MPI_Barrier(MPI_COMM_WORLD);
          if (me == 0) {  // 3.
            for (void *p : a) check(hipFree(p), "free A");
            std::vector<void *> b = owner_round(bytes, nbuf, 1);
            MPI_Barrier(MPI_COMM_WORLD);  // the importer has read B
            for (void *p : b) check(hipFree(p), "free B");
          } else {  // 4.
            MPI_Recv(f.data(), (int)(nbuf * sizeof(Export)), MPI_BYTE, 0, 1, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
            for (int j = 0; j < nbuf; j++) {
              for (int i = 0; i < nbuf; i++)
                if (f[j].addr == e[i].addr) same_addr++;
              void *m = nullptr;
              check(hipIpcOpenMemHandle(&m, f[j].h, hipIpcMemLazyEnablePeerAccess), "open B");
              const int v = read_views(m, f[j].nonce, scratch);
              copy_ok += v & 1;
              kernel_ok += (v >> 1) & 1;
              reads++;
              check(hipIpcCloseMemHandle(m), "close B");
            }
            MPI_Barrier(MPI_COMM_WORLD);
          }
          MPI_Barrier(MPI_COMM_WORLD);
        }
        for (void *m : kept) check(hipIpcCloseMemHandle(m), "close kept");
        if (me == 1)
          std::printf("{\"variant\": \"%s\", \"bytes\": %zu, \"buffers\": %d, \"rounds\": %d, \"devices\": %d, "
                      "\"reads\": %d, \"first_mapping_ok\": %d, \"recycled_address\": %d, "
                      "\"second_mapping_copy_engine_ok\": %d, \"second_mapping_kernel_ok\": %d}\n",
                      variant, bytes, nbuf, rounds, ndev, reads, first_ok, same_addr, copy_ok, kernel_ok);
        std::fflush(stdout);
        MPI_Barrier(MPI_COMM_WORLD);
      }
  check(hipFree(scratch), "free scratch");
  MPI_Finalize();
  return 0;
}
