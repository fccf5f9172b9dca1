// tests/cpp/ipc_reuse.cpp -- standalone reproducer of the HIP IPC behaviour
// the transport works around (include/hiccl/transport.h, IpcMapping:
// released mappings are retired, not closed).
//
// P processes (2..8; one device each, or all on device 0 of a one-GPU box),
// all-to-all like a communicator.  Per round, with `nbuf` buffers of
// `bytes` on every rank:
//   1. every rank hipMallocs A[0..nbuf), writes a nonce into each and
//      exports them to every other rank
//   2. every rank opens every peer's A, reads the nonces (copy engine and a
//      kernel), then releases the mappings by the case's policy: "close"
//      (hipIpcCloseMemHandle all), "keep" (leave all open), "mixed" (odd
//      ranks keep, even ranks close)
//   3. every rank hipFrees A and hipMallocs B of the same sizes (the
//      allocator usually hands A's addresses back), writes nonces, exports
//   4. every rank opens every peer's B and reads its nonces through the new
//      mappings, then closes them -- except in "late": there the A mappings
//      were kept open through 3-4 and are closed only now, while B's are
//      still open, and B is read once more after that close (the order a
//      capped retirement produces: an old mapping of a base closed after a
//      newer one of the same base was opened)
// Small buffers (1 MiB) are sub-allocated by HIP, large ones (64 MiB) are
// allocations of their own.  The reference exchanges hipIpcMemHandle_t
// across processes the same way (/root/reference/misc/test.md:85).
//
//   mpirun -np P build/ipc_reuse <rounds>   -> one JSON line per case (rank 0)
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
  uint64_t ok;  // 0: hipIpcGetMemHandle failed (recorded; peers skip it)
};

// read the first 8 bytes of `p` with the copy engine and with a kernel;
// bit 0 = copy engine saw `want`, bit 1 = kernel saw `want`
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

static uint64_t next_nonce(int me) {
  static uint64_t seq = 0x9e3779b97f4a7c15ull;
  seq = seq * 6364136223846793005ull + 1442695040888963407ull + (uint64_t)me;
  return seq;
}

// this rank's nbuf fresh allocations with nonces; every rank's exports.  A
// failed export is counted in *failed (an outcome this program records, like
// a failed open) and marked, so the peers do not open it.
static std::vector<void *> alloc_and_export(size_t bytes, int nbuf, int me, int np, std::vector<Export> &all,
                                            long *failed) {
  std::vector<void *> a(nbuf);
  std::vector<Export> mine(nbuf);
  for (int j = 0; j < nbuf; j++) {
    check(hipMalloc(&a[j], bytes), "hipMalloc");
    mine[j].nonce = next_nonce(me);
    check(hipMemcpy(a[j], &mine[j].nonce, 8, hipMemcpyHostToDevice), "write nonce");
    mine[j].ok = hipIpcGetMemHandle(&mine[j].h, a[j]) == hipSuccess;
    if (!mine[j].ok) {
      (void)hipGetLastError();
      (*failed)++;
    }
    mine[j].addr = (uint64_t)(uintptr_t)a[j];
  }
  check(hipDeviceSynchronize(), "sync");
  all.resize((size_t)np * nbuf);
  const int b = (int)(nbuf * sizeof(Export));
  MPI_Allgather(mine.data(), b, MPI_BYTE, all.data(), b, MPI_BYTE, MPI_COMM_WORLD);
  return a;
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int me = 0, np = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &me);
  MPI_Comm_size(MPI_COMM_WORLD, &np);
  if (np < 2) {
    if (me == 0) std::fprintf(stderr, "ipc_reuse: run with >= 2 ranks\n");
    MPI_Finalize();
    return 2;
  }
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
  int ndev = 0;
  check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  check(hipSetDevice(me % ndev), "hipSetDevice");
  uint64_t *scratch = nullptr;
  check(hipMalloc((void **)&scratch, 64), "hipMalloc(scratch)");
  const size_t sizes[2] = {(size_t)64 << 20, (size_t)1 << 20};
  const int nbufs[2] = {1, 3};
  for (size_t bytes : sizes)
    for (int nbuf : nbufs)
      for (const char *variant : {"close", "keep", "mixed", "late"}) {
        const std::string v = variant;
        const bool do_close = v == "close" || (v == "mixed" && me % 2 == 0);
        const bool late = v == "late";
        // B reads, A ok, recycled, B copy ok, B kernel ok, late reads, late ok, A opens, A open failed,
        // B open failed, A export failed, B export failed
        long st[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        std::vector<void *> kept;
        for (int r = 0; r < rounds; r++) {
          std::vector<Export> ea, eb;
          std::vector<void *> a = alloc_and_export(bytes, nbuf, me, np, ea, &st[10]);  // 1.
          std::vector<void *> ma;
          for (int p = 0; p < np; p++)  // 2.
            for (int j = 0; j < nbuf && p != me; j++) {
              const Export &e = ea[(size_t)p * nbuf + j];
              if (!e.ok) continue;
              void *m = nullptr;
              st[7]++;
              if (hipIpcOpenMemHandle(&m, e.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();  // recorded, not fatal: the outcome is what this program measures
                st[8]++;
                continue;
              }
              if (read_views(m, e.nonce, scratch) == 3) st[1]++;
              ma.push_back(m);
            }
          for (void *m : ma) {
            if (do_close) check(hipIpcCloseMemHandle(m), "close A");
            else if (!late) kept.push_back(m);
          }
          MPI_Barrier(MPI_COMM_WORLD);
          for (void *p : a) check(hipFree(p), "free A");  // 3.
          std::vector<void *> b = alloc_and_export(bytes, nbuf, me, np, eb, &st[11]);
          std::vector<void *> mb;
          std::vector<uint64_t> nb;
          for (int p = 0; p < np; p++)  // 4.
            for (int j = 0; j < nbuf && p != me; j++) {
              const Export &f = eb[(size_t)p * nbuf + j];
              if (!f.ok) continue;
              for (int i = 0; i < nbuf; i++)
                if (f.addr == ea[(size_t)p * nbuf + i].addr) st[2]++;
              void *m = nullptr;
              st[0]++;
              if (hipIpcOpenMemHandle(&m, f.h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                st[9]++;
                continue;
              }
              const int got = read_views(m, f.nonce, scratch);
              st[3] += got & 1;
              st[4] += (got >> 1) & 1;
              mb.push_back(m);
              nb.push_back(f.nonce);
            }
          if (late) {  // close A's mappings now, then read B through its (still open) mappings again
            for (void *m : ma) check(hipIpcCloseMemHandle(m), "late close A");
            for (size_t i = 0; i < mb.size(); i++) {
              st[5]++;
              st[6] += read_views(mb[i], nb[i], scratch) == 3;
            }
          }
          for (void *m : mb) check(hipIpcCloseMemHandle(m), "close B");
          MPI_Barrier(MPI_COMM_WORLD);
          for (void *p : b) check(hipFree(p), "free B");
          MPI_Barrier(MPI_COMM_WORLD);
        }
        for (void *m : kept) check(hipIpcCloseMemHandle(m), "close kept");
        long tot[12];
        MPI_Reduce(st, tot, 12, MPI_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
        if (me == 0)
          std::printf("{\"variant\": \"%s\", \"ranks\": %d, \"bytes\": %zu, \"buffers\": %d, \"rounds\": %d, "
                      "\"devices\": %d, \"first_opens\": %ld, \"first_open_failed\": %ld, \"first_mapping_ok\": %ld, "
                      "\"reads\": %ld, \"second_open_failed\": %ld, \"recycled_address\": %ld, "
                      "\"second_mapping_copy_engine_ok\": %ld, \"second_mapping_kernel_ok\": %ld, "
                      "\"late_close_reads\": %ld, \"after_late_close_ok\": %ld, \"first_export_failed\": %ld, "
                      "\"second_export_failed\": %ld}\n",
                      variant, np, bytes, nbuf, rounds, ndev, tot[7], tot[8], tot[1], tot[0], tot[9], tot[2], tot[3],
                      tot[4], tot[5], tot[6], tot[10], tot[11]);
        std::fflush(stdout);
        MPI_Barrier(MPI_COMM_WORLD);
      }
  check(hipFree(scratch), "free scratch");
  MPI_Finalize();
  return 0;
}
