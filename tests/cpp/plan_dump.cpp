// tests/cpp/plan_dump.cpp -- TEST TOOL: run the C++ factorization
// (include/hiccl/plan.h + Schedule + merge_steps) for EVERY rank of a
// virtual machine in one process and print the resulting pipeline as JSON
// lines, so tests/test_schedule.py can execute it with numpy and compare it
// bit for bit with oracle/schedule.py (the restatement of the reference).
//
//   plan_dump numproc pattern count numstripe ringnodes pipedepth hierarchy libs
//
// Buffers are fake, rank-independent addresses: send = 1<<40, recv = 2<<40,
// temporaries of rank r from (3<<40) + r*(1<<36) upward (printed as "alloc").
#define HICCL_PORT_HOST
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../hiccl_amd/csrc/compose.h"

using T = float;

static std::vector<int> ints(const char *s) {
  std::vector<int> v;
  for (const char *p = s; *p;) {
    v.push_back(std::atoi(p));
    while (*p && *p != ',') p++;
    if (*p == ',') p++;
  }
  return v;
}

static std::vector<CommBench::library> libs_of(const char *s) {
  std::vector<CommBench::library> v;
  std::string t(s);
  size_t p = 0;
  while (p < t.size()) {
    size_t q = t.find(',', p);
    if (q == std::string::npos) q = t.size();
    std::string w = t.substr(p, q - p);
    v.push_back(w == "ipc" ? CommBench::IPC : w == "ipc_get" ? CommBench::IPC_get : w == "xccl" ? CommBench::XCCL : CommBench::MPI);
    p = q + 1;
  }
  return v;
}

static unsigned long long addr(const T *p) { return (unsigned long long)(uintptr_t)p; }

static void print_ptr(const T *p) {
  if (p)
    std::printf("%llu", addr(p));
  else
    std::printf("null");
}

int main(int argc, char **argv) {
  if (argc < 9) {
    std::fprintf(stderr, "usage: plan_dump numproc pattern count numstripe ringnodes pipedepth hierarchy libs\n");
    return 2;
  }
  const int np = std::atoi(argv[1]), pattern = std::atoi(argv[2]);
  const size_t count = std::atol(argv[3]);
  HiCCL::Schedule<T> sch;
  sch.numstripe = std::atoi(argv[4]);
  sch.ringnodes = std::atoi(argv[5]);
  sch.pipedepth = std::atoi(argv[6]);
  sch.hierarchy = ints(argv[7]);
  sch.library = libs_of(argv[8]);
  sch.fence();  // epoch 0
  T *send = (T *)(uintptr_t)(1ull << 40), *recv = (T *)(uintptr_t)(2ull << 40);
  CommBench::numproc = np;
  if (!hiccl_driver::compose(sch, pattern, send, recv, count, np, 0)) return 2;

  for (int r = 0; r < np; r++) {
    unsigned long long next = (3ull << 40) + (unsigned long long)r * (1ull << 36);
    HiCCL::Planner<T> P(r, np, [&](size_t n) {
      T *p = (T *)(uintptr_t)next;
      std::printf("{\"kind\":\"alloc\",\"rank\":%d,\"addr\":%llu,\"count\":%zu}\n", r, next, n);
      next += ((n * sizeof(T) + 255) / 256) * 256;
      return p;
    });
    auto batches = sch.factorize(P);
    auto libs = HiCCL::libraries_used(batches);
    auto steps = HiCCL::merge_steps(batches, libs, 1);
    std::printf("{\"kind\":\"meta\",\"rank\":%d,\"steps\":%zu,\"libs\":[", r, steps.size());
    for (size_t i = 0; i < libs.size(); i++) std::printf("%s%d", i ? "," : "", (int)libs[i]);
    std::printf("]}\n");
    for (size_t s = 0; s < steps.size(); s++) {
      for (size_t i = 0; i < libs.size(); i++) {
        const auto &c = steps[s][i];
        for (size_t j = 0; j < c.xfers.size(); j++) {
          const auto &x = c.xfers[j];
          std::printf("{\"kind\":\"xfer\",\"rank\":%d,\"step\":%zu,\"lib\":%d,\"idx\":%zu,\"sendid\":%d,\"recvid\":%d,\"count\":%zu,\"src\":",
                      r, s, (int)libs[i], j, x.sendid, x.recvid, x.count);
          print_ptr(r == x.sendid ? HiCCL::at(x.sendbuf, x.sendoffset) : nullptr);
          std::printf(",\"dst\":");
          print_ptr(r == x.recvid ? HiCCL::at(x.recvbuf, x.recvoffset) : nullptr);
          std::printf(",\"feeds\":%s}\n", x.feeds ? "true" : "false");
        }
        for (const auto &k : c.comps) {
          if (k.compid != r) continue;  // Compute::add records on the owner only
          std::printf("{\"kind\":\"comp\",\"rank\":%d,\"step\":%zu,\"lib\":%d,\"count\":%zu,\"out\":", r, s, (int)libs[i], k.count);
          print_ptr(k.output);
          std::printf(",\"in\":[");
          for (size_t q = 0; q < k.inputs.size(); q++) {
            if (q) std::printf(",");
            print_ptr(k.inputs[q]);
          }
          std::printf("]}\n");
        }
      }
    }
    for (auto &b : batches)
      for (auto *c : b) delete c;
  }
  return 0;
}
