// hiccl_amd/csrc/collectives.cpp -- this build's counterpart of the
// reference driver collectives/main.cpp: compose one of the eight
// collectives from HiCCL primitives, init, measure per command and whole
// collective, validate with the known-answer test.
//
//   mpirun -np P build/collectives_{hip,host} pattern count numstripe ringnodes
//          pipedepth warmup numiter [hierarchy libs] [dump_prefix]
//
//   pattern   1 gather .. 8 allreduce (hiccl.h:41)
//   count     elements per rank per chunk (collectives/main.cpp:48)
//   hierarchy comma list, e.g. 1,4,2 (default: numproc)      -- set_hierarchy
//   libs      comma list of ipc|ipc_get|mpi|xccl per level    (default mpi)
//   dump_prefix  if given, float inputs from the counter hash are used and
//             every rank writes <prefix>.rank<r>.bin (its recvbuf) so tests
//             can compare the exact bits with oracle/schedule.py.
//
// Element type: size_t (as the reference driver, collectives/main.cpp:24) or
// float with -DHICCL_DRIVER_FLOAT.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>
#include <vector>

#include "compose.h"

#ifdef HICCL_DRIVER_FLOAT
typedef float Type;
#else
typedef size_t Type;
#endif

static std::vector<int> parse_ints(const char *s) {
  std::vector<int> v;
  std::string t(s);
  size_t p = 0;
  while (p <= t.size()) {
    size_t q = t.find(',', p);
    if (q == std::string::npos) q = t.size();
    if (q > p) v.push_back(std::atoi(t.substr(p, q - p).c_str()));
    p = q + 1;
  }
  return v;
}

static std::vector<CommBench::library> parse_libs(const char *s) {
  std::vector<CommBench::library> v;
  std::string t(s);
  size_t p = 0;
  while (p <= t.size()) {
    size_t q = t.find(',', p);
    if (q == std::string::npos) q = t.size();
    std::string w = t.substr(p, q - p);
    if (w == "ipc") v.push_back(CommBench::IPC);
    else if (w == "ipc_get") v.push_back(CommBench::IPC_get);
    else if (w == "mpi") v.push_back(CommBench::MPI);
    else if (w == "xccl") v.push_back(CommBench::XCCL);
    else if (!w.empty()) CommBench::die("driver", "unknown library " + w);
    p = q + 1;
  }
  return v;
}

// oracle/reduce_oracle.c's generator (uniform [-1,1) of hash(seed, k, i)).
static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline float uniform_f32(uint64_t seed, uint32_t k, uint64_t i) {
  uint64_t h = splitmix64(splitmix64(seed ^ ((uint64_t)k << 48)) + i);
  return (float)(uint32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;
}

// The known-answer pattern times `ranks`: ranks * ((i mod 1021) - 510).
static inline int64_t kat_value(size_t i, int ranks) { return (int64_t)ranks * ((int64_t)(i % 1021) - 510); }

// HICCL_DRIVER_JSON=<path> (rank 0 writes it): HiCCL::measure of the whole
// collective (bench.h:2-60 semantics: barrier, run, MAX over ranks), the
// per-step kernel time of each rank's batched compute (HIP events; MAX over
// ranks of the per-run total), and, for all-reduce, a known-answer check
// that is exact in any float type: sendbuf[i] = (i mod 1021) - 510 on every
// rank, so every partial sum is a small integer and recvbuf[i] must equal
// numproc * sendbuf[i] whatever the summation order.
static int bench_json(const char *path, HiCCL::Comm<Type> &coll, Type *sendbuf_d, Type *recvbuf_d, size_t count,
                      int pattern, int warmup, int numiter, const std::vector<int> &hierarchy,
                      const std::vector<CommBench::library> &libs, int pipedepth) {
  const int myid = CommBench::myid, numproc = CommBench::numproc;
  const size_t n = count * numproc;
  std::vector<Type> host(n);
  // built as a signed integer, then converted: a negative double converted
  // to the unsigned driver type (size_t) would be undefined behaviour, the
  // int64_t -> size_t conversion wraps (and the expected sums wrap alike)
  for (size_t i = 0; i < n; i++) host[i] = (Type)kat_value(i, 1);
  CommBench::memcpyH2D(sendbuf_d, host.data(), n);
  double kern_ms = 0, kern_bytes = 0;
  int ksteps = 0;
#ifndef HICCL_PORT_HOST
  for (auto &kt : coll.compute_kernel_times(5)) {
    kern_ms += kt.first;
    kern_bytes += (double)kt.second;
    ksteps++;
  }
#endif
  double kmax[2] = {kern_ms, kern_bytes};
  MPI_Allreduce(MPI_IN_PLACE, kmax, 2, MPI_DOUBLE, MPI_MAX, CommBench::comm_mpi);
  HiCCL::Times t = HiCCL::measure<Type>(warmup, numiter, n, coll);
  // known-answer check on the same inputs (the measure runs left recvbuf
  // holding the all-reduce of sendbuf)
  {
    std::vector<Type> fill(n);
    std::memset((void *)fill.data(), 0xff, n * sizeof(Type));
    CommBench::memcpyH2D(recvbuf_d, fill.data(), n);
  }
  MPI_Barrier(CommBench::comm_mpi);
  coll.run();
  std::vector<Type> out(n);
  CommBench::memcpyD2H(out.data(), recvbuf_d, n);
  size_t bad = 0;
  if (pattern == HiCCL::allreduce)
    for (size_t i = 0; i < n; i++)
      if (out[i] != (Type)kat_value(i, numproc)) bad++;
  unsigned long tot = bad;
  MPI_Allreduce(MPI_IN_PLACE, &tot, 1, MPI_UNSIGNED_LONG, MPI_SUM, CommBench::comm_mpi);
  // where each step's host time goes (Comm::set_step_timing: transport
  // start / wait, compute launch / wait in comm.h:195-204's order, or the
  // stream-ordered enqueue and final sync), microseconds per step, MAX over
  // ranks of each part
  // (HICCL_HOST_SPLIT_RUNS extra runs, default 1, 0: none -- never numiter
  // more full collectives inside a bench leg's time budget).  Rank 0's value
  // for every rank: each run is a barrier plus a full collective, so ranks
  // reading different values (a per-rank environment) would deadlock.
  int split_runs = 1;
  if (const char *e = std::getenv("HICCL_HOST_SPLIT_RUNS")) split_runs = std::max(0, std::atoi(e));
  MPI_Bcast(&split_runs, 1, MPI_INT, 0, CommBench::comm_mpi);
  coll.set_step_timing(true);
  for (int r = 0; r < split_runs; r++) {
    MPI_Barrier(CommBench::comm_mpi);
    coll.run();
  }
  const auto sp = coll.step_split();
  coll.set_step_timing(false);
  const double per = sp.runs && sp.steps ? 1e6 / ((double)sp.runs * (double)sp.steps) : 0.0;
  double split[7] = {sp.transport_start * per, sp.transport_wait * per, sp.compute_launch * per,
                     sp.compute_wait * per, sp.finish * per, sp.enqueue * per, sp.sync * per};
  MPI_Allreduce(MPI_IN_PLACE, split, 7, MPI_DOUBLE, MPI_MAX, CommBench::comm_mpi);
  // where the ranks ran: every rank's visible device count, its device and
  // that device's PCI bus id (a per-rank device mask that hid the other GPUs
  // shows as devices_seen 1 and repeated bus ids)
  char where[64];
  std::memset(where, 0, sizeof(where));
#ifndef HICCL_PORT_HOST
  {
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    char bus[32] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, CommBench::mydevice) != hipSuccess) std::strcpy(bus, "?");
    std::snprintf(where, sizeof(where), "%d|%d|%s", ndev, CommBench::mydevice, bus);
  }
#else
  std::snprintf(where, sizeof(where), "0|-1|host");
#endif
  std::vector<char> wall((size_t)numproc * sizeof(where));
  MPI_Gather(where, sizeof(where), MPI_CHAR, wall.data(), sizeof(where), MPI_CHAR, 0, CommBench::comm_mpi);
  if (myid == 0) {
    std::string seen, devs, buses;
    for (int r = 0; r < numproc; r++) {
      std::string w(wall.data() + (size_t)r * sizeof(where));
      const size_t a = w.find('|'), b = w.find('|', a + 1);
      seen += (r ? "," : "") + w.substr(0, a);
      devs += (r ? "," : "") + w.substr(a + 1, b - a - 1);
      buses += std::string(r ? ", " : "") + "\"" + w.substr(b + 1) + "\"";
    }
    std::string mode_used = coll.stream_ordered() ? "stream-ordered" : "host-driven";
    if (coll.graph_mode()) mode_used += "+graph";
    if (coll.fused_gather()) mode_used += "+fused";
#ifndef HICCL_PORT_HOST
    if (coll.xccl_on_rccl()) mode_used += "+xccl-rccl";
    if (coll.step_program_mode()) mode_used += "+program";
    if (coll.stream_ordered()) mode_used += hiccl_token_mode() == HICCL_TOKENS_LIGHT ? "+tokens-light" : "+tokens-fenced";
    if (coll.shares_device()) mode_used += " (ranks share a GPU)";
#endif
    std::string h, l;
    for (size_t i = 0; i < hierarchy.size(); i++) h += (i ? "," : "") + std::to_string(hierarchy[i]);
    for (size_t i = 0; i < libs.size(); i++) l += std::string(i ? "," : "") + CommBench::lib_name(libs[i]);
    FILE *f = std::fopen(path, "w");
    if (!f) CommBench::die("HICCL_DRIVER_JSON", path);
    const double data = (double)n * sizeof(Type);
    std::fprintf(f,
                 "{\"ranks\": %d, \"pattern\": %d, \"hierarchy\": \"%s\", \"libs\": \"%s\", \"pipedepth\": %d, "
                 "\"count_per_rank_chunk\": %zu, \"sendbuf_bytes_per_rank\": %.0f, \"mode\": \"%s%s%s\", "
                 "\"iterations\": %zu, \"collective_ms_min\": %.4f, \"collective_ms_median\": %.4f, "
                 "\"collective_ms_max\": %.4f, \"algorithmic_GBps_median\": %.2f, "
                 "\"kernel_steps_rank0\": %d, \"kernel_ms_per_run_max_rank\": %.4f, "
                 "\"kernel_us_per_step_rank0\": %.3f, \"kernel_GBps_max_rank\": %.1f, "
                 "\"kat_exact_mismatches\": %lu, \"kat\": \"%s\", \"devices_seen\": [%s], \"rank_devices\": [%s], "
                 "\"bus_ids\": [%s], \"mode_used\": \"%s\", \"host_split_us_per_step\": {\"transport_start\": %.3f, "
                 "\"transport_wait\": %.3f, \"compute_launch\": %.3f, \"compute_wait\": %.3f, \"finish\": %.3f, "
                 "\"enqueue\": %.3f, \"sync\": %.3f, \"steps\": %zu, \"runs\": %zu, \"over_ranks\": \"max\"}}\n",
                 numproc, pattern, h.c_str(), l.c_str(), pipedepth, count, data, coll.stream_ordered() ? "stream-ordered" : "host-driven",
                 coll.graph_mode() ? "+graph" : "", coll.fused_gather() ? "+fused" : "", t.t.size(), t.min() * 1e3,
                 t.median() * 1e3, t.max() * 1e3, t.median() > 0 ? data / t.median() / 1e9 : 0.0, ksteps, kmax[0],
                 ksteps ? kern_ms / ksteps * 1e3 : 0.0, kmax[0] > 0 ? kmax[1] / (kmax[0] * 1e-3) / 1e9 : 0.0, tot,
                 pattern != HiCCL::allreduce ? "n/a" : tot == 0 ? "PASSED" : "FAILED", seen.c_str(), devs.c_str(),
                 buses.c_str(), mode_used.c_str(), split[0], split[1], split[2], split[3], split[4], split[5], split[6],
                 sp.steps, sp.runs);
    std::fclose(f);
  }
  return tot == 0 ? 0 : 1;
}

int main(int argc, char *argv[]) {
  CommBench::init();
  const int myid = CommBench::myid, numproc = CommBench::numproc;
  if (argc < 8) {
    if (myid == 0)
      std::fprintf(stderr, "usage: %s pattern count numstripe ringnodes pipedepth warmup numiter [hierarchy libs] [dump]\n",
                   argv[0]);
    MPI_Finalize();
    return 2;
  }
  const int pattern = std::atoi(argv[1]);
  const size_t count = std::atol(argv[2]);
  const int numstripe = std::atoi(argv[3]), ringnodes = std::atoi(argv[4]), pipedepth = std::atoi(argv[5]);
  const int warmup = std::atoi(argv[6]), numiter = std::atoi(argv[7]);
  std::vector<int> hierarchy = {numproc};
  std::vector<CommBench::library> libs = {CommBench::MPI};
  if (argc > 9) {
    hierarchy = parse_ints(argv[8]);
    libs = parse_libs(argv[9]);
  }
  const char *dump = argc > 10 ? argv[10] : nullptr;
  const int root = 0;

  if (myid == 0) {
    std::printf("\nNumber of processes: %d\nPattern: %d  count %zu (", numproc, pattern, count);
    CommBench::print_data(count * sizeof(Type));
    std::printf(")  numstripe %d ringnodes %d pipedepth %d\n", numstripe, ringnodes, pipedepth);
  }

  Type *sendbuf_d = nullptr, *recvbuf_d = nullptr;
  CommBench::allocate(sendbuf_d, count * numproc);
  CommBench::allocate(recvbuf_d, count * numproc);

  int rc = 0;
  {
    HiCCL::Comm<Type> coll;
    hiccl_driver::CommSink<Type> sink{coll};
    if (!hiccl_driver::compose(sink, pattern, sendbuf_d, recvbuf_d, count, numproc, root)) {
      if (myid == 0) std::printf("invalid collective option\n");
      MPI_Finalize();
      return 2;
    }
    coll.set_hierarchy(hierarchy, libs);
    coll.set_numstripe(numstripe);
    coll.set_ringnodes(ringnodes);
    coll.set_pipedepth(pipedepth);
    coll.init();
    coll.report();

    if (dump) {  // exact-bits run on float inputs from the counter hash
      std::vector<Type> in(count * numproc);
      for (size_t i = 0; i < in.size(); i++) in[i] = (Type)uniform_f32(1234, (uint32_t)myid, i);
      CommBench::memcpyH2D(sendbuf_d, in.data(), in.size());
      std::vector<Type> nanfill(count * numproc, (Type)-1);
      // HICCL_DRIVER_REPEAT=k: k runs, the receive buffer refilled before
      // each (graph mode: eager, capture + replay, replays), last one dumped
      const char *rep = std::getenv("HICCL_DRIVER_REPEAT");
      const int repeat = rep && std::atoi(rep) > 1 ? std::atoi(rep) : 1;
      for (int r = 0; r < repeat; r++) {
        CommBench::memcpyH2D(recvbuf_d, nanfill.data(), nanfill.size());
        MPI_Barrier(CommBench::comm_mpi);
        coll.run();
      }
      std::vector<Type> out(count * numproc);
      CommBench::memcpyD2H(out.data(), recvbuf_d, out.size());
      std::string path = std::string(dump) + ".rank" + std::to_string(myid) + ".bin";
      FILE *f = std::fopen(path.c_str(), "wb");
      if (!f || std::fwrite(out.data(), sizeof(Type), out.size(), f) != out.size()) CommBench::die("dump", path);
      std::fclose(f);
    }
    const char *json = std::getenv("HICCL_DRIVER_JSON");
    if (json && numiter > 0) {
      // bench.py's config-5 leg: whole-collective times, per-step kernel
      // times, and a float-exact known-answer check, as one JSON object
      rc = bench_json(json, coll, sendbuf_d, recvbuf_d, count, pattern, warmup, numiter, hierarchy, libs, pipedepth);
    } else {
      if (numiter > 0) {
        coll.measure(warmup, numiter, count * numproc / pipedepth);
        HiCCL::measure<Type>(warmup, numiter, count * numproc, coll);
      }
      if (!dump || sizeof(Type) == 8) rc = HiCCL::validate(sendbuf_d, recvbuf_d, count, pattern, root, coll) ? 0 : 1;
    }
  }
  CommBench::free(sendbuf_d);
  CommBench::free(recvbuf_d);
  MPI_Finalize();
  return rc;
}
