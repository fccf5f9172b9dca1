// include/hiccl/compute.h -- HiCCL::Compute<T>, the reduction compute stage.
//
// Same object contract as the reference (source/compute.h:26-204): add()
// registers one compute on its owning rank (SPMD filter, compute.h:66),
// start() launches every registered compute, wait() blocks until they are
// done, report()/measure() print the reference's tables.  The MI355X port
// keeps all registered computes in ONE hiccl_reduce_plan and start() is a
// single batched kernel launch on the process's compute stream (the
// reference launches one reduce_kernel per compute on a stream of its own,
// compute.h:87-106, and synchronises each, compute.h:107-117).
//
// Host port (HICCL_PORT_HOST, no GPU: config 1) runs the same in-order sum
// with OpenMP on host memory, like the reference's no-PORT build
// (compute.h:14-23).  It is selected at compile time; a HIP build contains no
// CPU reduction.
#ifndef HICCL_COMPUTE_H
#define HICCL_COMPUTE_H

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "transport.h"

#ifndef HICCL_PORT_HOST
#include "../hiccl_reduce.h"
#endif

namespace HiCCL {

// bfloat16 storage type for Comm<bf16> / Compute<bf16>.  The arithmetic is
// the reference's `T acc = 0; acc += x` (compute.h:7-9) with T = bf16: an
// f32 add rounded to nearest-even bf16 after every add -- the host port
// below and the GPU kernels (HICCL_BFLOAT16, HICCL_ACC_NATIVE) give the same
// bits.  Only this type maps to HICCL_BFLOAT16: other 2-byte types
// (int16_t, uint16_t) have no reduction here and fail to compile.
struct bf16 {
  uint16_t bits = 0;
  bf16() = default;
  bf16(int v) : bits(round((float)v)) {}  // T acc = 0
  explicit bf16(float f) : bits(round(f)) {}
  explicit operator float() const {
    uint32_t w = (uint32_t)bits << 16;
    float f;
    std::memcpy(&f, &w, 4);
    return f;
  }
  bf16 &operator+=(bf16 o) {
    bits = round((float)*this + (float)o);
    return *this;
  }
  bool operator==(bf16 o) const { return bits == o.bits; }
  bool operator!=(bf16 o) const { return bits != o.bits; }
  static uint16_t round(float f) {  // round to nearest even; NaN stays NaN
    uint32_t w;
    std::memcpy(&w, &f, 4);
    if ((w & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((w >> 16) | 0x40);
    w += 0x7fffu + ((w >> 16) & 1u);
    return (uint16_t)(w >> 16);
  }
};
static_assert(sizeof(bf16) == 2, "bf16 storage");

// T -> hiccl_dtype_t
template <typename T>
constexpr int dtype_of() {
  if constexpr (std::is_same<T, float>::value) return 0;
  else if constexpr (std::is_same<T, double>::value) return 1;
  else if constexpr (std::is_integral<T>::value && sizeof(T) == 8) return 3;
  else if constexpr (std::is_integral<T>::value && sizeof(T) == 4) return 4;
  else if constexpr (std::is_same<T, bf16>::value) return 2;
  else return -1;
}

#ifndef HICCL_PORT_HOST
// One compute stream per process (see transport_stream()).
inline hipStream_t compute_stream() {
  static hipStream_t s = [] {
    hipStream_t t;
    CommBench::hip_check(hipStreamCreateWithFlags(&t, hipStreamNonBlocking), "hipStreamCreate(compute)");
    return t;
  }();
  return s;
}
#endif

template <typename T>
class Compute {
 public:
  int numcomp = 0;
  std::vector<std::vector<T *>> inputbuf;
  std::vector<T *> outputbuf;
  std::vector<size_t> count;

  Compute() {}
  ~Compute() {
#ifndef HICCL_PORT_HOST
    if (plan) hiccl_reduce_plan_destroy(plan);
#endif
  }
  Compute(const Compute &) = delete;
  Compute &operator=(const Compute &) = delete;

  // compute.h:47-85.  Every rank calls add; the owning rank records.
  // `peer_inputs`: some input is a peer GPU's buffer read in place (fused
  // gather): the step's kernel then loads with system scope
  // (hiccl_reduce_plan_set_peer).
  void add(std::vector<T *> &in, T *out, size_t n, int compid, bool peer_inputs = false) {
    if (CommBench::myid != compid) return;
    inputbuf.push_back(in);
    outputbuf.push_back(out);
    count.push_back(n);
    numcomp++;
#ifndef HICCL_PORT_HOST
    static_assert(dtype_of<T>() >= 0, "HiCCL::Compute: unsupported element type");
    if (!plan) {
      check(hiccl_reduce_plan_create(&plan, dtype_of<T>(), CommBench::mydevice), "plan_create");
      // HICCL_ENGINE=tile|phase|auto pins the kernel engine (same bits either
      // way, so ranks need not agree); default auto.
      if (const char *e = std::getenv("HICCL_ENGINE")) {
        const std::string v(e);
        const int eng = v == "tile" ? HICCL_ENGINE_TILE : v == "phase" ? HICCL_ENGINE_PHASE : HICCL_ENGINE_AUTO;
        check(hiccl_reduce_plan_set_engine(plan, eng), "plan_set_engine");
      }
    }
    if (peer_inputs && !(hiccl_reduce_plan_peer(plan) & HICCL_PEER_LOADS))
      check(hiccl_reduce_plan_set_peer(plan, hiccl_reduce_plan_peer(plan) | HICCL_PEER_LOADS), "plan_set_peer");
    check(hiccl_reduce_plan_add(plan, out, (const void *const *)in.data(), (int)in.size(), n), "plan_add");
#else
    (void)peer_inputs;
#endif
  }

  // compute.h:87-106: nonblocking launch of all registered computes.
  void start() {
    if (!numcomp) return;
#ifndef HICCL_PORT_HOST
    check(hiccl_reduce_plan_launch(plan, compute_stream()), "plan_launch");
#else
    for (int c = 0; c < numcomp; c++) host_sum(outputbuf[c], count[c], inputbuf[c]);
#endif
  }

#ifndef HICCL_PORT_HOST
  // Stream-ordered execution: enqueue the step's batched kernel on `s`.
  void launch(hipStream_t s) {
    if (!numcomp) return;
    CommBench::flush_signals();  // queued signal/wait steps precede this kernel on the stream
    if (CommBench::step_recorder()) return CommBench::record_plan(plan, 2, this);  // a step program's element
    check(hiccl_reduce_plan_enqueue(plan, s), "plan_enqueue");  // the caller syncs the stream
  }
#endif

  // Algorithmic bytes of one start(): sum of count * (n + 1) * sizeof(T)
  // (the compute.h:197-203 accounting).
  size_t bytes() const {
    size_t b = 0;
    for (int c = 0; c < numcomp; c++) b += count[c] * (inputbuf[c].size() + 1) * sizeof(T);
    return b;
  }

  // compute.h:107-117
  void wait() {
#ifndef HICCL_PORT_HOST
    if (numcomp) check(hiccl_reduce_plan_sync(plan), "plan_sync");
#endif
  }

  // compute.h:119-135
  void report() {
    std::vector<int> nc(CommBench::numproc), ni(CommBench::numproc);
    int numinput = 0;
    for (auto &v : inputbuf) numinput += (int)v.size();
    MPI_Allgather(&numcomp, 1, MPI_INT, nc.data(), 1, MPI_INT, CommBench::comm_mpi);
    MPI_Allgather(&numinput, 1, MPI_INT, ni.data(), 1, MPI_INT, CommBench::comm_mpi);
    if (CommBench::myid == CommBench::printid) {
      std::printf("numcomp: ");
      for (int p = 0; p < CommBench::numproc; p++) std::printf("%d(%d) ", nc[p], ni[p]);
      std::printf("\n\n");
    }
  }

  // compute.h:137-196: time start()+wait() with barriers, MAX over ranks,
  // price `count` elements (the caller's choice, as the reference does).
  void measure(int warmup, int numiter, size_t cnt) {
    report();
    unsigned long busiest = 0;  // algorithmic bytes (n reads + 1 write) of the busiest rank
    for (int c = 0; c < numcomp; c++) busiest += (unsigned long)(count[c] * (inputbuf[c].size() + 1) * sizeof(T));
    MPI_Allreduce(MPI_IN_PLACE, &busiest, 1, MPI_UNSIGNED_LONG, MPI_MAX, CommBench::comm_mpi);
    roofline_bytes = (double)busiest;
    std::vector<double> times;
    if (CommBench::myid == CommBench::printid) {
      std::printf("Measure Reduction Kernel\n%d warmup iterations (in order)\n", warmup);
    }
    for (int it = -warmup; it < numiter; it++) {
#ifndef HICCL_PORT_HOST
      CommBench::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
#endif
      MPI_Barrier(CommBench::comm_mpi);
      double t0 = MPI_Wtime();
      start();
      double st = MPI_Wtime() - t0;
      wait();
      double t = MPI_Wtime() - t0;
      MPI_Allreduce(MPI_IN_PLACE, &st, 1, MPI_DOUBLE, MPI_MAX, CommBench::comm_mpi);
      MPI_Allreduce(MPI_IN_PLACE, &t, 1, MPI_DOUBLE, MPI_MAX, CommBench::comm_mpi);
      if (it < 0) {
        if (CommBench::myid == CommBench::printid) std::printf("startup %.2e warmup: %e\n", st, t);
      } else {
        times.push_back(t);
      }
    }
    print_times(times, (double)cnt * sizeof(T));
    roofline_bytes = 0;
  }

  // compute.h:197-203: price reads + writes, sum over ranks.  Also prints
  // the per-GPU HBM roofline fraction: the busiest rank's algorithmic bytes
  // over the median time against the 8 TB/s MI355X peak.
  void measure(int warmup, int numiter) {
    size_t tot = 0;
    for (int c = 0; c < numcomp; c++) tot += count[c] * (inputbuf[c].size() + 1);
    MPI_Allreduce(MPI_IN_PLACE, &tot, 1, MPI_UNSIGNED_LONG, MPI_SUM, CommBench::comm_mpi);
    measure(warmup, numiter, tot);
  }

  static constexpr double hbm_peak = 8.0e12;  // MI355X HBM3E, bytes/s

  static void print_times(std::vector<double> &times, double data) {
    if (times.empty() || CommBench::myid != CommBench::printid) return;
    std::sort(times.begin(), times.end());
    const int n = (int)times.size();
    std::printf("%d measurement iterations (sorted):\n", n);
    for (int i = 0; i < n; i++)
      std::printf("time: %.4e%s\n", times[i], i == 0 ? " -> min" : i == n / 2 ? " -> median" : i == n - 1 ? " -> max" : "");
    double avg = 0;
    for (double t : times) avg += t;
    avg /= n;
    std::printf("\ndata: ");
    CommBench::print_data((size_t)data);
    std::printf("\n");
    const double v[4] = {times[0], times[n / 2], times[n - 1], avg};
    const char *name[4] = {"min", "med", "max", "avg"};
    for (int i = 0; i < 4; i++)
      std::printf("%sTime: %.4e us, %.4e ms/GB, %.4e GB/s\n", name[i], v[i] * 1e6, v[i] / data * 1e12, data / v[i] / 1e9);
#ifndef HICCL_PORT_HOST
    if (roofline_bytes > 0)
      std::printf("HBM roofline (busiest rank, median): %.1f GB/s = %.1f %% of %.0f GB/s\n",
                  roofline_bytes / v[1] / 1e9, 100.0 * roofline_bytes / v[1] / hbm_peak, hbm_peak / 1e9);
#endif
    std::printf("\n");
  }

  static inline double roofline_bytes = 0;  // set by measure(warmup, numiter)

 private:
#ifndef HICCL_PORT_HOST
  hiccl_reduce_plan_t *plan = nullptr;
  static void check(int e, const char *what) {
    if (e) CommBench::die(what, hiccl_last_error());
  }
#else
  static void host_sum(T *out, size_t n, const std::vector<T *> &in) {
    const int k = (int)in.size();
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; i++) {
      T acc = 0;
      for (int j = 0; j < k; j++) acc += in[j][i];
      out[i] = acc;
    }
  }
#endif
};

}  // namespace HiCCL

#endif  // HICCL_COMPUTE_H
