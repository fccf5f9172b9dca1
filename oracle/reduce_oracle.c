/*
 * oracle/reduce_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of HiCCL's local bucket-reduction compute stage.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline.  The
 * product path (hiccl_amd/, include/) never links or calls it.
 *
 * What it restates (reference @ 2024-12-20, /root/reference):
 *   source/compute.h:14-23   CPU reduce_kernel<T>:
 *                              #pragma omp parallel for over i;
 *                              T acc = 0; for in: acc += input[in][i];
 *                              output[i] = acc;
 *   source/compute.h:2-12    GPU reduce_kernel<T>: same arithmetic, one
 *                              element per thread.
 * The summation order is exactly the order of the input list (which
 * source/reduce.h:134-169 fixes as ascending rank order), the accumulator
 * starts at +0 in type T, and every add is rounded to T.  Consequences the
 * GPU kernel must reproduce bit for bit:
 *   - all-(-0) inputs give +0 (0x00000000), also for n == 1;
 *   - n == 0 writes +0;
 *   - bf16 (not instantiated by the reference, whose T is float/size_t):
 *     acc is bf16, each add is float(acc)+float(x) rounded to float, then
 *     rounded to bf16 (round-to-nearest-even, NaN kept NaN) -- the
 *     semantics of `bf16 acc; acc += x` with a float-promoting bf16 type.
 *
 * Parity of this restatement is pinned against the reference's own
 * reduce_kernel compiled from /root/reference/source/compute.h
 * (oracle/build_ref.sh -> oracle/_ref/libhiccl_ref.so) by
 * tests/golden/make_golden.py, which also writes the committed fixtures.
 *
 * Synthetic inputs: element i of input k is a
 * uniform value in [-1, 1) from a counter-based hash of (seed, k, i), so
 * the GPU fill kernel, this oracle and the fixtures agree without
 * transferring data.
 */
#define _GNU_SOURCE /* sched_getcpu: oracle_thread_cpus */
#include <sched.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <math.h>

/* ---------------------------------------------------------------- sums -- */

/* compute.h:14-23, T = float */
void oracle_reduce_f32(float *out, const float *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    float acc = 0.0f;
    for (int k = 0; k < n; k++)
      acc += in[k][i];
    out[i] = acc;
  }
}

/* compute.h:14-23, T = double */
void oracle_reduce_f64(double *out, const double *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    double acc = 0.0;
    for (int k = 0; k < n; k++)
      acc += in[k][i];
    out[i] = acc;
  }
}

/* compute.h:14-23, T = size_t (the type collectives/main.cpp:24 uses) */
void oracle_reduce_u64(uint64_t *out, const uint64_t *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    uint64_t acc = 0;
    for (int k = 0; k < n; k++)
      acc += in[k][i];
    out[i] = acc;
  }
}

/* compute.h:14-23, T = int (wrap-around done in unsigned to stay defined) */
void oracle_reduce_i32(int32_t *out, const int32_t *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    uint32_t acc = 0;
    for (int k = 0; k < n; k++)
      acc += (uint32_t)in[k][i];
    out[i] = (int32_t)acc;
  }
}

static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

/* float -> bf16, round to nearest even; a NaN stays a NaN (quiet bit set). */
static inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu))
    return (uint16_t)((u >> 16) | 0x0040u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

/* compute.h:14-23 with T = bf16 (acc rounded to bf16 after every add). */
void oracle_reduce_bf16(uint16_t *out, const uint16_t *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    uint16_t acc = 0;
    for (int k = 0; k < n; k++) {
      float s = bf16_to_f32(acc) + bf16_to_f32(in[k][i]);
      acc = f32_to_bf16(s);
    }
    out[i] = acc;
  }
}

/* bf16 inputs, f32 accumulator, one rounding at the end (the optional
 * "accumulate wide" mode of the build; NOT the reference semantics). */
void oracle_reduce_bf16_accf32(uint16_t *out, const uint16_t *const *in, int n, size_t count) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++) {
    float acc = 0.0f;
    for (int k = 0; k < n; k++)
      acc += bf16_to_f32(in[k][i]);
    out[i] = f32_to_bf16(acc);
  }
}

/* ------------------------------------------------------ synthetic data -- */

static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* hash of (seed, k, i) -> 64 random bits */
static inline uint64_t hash3(uint64_t seed, uint32_t k, uint64_t i) {
  return splitmix64(splitmix64(seed ^ ((uint64_t)k << 48)) + i);
}

/* uniform [-1, 1) on a 2^-23 grid: exact in f32 on every platform. */
static inline float uniform_f32(uint64_t h) {
  return (float)(uint32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;
}

void oracle_fill_uniform_f32(float *out, size_t count, uint64_t seed, uint32_t k, size_t first) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++)
    out[i] = uniform_f32(hash3(seed, k, first + i));
}

void oracle_fill_uniform_bf16(uint16_t *out, size_t count, uint64_t seed, uint32_t k, size_t first) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++)
    out[i] = f32_to_bf16(uniform_f32(hash3(seed, k, first + i)));
}

void oracle_fill_uniform_f64(double *out, size_t count, uint64_t seed, uint32_t k, size_t first) {
  #pragma omp parallel for schedule(static)
  for (size_t i = 0; i < count; i++)
    out[i] = (double)uniform_f32(hash3(seed, k, first + i));
}

/* Sum of the synthetic inputs at an arbitrary list of element indices:
 * the size-independent check for full-size (1 GiB/input) GPU outputs. */
void oracle_sample_sum_f32(float *out, const uint64_t *idx, size_t nidx, uint64_t seed, int n) {
  #pragma omp parallel for schedule(static)
  for (size_t j = 0; j < nidx; j++) {
    float acc = 0.0f;
    for (int k = 0; k < n; k++)
      acc += uniform_f32(hash3(seed, (uint32_t)k, idx[j]));
    out[j] = acc;
  }
}

void oracle_sample_sum_bf16(uint16_t *out, const uint64_t *idx, size_t nidx, uint64_t seed, int n) {
  #pragma omp parallel for schedule(static)
  for (size_t j = 0; j < nidx; j++) {
    uint16_t acc = 0;
    for (int k = 0; k < n; k++) {
      uint16_t x = f32_to_bf16(uniform_f32(hash3(seed, (uint32_t)k, idx[j])));
      float s = bf16_to_f32(acc) + bf16_to_f32(x);
      acc = f32_to_bf16(s);
    }
    out[j] = acc;
  }
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* The CPU each thread of an OpenMP team runs on (out[t] for thread t < n,
 * -1 where unknown): where bench.py's CPU baseline leg put the threads
 * whose static blocks it then checks for NUMA locality.  Returns the team
 * size. */
int oracle_thread_cpus(int *out, int n) {
  int team = 1;
  for (int t = 0; t < n; t++) out[t] = -1;
#ifdef _OPENMP
  extern int omp_get_thread_num(void);
  extern int omp_get_num_threads(void);
  #pragma omp parallel
  {
    const int t = omp_get_thread_num();
    if (t < n) out[t] = sched_getcpu();
    if (t == 0) team = omp_get_num_threads();
  }
#else
  out[0] = sched_getcpu();
#endif
  return team;
}
