// tools/phase_probe.hip -- bench-only probes (not part of the product).
//
// Question: the 8-read + 1-write reduction runs at 5.5-5.65 TB/s or at
// 6.1-6.3 TB/s depending on the physical placement of the nine 1 GiB
// buckets (profiles/r01_placement.txt).  A placement effect of that kind is
// what DRAM bank/row conflicts between streams look like: the product kernel
// keeps all nine streams open at the same element offset at the same time.
// These probes change WHICH streams are open at once:
//
//   k_phase<B,P>  input-phased: a workgroup owns a chunk of B*P packets; it
//                 sweeps input 0 of the chunk, then input 1, ... (register
//                 accumulators, next input's loads in flight while the
//                 current one is added), then stores the chunk.  Chip-wide
//                 only ~1-2 input streams are open at any moment.
//   k_slab<B,U>   the product's tile order, but each workgroup walks its
//                 own contiguous slab instead of grid-striding.
//
// Plus allocation modes for the placement itself (hipMalloc, contiguous
// hipExtMallocWithFlags, VMM physical handles mapped into one range).
//
// Sums are f32 in input order starting from +0: bit-identical to the
// reference's reduce_kernel (source/compute.h:2-12) whatever the order of
// the loop nest, since each element's additions are still in input order.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t mk(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)n, 0x00020000);
}

struct PArgs {
  const char *in[16];
  char *out;
  uint64_t bytes;  // per stream, multiple of 16
  int n;
};

template <int AUX>
__device__ __forceinline__ f32x4 ld(rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, AUX));
}

// Input-phased chunk sweep.
template <int B, int P, int AUXL, int AUXS>
__global__ __launch_bounds__(B) void k_phase(PArgs a) {
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t off = c * CH;
    const uint32_t nb = (uint32_t)((a.bytes - off) < CH ? (a.bytes - off) : CH);
    f32x4 acc[P], x[P], y[P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
    rsrc_t r = mk(a.in[0] + off, nb);
#pragma unroll
    for (int p = 0; p < P; p++) x[p] = ld<AUXL>(r, voff[p]);
    int j = 0;
    for (; j + 2 <= a.n; j += 2) {  // x holds input j (in flight)
      rsrc_t ry = mk(a.in[j + 1] + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++) y[p] = ld<AUXL>(ry, voff[p]);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[p];
      if (j + 2 < a.n) {
        rsrc_t rx = mk(a.in[j + 2] + off, nb);
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = ld<AUXL>(rx, voff[p]);
      }
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += y[p];
    }
    if (j < a.n) {
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[p];
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, AUXS);
  }
}

// Input-phased, N static, D input stages in flight: input j+D-1's loads are
// issued before input j's adds; sched_barriers keep the scheduler from
// hoisting later inputs.
template <int B, int P, int N, int D, int AUXL, int AUXS>
__global__ __launch_bounds__(B) void k_phase_n(PArgs a) {
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t off = c * CH;
    const uint32_t nb = (uint32_t)((a.bytes - off) < CH ? (a.bytes - off) : CH);
    f32x4 acc[P], x[D][P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
#pragma unroll
    for (int j = 0; j < D - 1 && j < N; j++) {
      rsrc_t r = mk(a.in[j] + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++) x[j % D][p] = ld<AUXL>(r, voff[p]);
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j + D - 1 < N) {
        rsrc_t r = mk(a.in[j + D - 1] + off, nb);
#pragma unroll
        for (int p = 0; p < P; p++) x[(j + D - 1) % D][p] = ld<AUXL>(r, voff[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[j % D][p];
      __builtin_amdgcn_sched_barrier(0);
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, AUXS);
  }
}

// Phased, N static (8), D = 2, with order/store variants:
//   MODE & 1: no store (read-only ceiling of the phased order)
//   MODE & 2: slab order (workgroup b owns chunks [b*per, (b+1)*per))
//   MODE & 4: staggered start (workgroup b sleeps (b % 9) x ~5 us first)
// AUXS: store cache-policy bits (gfx950: 1 sc0, 2 nt, 16 sc1).
template <int B, int P, int MODE, int AUXS = 2>
__global__ __launch_bounds__(B) void k_phase_x(PArgs a) {
  constexpr int N = 8;
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  uint64_t c0 = blockIdx.x, c1 = nch, cs = gridDim.x;
  if (MODE & 2) {
    const uint64_t per = (nch + gridDim.x - 1) / gridDim.x;
    c0 = blockIdx.x * per;
    c1 = c0 + per < nch ? c0 + per : nch;
    cs = 1;
  }
  f32x4 sink = (f32x4)(0.0f);
  if (MODE & 4) {
    for (uint32_t k = 0; k < (blockIdx.x % 9) * 2; k++) __builtin_amdgcn_s_sleep(127);
  }
  for (uint64_t c = c0; c < c1; c += cs) {
    const uint64_t off = c * CH;
    const uint32_t nb = (uint32_t)((a.bytes - off) < CH ? (a.bytes - off) : CH);
    f32x4 acc[P], x[2][P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
    {
      rsrc_t r = mk(a.in[0] + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++) x[0][p] = ld<2>(r, voff[p]);
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j + 1 < N) {
        rsrc_t r = mk(a.in[j + 1] + off, nb);
#pragma unroll
        for (int p = 0; p < P; p++) x[(j + 1) & 1][p] = ld<2>(r, voff[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[j & 1][p];
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE & 1) {
#pragma unroll
      for (int p = 0; p < P; p++) sink += acc[p];
    } else {
      rsrc_t w = mk(a.out + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, AUXS);
    }
  }
  if ((MODE & 1) && sink.x == 1.2345f && sink.y == 5.4321f) a.out[threadIdx.x] = 1;
}

// Phased with a 2-part chunk: part 0's accumulator in registers, part 1's in
// LDS (B*P*16 B); chunk = 2*B*P*16 B (256 KiB at 512 x 16).  Loads stream
// (j,0), (j,1), (j+1,0), ...: one part in flight while the other is added.
template <int B, int P>
__global__ __launch_bounds__(B) void k_phase_lds(PArgs a) {
  constexpr uint64_t PART = (uint64_t)B * P * 16;
  constexpr uint64_t CH = 2 * PART;
  __shared__ f32x4 lacc[P * B];
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t off0 = c * CH, off1 = off0 + PART;
    const uint64_t left0 = a.bytes - off0;
    const uint32_t nb0 = (uint32_t)(left0 < PART ? left0 : PART);
    const uint32_t nb1 = (uint32_t)(left0 <= PART ? 0 : (left0 - PART < PART ? left0 - PART : PART));
    f32x4 acc[P], x[P], y[P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
    {
      rsrc_t r0 = mk(a.in[0] + off0, nb0);
#pragma unroll
      for (int p = 0; p < P; p++) x[p] = ld<2>(r0, voff[p]);
      rsrc_t r1 = mk(a.in[0] + off1, nb1);
#pragma unroll
      for (int p = 0; p < P; p++) y[p] = ld<2>(r1, voff[p]);
    }
    for (int j = 0; j < a.n; j++) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[p];
      __builtin_amdgcn_sched_barrier(0);
      const bool more = j + 1 < a.n;
      {
        rsrc_t r0 = mk(a.in[more ? j + 1 : j] + off0, more ? nb0 : 0u);
#pragma unroll
        for (int p = 0; p < P; p++) x[p] = ld<2>(r0, voff[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j == 0) {
#pragma unroll
        for (int p = 0; p < P; p++) lacc[p * B + threadIdx.x] = (f32x4)(0.0f) + y[p];
      } else {
#pragma unroll
        for (int p = 0; p < P; p++) lacc[p * B + threadIdx.x] += y[p];
      }
      __builtin_amdgcn_sched_barrier(0);
      {
        rsrc_t r1 = mk(a.in[more ? j + 1 : j] + off1, more ? nb1 : 0u);
#pragma unroll
        for (int p = 0; p < P; p++) y[p] = ld<2>(r1, voff[p]);
      }
    }
    rsrc_t w0 = mk(a.out + off0, nb0), w1 = mk(a.out + off1, nb1);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w0, (int)voff[p], 0, 2);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lacc[p * B + threadIdx.x]), w1,
                                             (int)voff[p], 0, 2);
  }
}

// Phased, pipelined ACROSS chunks: the workgroup walks a flat sequence of
// units (chunk c, input j) with two register buffers; the load of unit k+2
// is issued right after unit k is added, so the next chunk's input 0 is in
// flight while the current chunk's last input is added and stored.
template <int B, int P>
__global__ __launch_bounds__(B) void k_phase_flat(PArgs a) {
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  if (blockIdx.x >= nch) return;
  const int n = a.n;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  // load cursor (unit to be loaded next)
  uint64_t lc = blockIdx.x;
  int lj = 0;
  auto chunk_bytes = [&](uint64_t c) -> uint32_t {
    const uint64_t left = a.bytes - c * CH;
    return (uint32_t)(left < CH ? left : CH);
  };
  auto issue = [&](f32x4 (&buf)[P]) {
    const bool valid = lc < nch;
    rsrc_t r = mk(a.in[valid ? lj : 0] + (valid ? lc * CH : 0), valid ? chunk_bytes(lc) : 0u);
#pragma unroll
    for (int p = 0; p < P; p++) buf[p] = ld<2>(r, voff[p]);
    if (++lj == n) { lj = 0; lc += gridDim.x; }
  };
  // add cursor
  uint64_t ac = blockIdx.x;
  int aj = 0;
  f32x4 acc[P], x[P], y[P];
#pragma unroll
  for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
  auto consume = [&](f32x4 (&buf)[P]) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] += buf[p];
    if (++aj == n) {
      rsrc_t w = mk(a.out + ac * CH, chunk_bytes(ac));
#pragma unroll
      for (int p = 0; p < P; p++) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, 2);
        acc[p] = (f32x4)(0.0f);
      }
      aj = 0;
      ac += gridDim.x;
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  issue(x);
  issue(y);
  while (ac < nch) {
    consume(x);
    issue(x);
    if (ac >= nch) break;
    consume(y);
    issue(y);
  }
}

// Phased, pipelined across chunks with static buffer roles.  pass<A,B>:
// A holds (chunk c, input 0) in flight on entry; on exit the buffer named by
// the return value holds (next chunk, input 0): B for odd n, A for even n.
// Odd n therefore runs chunk pairs (x,y) then (y,x); even n runs (x,y).
template <int P>
__device__ __forceinline__ void pp_load(f32x4 (&buf)[P], const char *base, uint32_t nb,
                                        const uint32_t (&voff)[P]) {
  rsrc_t r = mk(base, nb);
#pragma unroll
  for (int p = 0; p < P; p++) buf[p] = ld<2>(r, voff[p]);
}

template <int P>
__device__ __forceinline__ void pp_add(f32x4 (&acc)[P], const f32x4 (&buf)[P]) {
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int p = 0; p < P; p++) acc[p] += buf[p];
  __builtin_amdgcn_sched_barrier(0);
}

template <int P, bool ODD>
__device__ __forceinline__ void pp_pass(f32x4 (&A)[P], f32x4 (&B)[P], const PArgs &a, uint64_t off,
                                        uint32_t nb, uint64_t offn, uint32_t nbn,
                                        const uint32_t (&voff)[P]) {
  f32x4 acc[P];
#pragma unroll
  for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
  const int n = a.n;
  int j = 0;
  for (; j + 2 < n; j += 2) {
    pp_load(B, a.in[j + 1] + off, nb, voff);
    pp_add(acc, A);
    pp_load(A, a.in[j + 2] + off, nb, voff);
    pp_add(acc, B);
  }
  if constexpr (ODD) {
    pp_load(B, a.in[0] + offn, nbn, voff);
    pp_add(acc, A);
  } else {
    pp_load(B, a.in[n - 1] + off, nb, voff);
    pp_add(acc, A);
    pp_load(A, a.in[0] + offn, nbn, voff);
    pp_add(acc, B);
  }
  rsrc_t w = mk(a.out + off, nb);
#pragma unroll
  for (int p = 0; p < P; p++)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, 2);
}

template <int B, int P>
__global__ __launch_bounds__(B) void k_phase_pipe(PArgs a) {
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  auto nbytes = [&](uint64_t c) -> uint32_t {
    if (c >= nch) return 0u;
    const uint64_t left = a.bytes - c * CH;
    return (uint32_t)(left < CH ? left : CH);
  };
  auto offs = [&](uint64_t c) -> uint64_t { return c < nch ? c * CH : 0; };
  f32x4 x[P], y[P];
  uint64_t c = blockIdx.x;
  if (c >= nch) return;
  pp_load(x, a.in[0] + offs(c), nbytes(c), voff);
  const uint64_t g = gridDim.x;
  if (a.n & 1) {
    while (true) {
      pp_pass<P, true>(x, y, a, offs(c), nbytes(c), offs(c + g), nbytes(c + g), voff);
      c += g;
      if (c >= nch) break;
      pp_pass<P, true>(y, x, a, offs(c), nbytes(c), offs(c + g), nbytes(c + g), voff);
      c += g;
      if (c >= nch) break;
    }
  } else {
    for (; c < nch; c += g) pp_pass<P, false>(x, y, a, offs(c), nbytes(c), offs(c + g), nbytes(c + g), voff);
  }
}

// Phased (N = 8), with a soft grid barrier before each round's stores so the
// output writes of all workgroups land together (one write burst per round
// instead of a steady 1-in-9 write trickle).  Bounded spin (SPIN_TICKS of the
// 100 MHz s_memrealtime clock): never hangs even if the grid is not fully
// co-resident.  SYNC_EVERY: barrier every k rounds.
__device__ unsigned int g_round_counter[64];

template <int B, int P, int SYNC_EVERY>
__global__ __launch_bounds__(B) void k_phase_sync(PArgs a, unsigned int *counter) {
  constexpr int N = 8;
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  constexpr uint64_t SPIN_TICKS = 20000;  // 200 us
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  __shared__ int go;
  unsigned int round = 0;
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x, round++) {
    const uint64_t off = c * CH;
    const uint32_t nb = (uint32_t)((a.bytes - off) < CH ? (a.bytes - off) : CH);
    f32x4 acc[P], x[2][P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
    {
      rsrc_t r = mk(a.in[0] + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++) x[0][p] = ld<2>(r, voff[p]);
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j + 1 < N) {
        rsrc_t r = mk(a.in[j + 1] + off, nb);
#pragma unroll
        for (int p = 0; p < P; p++) x[(j + 1) & 1][p] = ld<2>(r, voff[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[j & 1][p];
      __builtin_amdgcn_sched_barrier(0);
    }
    if (round % SYNC_EVERY == 0) {
      if (threadIdx.x == 0) {
        // workgroups that own a chunk in this round
        const uint64_t first = (uint64_t)round * gridDim.x;
        const uint64_t active = (nch - first) < gridDim.x ? (nch - first) : gridDim.x;
        const unsigned int target = (unsigned int)(first + active);
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(8);
          if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS) break;
        }
        go = 1;
      }
      __syncthreads();
    } else {
      if (threadIdx.x == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, 2);
  }
  (void)go;
}

static unsigned int *sync_counter() {
  static unsigned int *p = nullptr;
  if (!p) (void)hipGetSymbolAddress((void **)&p, HIP_SYMBOL(g_round_counter));
  return p;
}

template <int SE>
static int launch_sync(int grid, const PArgs &a, hipStream_t s) {
  unsigned int *ctr = sync_counter();
  if (hipMemsetAsync(ctr, 0, 64 * sizeof(unsigned int), s)) return -5;
  hipLaunchKernelGGL((k_phase_sync<512, 16, SE>), dim3(grid), dim3(512), 0, s, a, ctr);
  return (int)hipGetLastError();
}

// Phased with split units: a chunk = Q units of B*U packets; the unit
// sequence (j,0), (j,1), ..., (j,Q-1), (j+1,0), ... is double-buffered, so
// the two units in flight are different inputs at offsets one unit apart
// (not the same offset), and the in-flight buffers are U (not Q*U) packets
// per lane: acc Q*U + 2*U packets.  Q even.
template <int B, int U, int Q>
__global__ __launch_bounds__(B) void k_phase_q(PArgs a) {
  static_assert(Q % 2 == 0, "Q even");
  constexpr uint64_t UB = (uint64_t)B * U * 16;
  constexpr uint64_t CH = UB * Q;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  const int n = a.n;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * B + threadIdx.x) * 16);
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t off = c * CH;
    uint32_t nb[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const uint64_t o = off + q * UB;
      nb[q] = o >= a.bytes ? 0u : (uint32_t)((a.bytes - o) < UB ? (a.bytes - o) : UB);
    }
    f32x4 acc[Q][U], x[U], y[U];
#pragma unroll
    for (int q = 0; q < Q; q++)
#pragma unroll
      for (int u = 0; u < U; u++) acc[q][u] = (f32x4)(0.0f);
    {
      rsrc_t r = mk(a.in[0] + off, nb[0]);
#pragma unroll
      for (int u = 0; u < U; u++) x[u] = ld<2>(r, voff[u]);
    }
    for (int j = 0; j < n; j++) {
      const bool more = j + 1 < n;
#pragma unroll
      for (int q = 0; q < Q; q += 2) {
        {  // y <- (j, q+1)
          rsrc_t r = mk(a.in[j] + off + (q + 1) * UB, nb[q + 1]);
#pragma unroll
          for (int u = 0; u < U; u++) y[u] = ld<2>(r, voff[u]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++) acc[q][u] += x[u];
        __builtin_amdgcn_sched_barrier(0);
        {  // x <- (j, q+2) or (j+1, 0) or nothing
          const bool last = q + 2 >= Q;
          const int jj = last ? (more ? j + 1 : j) : j;
          const uint64_t o = last ? off : off + (q + 2) * UB;
          const uint32_t m = last ? (more ? nb[0] : 0u) : nb[(q + 2) % Q];
          rsrc_t r = mk(a.in[jj] + o, m);
#pragma unroll
          for (int u = 0; u < U; u++) x[u] = ld<2>(r, voff[u]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; u++) acc[q + 1][u] += y[u];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int q = 0; q < Q; q++) {
      rsrc_t w = mk(a.out + off + q * UB, nb[q]);
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[q][u]), w, (int)voff[u], 0, 2);
    }
  }
}

// Phased (N = 8, D = 2) with DYNAMIC chunk assignment: each workgroup takes
// its next chunk from a device counter (zeroed per launch), so workgroups the
// memory system serves faster do more chunks and the kernel's tail is one
// chunk, not the slowest workgroup's share.  The next index is fetched one
// chunk ahead (the atomic's latency hides under the current chunk).
template <int B, int P>
__global__ __launch_bounds__(B) void k_phase_dyn(PArgs a, unsigned int *counter) {
  constexpr int N = 8;
  constexpr uint64_t CH = (uint64_t)B * P * 16;
  const uint64_t nch = (a.bytes + CH - 1) / CH;
  uint32_t voff[P];
#pragma unroll
  for (int p = 0; p < P; p++) voff[p] = (uint32_t)((p * B + threadIdx.x) * 16);
  __shared__ unsigned int next_c[2];
  if (threadIdx.x == 0) {
    next_c[0] = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  uint64_t c = next_c[0];
  int slot = 1;
  while (c < nch) {
    if (threadIdx.x == 0)
      next_c[slot] = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t off = c * CH;
    const uint32_t nb = (uint32_t)((a.bytes - off) < CH ? (a.bytes - off) : CH);
    f32x4 acc[P], x[2][P];
#pragma unroll
    for (int p = 0; p < P; p++) acc[p] = (f32x4)(0.0f);
    {
      rsrc_t r = mk(a.in[0] + off, nb);
#pragma unroll
      for (int p = 0; p < P; p++) x[0][p] = ld<2>(r, voff[p]);
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j + 1 < N) {
        rsrc_t r = mk(a.in[j + 1] + off, nb);
#pragma unroll
        for (int p = 0; p < P; p++) x[(j + 1) & 1][p] = ld<2>(r, voff[p]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] += x[j & 1][p];
      __builtin_amdgcn_sched_barrier(0);
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int p = 0; p < P; p++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[p]), w, (int)voff[p], 0, 2);
    __syncthreads();
    c = next_c[slot];
    slot ^= 1;
  }
}

template <int B, int P>
static int launch_dyn(int grid, const PArgs &a, hipStream_t s) {
  unsigned int *ctr = sync_counter();
  if (hipMemsetAsync(ctr, 0, sizeof(unsigned int), s)) return -5;
  hipLaunchKernelGGL((k_phase_dyn<B, P>), dim3(grid), dim3(B), 0, s, a, ctr);
  return (int)hipGetLastError();
}

// Per-WAVE dynamic tiles (N = 8): every wave takes its own unit of 64 lanes
// x U packets (U*1 KiB per input) from the ticket counter -- no workgroup
// barrier, and the chip-wide window is 4x narrower than per-workgroup 16 KiB
// tiles.  Next ticket grabbed before the current unit's loads.
template <int B, int U>
__global__ __launch_bounds__(B) void k_wave_dyn(PArgs a, unsigned int *counter) {
  constexpr int N = 8;
  constexpr uint64_t UB = 64ull * U * 16;  // bytes per input per unit
  const uint64_t nunits = (a.bytes + UB - 1) / UB;
  const int lane = threadIdx.x & 63;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * 64 + lane) * 16);
  uint32_t t;
  {
    uint32_t v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __builtin_amdgcn_readfirstlane(v);
  }
  while (t < nunits) {
    uint32_t nv;
    if (lane == 0) nv = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t off = (uint64_t)t * UB;
    const uint32_t nb = (uint32_t)((a.bytes - off) < UB ? (a.bytes - off) : UB);
    f32x4 x[N][U];
#pragma unroll
    for (int j = 0; j < N; j++) {
      rsrc_t r = mk(a.in[j] + off, nb);
#pragma unroll
      for (int u = 0; u < U; u++) x[j][u] = ld<2>(r, voff[u]);
    }
    f32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = (f32x4)(0.0f);
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] += x[j][u];
    t = __builtin_amdgcn_readfirstlane(nv);
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[u]), w, (int)voff[u], 0, 2);
  }
}

template <int B, int U>
static int launch_wave_dyn(int grid, const PArgs &a, hipStream_t s) {
  unsigned int *ctr = sync_counter();
  if (hipMemsetAsync(ctr, 0, sizeof(unsigned int), s)) return -5;
  hipLaunchKernelGGL((k_wave_dyn<B, U>), dim3(grid), dim3(B), 0, s, a, ctr);
  return (int)hipGetLastError();
}

// Per-workgroup dynamic 16 KiB tiles (the product's default) for comparison
template <int B, int U>
__global__ __launch_bounds__(B) void k_wg_dyn(PArgs a, unsigned int *counter) {
  constexpr int N = 8;
  constexpr uint64_t UB = (uint64_t)B * U * 16;
  const uint64_t nunits = (a.bytes + UB - 1) / UB;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * B + threadIdx.x) * 16);
  __shared__ uint32_t s_t[2];
  if (threadIdx.x == 0) s_t[0] = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  uint32_t t = s_t[0];
  int slot = 1;
  while (t < nunits) {
    uint32_t nv;
    if (threadIdx.x == 0) nv = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t off = (uint64_t)t * UB;
    const uint32_t nb = (uint32_t)((a.bytes - off) < UB ? (a.bytes - off) : UB);
    f32x4 x[N][U];
#pragma unroll
    for (int j = 0; j < N; j++) {
      rsrc_t r = mk(a.in[j] + off, nb);
#pragma unroll
      for (int u = 0; u < U; u++) x[j][u] = ld<2>(r, voff[u]);
    }
    f32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = (f32x4)(0.0f);
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] += x[j][u];
    if (threadIdx.x == 0) s_t[slot] = nv;
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[u]), w, (int)voff[u], 0, 2);
    __syncthreads();
    t = s_t[slot];
    slot ^= 1;
  }
}

template <int B, int U>
static int launch_wg_dyn(int grid, const PArgs &a, hipStream_t s) {
  unsigned int *ctr = sync_counter();
  if (hipMemsetAsync(ctr, 0, sizeof(unsigned int), s)) return -5;
  hipLaunchKernelGGL((k_wg_dyn<B, U>), dim3(grid), dim3(B), 0, s, a, ctr);
  return (int)hipGetLastError();
}

// Dynamic tiles with C counters (64 B apart): workgroup b (wave w for
// PER_WAVE) uses counter (b % C); its ticket k from that counter is unit
// k*C + (b % C).  Spreads the atomic traffic over C addresses.
template <int B, int U, int C, bool PER_WAVE>
__global__ __launch_bounds__(B) void k_multi_dyn(PArgs a, unsigned int *counter) {
  constexpr int N = 8;
  constexpr int LANES = PER_WAVE ? 64 : B;
  constexpr uint64_t UB = (uint64_t)LANES * U * 16;
  const uint64_t nunits = (a.bytes + UB - 1) / UB;
  const int lid = PER_WAVE ? (threadIdx.x & 63) : threadIdx.x;
  const uint32_t who = PER_WAVE ? (blockIdx.x * (B / 64) + threadIdx.x / 64) : blockIdx.x;
  const uint32_t cidx = who % C;
  unsigned int *ctr = counter + cidx * 16;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * LANES + lid) * 16);
  __shared__ uint32_t s_t[2];
  auto grab = [&]() -> uint32_t {
    return __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  uint64_t t;
  if (PER_WAVE) {
    uint32_t v = 0;
    if (lid == 0) v = grab();
    t = (uint64_t)__builtin_amdgcn_readfirstlane(v) * C + cidx;
  } else {
    if (threadIdx.x == 0) s_t[0] = grab();
    __syncthreads();
    t = (uint64_t)s_t[0] * C + cidx;
  }
  int slot = 1;
  while (t < nunits) {
    uint32_t nv;
    if (lid == 0) nv = grab();
    const uint64_t off = t * UB;
    const uint32_t nb = (uint32_t)((a.bytes - off) < UB ? (a.bytes - off) : UB);
    f32x4 x[N][U];
#pragma unroll
    for (int j = 0; j < N; j++) {
      rsrc_t r = mk(a.in[j] + off, nb);
#pragma unroll
      for (int u = 0; u < U; u++) x[j][u] = ld<2>(r, voff[u]);
    }
    f32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = (f32x4)(0.0f);
#pragma unroll
    for (int j = 0; j < N; j++)
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] += x[j][u];
    if (PER_WAVE) {
      t = (uint64_t)__builtin_amdgcn_readfirstlane(nv) * C + cidx;
    } else if (threadIdx.x == 0) {
      s_t[slot] = nv;
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[u]), w, (int)voff[u], 0, 2);
    if (!PER_WAVE) {
      __syncthreads();
      t = (uint64_t)s_t[slot] * C + cidx;
      slot ^= 1;
    }
  }
}

template <int B, int U, int C, bool PW>
static int launch_multi_dyn(int grid, const PArgs &a, hipStream_t s) {
  static_assert(C * 16 <= 64, "counters are 16 words apart; only 64 words are cleared");
  unsigned int *ctr = sync_counter();
  if (hipMemsetAsync(ctr, 0, 64 * sizeof(unsigned int), s)) return -5;
  hipLaunchKernelGGL((k_multi_dyn<B, U, C, PW>), dim3(grid), dim3(B), 0, s, a, ctr);
  return (int)hipGetLastError();
}

// Product tile order (all n inputs of a tile loaded together), slab-walked.
template <int B, int U, int AUXL, int AUXS>
__global__ __launch_bounds__(B) void k_slab(PArgs a) {
  constexpr uint64_t TILE = (uint64_t)B * U * 16;
  const uint64_t nt = (a.bytes + TILE - 1) / TILE;
  const uint64_t per = (nt + gridDim.x - 1) / gridDim.x;
  const uint64_t t0 = blockIdx.x * per, t1 = (t0 + per < nt) ? t0 + per : nt;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * B + threadIdx.x) * 16);
  for (uint64_t t = t0; t < t1; t++) {
    const uint64_t off = t * TILE;
    const uint32_t nb = (uint32_t)((a.bytes - off) < TILE ? (a.bytes - off) : TILE);
    f32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = (f32x4)(0.0f);
    for (int g = 0; g < a.n; g += 8) {
      f32x4 x[8][U];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        rsrc_t r = mk(a.in[g + j < a.n ? g + j : 0] + off, g + j < a.n ? nb : 0u);
#pragma unroll
        for (int u = 0; u < U; u++) x[j][u] = ld<AUXL>(r, voff[u]);
      }
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (g + j < a.n)
#pragma unroll
          for (int u = 0; u < U; u++) acc[u] += x[j][u];
    }
    rsrc_t w = mk(a.out + off, nb);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[u]), w, (int)voff[u], 0, AUXS);
  }
}

template <class K>
static int launch(K k, int grid, int block, const PArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" {

// kind 0: phase, kind 1: slab.  param = P (phase) or U (slab).
int pp_run(int kind, int block, int param, int depth, int nt, int grid, const void *const *in, int n,
           void *out, uint64_t bytes, void *stream) {
  if (n < 1 || n > 16 || (bytes & 15)) return -2;
  PArgs a;
  for (int k = 0; k < 16; k++) a.in[k] = (const char *)(k < n ? in[k] : in[0]);
  a.out = (char *)out;
  a.bytes = bytes;
  a.n = n;
  hipStream_t s = (hipStream_t)stream;
#define PH(B, P)                                                                        \
  if (block == B && param == P)                                                          \
    return nt ? launch(k_phase<B, P, 2, 2>, grid, B, a, s) : launch(k_phase<B, P, 0, 0>, grid, B, a, s);
#define SL(B, U)                                                                        \
  if (block == B && param == U)                                                          \
    return nt ? launch(k_slab<B, U, 2, 2>, grid, B, a, s) : launch(k_slab<B, U, 0, 0>, grid, B, a, s);
#define PN(B, P, D)                                                                     \
  if (block == B && param == P && depth == D)                                            \
    return nt ? launch(k_phase_n<B, P, 8, D, 2, 2>, grid, B, a, s)                       \
              : launch(k_phase_n<B, P, 8, D, 0, 0>, grid, B, a, s);
  if (kind == 0) {
    PH(256, 4) PH(256, 8) PH(256, 16) PH(256, 32) PH(512, 8) PH(512, 16) PH(1024, 4) PH(1024, 8)
  } else if (kind == 2) {
    if (n != 8) return -3;
    PN(256, 8, 2) PN(256, 16, 2) PN(512, 8, 2) PN(1024, 4, 2) PN(1024, 8, 2)
    PN(512, 8, 3) PN(1024, 4, 3) PN(512, 4, 3) PN(512, 4, 4) PN(1024, 8, 3) PN(256, 16, 3)
    PN(512, 16, 2) PN(512, 12, 2) PN(512, 14, 2) PN(256, 24, 2) PN(256, 32, 2) PN(256, 36, 2)
    PN(1024, 6, 2) PN(768, 8, 2) PN(512, 16, 1) PN(1024, 8, 1) PN(512, 8, 1)
  } else if (kind == 3) {
    if (block == 512 && param == 16) return launch(k_phase_lds<512, 16>, grid, 512, a, s);
    if (block == 512 && param == 8) return launch(k_phase_lds<512, 8>, grid, 512, a, s);
    if (block == 1024 && param == 8) return launch(k_phase_lds<1024, 8>, grid, 1024, a, s);
    if (block == 256 && param == 16) return launch(k_phase_lds<256, 16>, grid, 256, a, s);
  } else if (kind == 5) {
    if (block == 512 && param == 16) return launch(k_phase_flat<512, 16>, grid, 512, a, s);
    if (block == 512 && param == 8) return launch(k_phase_flat<512, 8>, grid, 512, a, s);
    if (block == 1024 && param == 8) return launch(k_phase_flat<1024, 8>, grid, 1024, a, s);
  } else if (kind == 6) {
    if (block == 512 && param == 16) return launch(k_phase_pipe<512, 16>, grid, 512, a, s);
    if (block == 512 && param == 8) return launch(k_phase_pipe<512, 8>, grid, 512, a, s);
    if (block == 1024 && param == 8) return launch(k_phase_pipe<1024, 8>, grid, 1024, a, s);
  } else if (kind == 7) {  // depth = SYNC_EVERY
    if (n != 8 || block != 512 || param != 16) return -3;
    if (depth == 1) return launch_sync<1>(grid, a, s);
    if (depth == 2) return launch_sync<2>(grid, a, s);
    if (depth == 4) return launch_sync<4>(grid, a, s);
  } else if (kind == 8) {  // param = U, depth = Q
    if (block == 512 && param == 8 && depth == 2) return launch(k_phase_q<512, 8, 2>, grid, 512, a, s);
    if (block == 512 && param == 4 && depth == 4) return launch(k_phase_q<512, 4, 4>, grid, 512, a, s);
    if (block == 512 && param == 8 && depth == 4) return launch(k_phase_q<512, 8, 4>, grid, 512, a, s);
    if (block == 512 && param == 4 && depth == 8) return launch(k_phase_q<512, 4, 8>, grid, 512, a, s);
    if (block == 1024 && param == 4 && depth == 2) return launch(k_phase_q<1024, 4, 2>, grid, 1024, a, s);
    if (block == 1024 && param == 4 && depth == 4) return launch(k_phase_q<1024, 4, 4>, grid, 1024, a, s);
    if (block == 256 && param == 8 && depth == 8) return launch(k_phase_q<256, 8, 8>, grid, 256, a, s);
    if (block == 512 && param == 6 && depth == 4) return launch(k_phase_q<512, 6, 4>, grid, 512, a, s);
  } else if (kind == 9) {
    if (n != 8) return -3;
    if (block == 512 && param == 16) return launch_dyn<512, 16>(grid, a, s);
    if (block == 1024 && param == 8) return launch_dyn<1024, 8>(grid, a, s);
    if (block == 512 && param == 8) return launch_dyn<512, 8>(grid, a, s);
  } else if (kind == 10) {  // per-wave dynamic, param = U
    if (n != 8) return -3;
    if (block == 256 && param == 4) return launch_wave_dyn<256, 4>(grid, a, s);
    if (block == 512 && param == 4) return launch_wave_dyn<512, 4>(grid, a, s);
    if (block == 256 && param == 2) return launch_wave_dyn<256, 2>(grid, a, s);
    if (block == 1024 && param == 4) return launch_wave_dyn<1024, 4>(grid, a, s);
  } else if (kind == 11) {  // per-workgroup dynamic tiles
    if (n != 8) return -3;
    if (block == 256 && param == 4) return launch_wg_dyn<256, 4>(grid, a, s);
    if (block == 256 && param == 2) return launch_wg_dyn<256, 2>(grid, a, s);
    if (block == 512 && param == 2) return launch_wg_dyn<512, 2>(grid, a, s);
  } else if (kind == 12) {  // multi-counter dynamic: depth = C; nt = 1 per-wave
    if (n != 8) return -3;
    if (block == 256 && param == 4 && depth == 2 && !nt) return launch_multi_dyn<256, 4, 2, false>(grid, a, s);
    if (block == 256 && param == 4 && depth == 4 && !nt) return launch_multi_dyn<256, 4, 4, false>(grid, a, s);
    if (block == 256 && param == 2 && depth == 4 && !nt) return launch_multi_dyn<256, 2, 4, false>(grid, a, s);
    if (block == 256 && param == 4 && depth == 4 && nt) return launch_multi_dyn<256, 4, 4, true>(grid, a, s);
    if (block == 256 && param == 4 && depth == 2 && nt) return launch_multi_dyn<256, 4, 2, true>(grid, a, s);
  } else if (kind == 4) {  // depth = MODE
    if (n != 8) return -3;
    if (block == 512 && param == 16 && depth == 0) return launch(k_phase_x<512, 16, 0>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 1) return launch(k_phase_x<512, 16, 1>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 2) return launch(k_phase_x<512, 16, 2>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 3) return launch(k_phase_x<512, 16, 3>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 4) return launch(k_phase_x<512, 16, 4>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 5) return launch(k_phase_x<512, 16, 5>, grid, 512, a, s);
    // depth 16+: store policy variants (aux = depth - 16)
    if (block == 512 && param == 16 && depth == 16 + 3) return launch(k_phase_x<512, 16, 0, 3>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 16 + 16) return launch(k_phase_x<512, 16, 0, 16>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 16 + 17) return launch(k_phase_x<512, 16, 0, 17>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 16 + 18) return launch(k_phase_x<512, 16, 0, 18>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 16 + 19) return launch(k_phase_x<512, 16, 0, 19>, grid, 512, a, s);
    if (block == 512 && param == 16 && depth == 16 + 1) return launch(k_phase_x<512, 16, 0, 1>, grid, 512, a, s);
  } else {
    SL(256, 4) SL(256, 2) SL(512, 4)
  }
#undef PH
#undef SL
  return -1;
}

// Allocation modes: 0 hipMalloc, 1 hipExtMallocWithFlags(contiguous),
// 2 VMM (hipMemCreate physical handle, reserved + mapped + RW access).
int pp_alloc(void **p, uint64_t bytes, int mode) {
  if (mode == 0) return (int)hipMalloc(p, bytes);
  if (mode == 1) return (int)hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous);
  if (mode == 2) {
    int dev = 0;
    hipGetDevice(&dev);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
    if (e) return (int)e;
    bytes = (bytes + gran - 1) / gran * gran;
    hipMemGenericAllocationHandle_t h;
    if ((e = hipMemCreate(&h, bytes, &prop, 0))) return (int)e;
    void *va = nullptr;
    if ((e = hipMemAddressReserve(&va, bytes, 0, nullptr, 0))) return (int)e;
    if ((e = hipMemMap(va, bytes, 0, h, 0))) return (int)e;
    hipMemAccessDesc d = {};
    d.location = prop.location;
    d.flags = hipMemAccessFlagsProtReadWrite;
    if ((e = hipMemSetAccess(va, bytes, &d, 1))) return (int)e;
    *p = va;
    return 0;
  }
  return -1;
}

uint64_t pp_granularity(void) {
  int dev = 0;
  hipGetDevice(&dev);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t g0 = 0, g1 = 0;
  hipMemGetAllocationGranularity(&g0, &prop, hipMemAllocationGranularityMinimum);
  hipMemGetAllocationGranularity(&g1, &prop, hipMemAllocationGranularityRecommended);
  return (g0 << 32) | (g1 & 0xffffffffu);
}
}

__global__ void k_diff(const uint32_t *a, const uint32_t *b, uint64_t nw, unsigned long long *cnt) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x)
    c += (a[i] != b[i]);
  if (c) atomicAdd(cnt, c);
}

extern "C" long long pp_diff(const void *a, const void *b, uint64_t bytes) {
  unsigned long long *d = nullptr, h = 0;
  if (hipMalloc(&d, 8)) return -1;
  hipMemset(d, 0, 8);
  hipLaunchKernelGGL(k_diff, dim3(2048), dim3(256), 0, 0, (const uint32_t *)a, (const uint32_t *)b, bytes / 4, d);
  hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  hipFree(d);
  return (long long)h;
}
