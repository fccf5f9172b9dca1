// hiccl_amd/csrc/reduce.hip -- MI355X (gfx950 / CDNA4) bucket-reduction stage.
//
// Implements include/hiccl_reduce.h.  The arithmetic is the reference's
// reduce_kernel<T> (source/compute.h:2-12 GPU, :14-23 CPU):
//
//     T acc = 0; for (k = 0; k < n; k++) acc += in[k][i]; out[i] = acc;
//
// reproduced bit for bit (same order, accumulator starts at +0 in T, every
// add rounded to T, no FMA, no tree).  Everything else is MI355X-first:
//
//  * pure HBM stream, (n + 1) * sizeof(T) bytes per element, no MFMA;
//  * 16-byte packets per lane (global_load_dwordx4 with an SGPR base +
//    32-bit lane offset), U packets per input per lane per tile, so each
//    lane has G*U independent 16-B loads in flight before the in-order adds;
//  * a persistent grid (CUs x blocks_per_cu workgroups); work units handed
//    out grid-stride or by a device ticket counter (dynamic schedule: no
//    workgroup is bound to a fixed subset of DRAM channels), buffer
//    descriptors make partial units predicate-free;
//  * two engines: TILE (all n inputs of a 16 KiB tile loaded together) and
//    PHASE (a 128 KiB chunk swept input by input); AUTO picks per launch;
//  * the input pointer table travels in the kernarg segment (scalar loads,
//    no device-side T** table and no H2D copy per call, cf. compute.h:70-72);
//  * the output is 16-B aligned by peeling a scalar head; inputs may be
//    mutually misaligned (partition() element offsets, reduce.h:401-415):
//    gfx950 serves unaligned dwordx4 loads in hardware;
//  * a batched plan kernel runs every compute of a pipeline step in ONE launch
//    from a device descriptor table (vs one kernel + one stream + one
//    hipStreamSynchronize per compute, compute.h:87-117);
//  * stream-ordered transport signalling (k_sigwait_phases) and step
//    programs (k_program: token phases folded into a batch's launch), with
//    fenced tokens by default (release stores, relaxed polls closed by one
//    acquire fence per phase; hiccl_token_mode).
//
// Layout / roofline / measured numbers: DESIGN.md.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <cctype>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/hiccl_reduce.h"

#define HICCL_VERSION_INT 100  // 0.1.0

namespace {

// ------------------------------------------------------------------ errors --

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

int check_hip(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return (int)e;
  }
  return 0;
}

// ------------------------------------------------------------ vector types --

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16-byte packet type with 1-byte alignment: a misaligned input still loads
// as one global_load_dwordx4 (gfx950 unaligned access mode).
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kPacket = 16;  // bytes per lane per load

// Buffer resources: one SGPR descriptor per input per tile (base = input +
// tile offset, range = the tile's valid bytes).  Loads/stores then take only
// the tile-invariant 32-bit lane offset, and the hardware range check turns
// the lanes past the end of the last (partial) tile into no-ops.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int kRsrcFlags = 0x00020000;  // raw buffer, 32-bit data format

__device__ __forceinline__ rsrc_t make_rsrc(const char *base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nbytes, kRsrcFlags);
}

// Cache policy, POL = 10*store + load.  load: 0 default, 1 nt (aux bit 1),
// 2 system scope (sc0 sc1: coherent with a peer GPU's writes -- the
// reading XCD's L2 does not serve a line of peer memory it cached earlier).
// store: 0 default, 1 nt, 2 sc1 (aux bit 4: write-through, line dropped
// from the XCD L2), 3 system scope (sc0 sc1: written through to the memory
// that owns the line, a peer GPU's HBM over xGMI included -- nt stores are
// not write-through and may sit dirty in this XCD's L2 after the kernel).
// The system-scope forms are the PEER policies of plans whose outputs or
// inputs live in another GPU's memory (hiccl_reduce_plan_set_peer).
constexpr int kPolLoadSys = 2;
constexpr int kPolStoreSys = 3;

template <int POL>
__device__ __forceinline__ u32x4 load_pkt(rsrc_t r, uint32_t voff) {
  constexpr int lp = POL % 10;
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, lp == 1 ? 2 : lp == kPolLoadSys ? 17 : 0);
}

template <int POL>
__device__ __forceinline__ void store_pkt(rsrc_t r, uint32_t voff, u32x4 v) {
  constexpr int sp = POL / 10;
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, 0, sp == 1 ? 2 : sp == 2 ? 16 : sp == kPolStoreSys ? 17 : 0);
}

// bf16 <-> f32.  f32 -> bf16 is round-to-nearest-even; on gfx950 the cast
// lowers to v_cvt_pk_bf16_f32, which keeps a NaN a NaN.
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t bf_pack(float lo, float hi) {
  bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ uint16_t bf_round(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

// Scalar head/tail accesses through the GLOBAL address space: a generic
// pointer becomes a flat access, and a flat load pending anywhere inside the
// plan kernel's unit loop makes the waitcnt pass treat vmcnt as out of order
// -- every tile's adds then waited with vmcnt(0) instead of a staircase.
template <class T>
__device__ __forceinline__ T gld(const char *p) {
  return *(const __attribute__((address_space(1))) T *)p;
}
template <class T>
__device__ __forceinline__ void gst(char *p, T v) {
  *(__attribute__((address_space(1))) T *)p = v;
}

// ------------------------------------------------------------ element ops --
// Each op: elem size, packet accumulator (acc_t) with zero/add/pack, and a
// scalar accumulator for the peeled head/tail elements.  zero() + x keeps the
// reference's `T acc = 0; acc += x` (so -0 inputs sum to +0).

struct OpF32 {
  static constexpr bool kWidens = false;
  static constexpr int kEsz = 4;
  typedef f32x4 acc_t;
  __device__ static acc_t zero() { return (f32x4)(0.0f); }
  __device__ static acc_t add(acc_t a, u32x4 p) { return a + __builtin_bit_cast(f32x4, p); }
  __device__ static u32x4 pack(acc_t a) { return __builtin_bit_cast(u32x4, a); }
  typedef float sacc_t;
  __device__ static sacc_t szero() { return 0.0f; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) { return a + gld<float>(p); }
  __device__ static void sstore(char *p, sacc_t a) { gst<float>(p, a); }
};

struct OpF64 {
  static constexpr bool kWidens = false;
  static constexpr int kEsz = 8;
  typedef f64x2 acc_t;
  __device__ static acc_t zero() { return (f64x2)(0.0); }
  __device__ static acc_t add(acc_t a, u32x4 p) { return a + __builtin_bit_cast(f64x2, p); }
  __device__ static u32x4 pack(acc_t a) { return __builtin_bit_cast(u32x4, a); }
  typedef double sacc_t;
  __device__ static sacc_t szero() { return 0.0; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) { return a + gld<double>(p); }
  __device__ static void sstore(char *p, sacc_t a) { gst<double>(p, a); }
};

struct OpU64 {
  static constexpr bool kWidens = false;
  static constexpr int kEsz = 8;
  typedef u64x2 acc_t;
  __device__ static acc_t zero() { return (u64x2)(0); }
  __device__ static acc_t add(acc_t a, u32x4 p) { return a + __builtin_bit_cast(u64x2, p); }
  __device__ static u32x4 pack(acc_t a) { return __builtin_bit_cast(u32x4, a); }
  typedef uint64_t sacc_t;
  __device__ static sacc_t szero() { return 0; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) { return a + gld<uint64_t>(p); }
  __device__ static void sstore(char *p, sacc_t a) { gst<uint64_t>(p, a); }
};

struct OpI32 {  // two's-complement wrap-around, done in unsigned
  static constexpr bool kWidens = false;
  static constexpr int kEsz = 4;
  typedef u32x4 acc_t;
  __device__ static acc_t zero() { return (u32x4)(0u); }
  __device__ static acc_t add(acc_t a, u32x4 p) { return a + p; }
  __device__ static u32x4 pack(acc_t a) { return a; }
  typedef uint32_t sacc_t;
  __device__ static sacc_t szero() { return 0u; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) { return a + gld<uint32_t>(p); }
  __device__ static void sstore(char *p, sacc_t a) { gst<uint32_t>(p, a); }
};

// bf16, reference semantics: acc is bf16, every add = f32 add then round to
// bf16.  The accumulator is kept PACKED (8 bf16 in a u32x4, the packet's own
// layout): widen both operands (exact), add in f32, round-to-nearest-even
// back (v_cvt_pk_bf16_f32).  4 VGPRs per packet, so the phased engine runs
// bf16 at the same 128 KiB chunk as f32.
// The pack is an opaque v_cvt_pk_bf16_f32 (the same instruction the __bf16
// casts lower to) so the compiler cannot see through pack->widen and keep the
// accumulator widened in 8 VGPRs per packet (it does, and spills).
__device__ __forceinline__ uint32_t bf_pack_opaque(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

struct OpBF16 {
  static constexpr bool kWidens = true;
  static constexpr int kEsz = 2;
  typedef u32x4 acc_t;
  __device__ static acc_t zero() { return (u32x4)(0u); }  // +0 bf16
  __device__ static acc_t add(acc_t a, u32x4 p) {
    acc_t r;
#pragma unroll
    for (int w = 0; w < 4; w++)
      r[w] = bf_pack_opaque(bf_lo(a[w]) + bf_lo(p[w]), bf_hi(a[w]) + bf_hi(p[w]));
    return r;
  }
  __device__ static u32x4 pack(acc_t a) { return a; }
  typedef float sacc_t;
  __device__ static sacc_t szero() { return 0.0f; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) {
    float s = a + __uint_as_float((uint32_t)(gld<uint16_t>(p)) << 16);
    return __uint_as_float((uint32_t)bf_round(s) << 16);
  }
  __device__ static void sstore(char *p, sacc_t a) { gst<uint16_t>(p, bf_round(a)); }
};

// bf16 inputs, f32 accumulator, one rounding at the end (HICCL_ACC_WIDE).
struct OpBF16Wide {
  static constexpr bool kWidens = true;
  static constexpr int kEsz = 2;
  typedef f32x8 acc_t;
  __device__ static acc_t zero() { return (f32x8)(0.0f); }
  __device__ static acc_t add(acc_t a, u32x4 p) {
#pragma unroll
    for (int w = 0; w < 4; w++) {
      a[2 * w] += bf_lo(p[w]);
      a[2 * w + 1] += bf_hi(p[w]);
    }
    return a;
  }
  __device__ static u32x4 pack(acc_t a) {
    u32x4 r;
#pragma unroll
    for (int w = 0; w < 4; w++) r[w] = bf_pack(a[2 * w], a[2 * w + 1]);
    return r;
  }
  typedef float sacc_t;
  __device__ static sacc_t szero() { return 0.0f; }
  __device__ static sacc_t sadd(sacc_t a, const char *p) {
    return a + __uint_as_float((uint32_t)(gld<uint16_t>(p)) << 16);
  }
  __device__ static void sstore(char *p, sacc_t a) { gst<uint16_t>(p, bf_round(a)); }
};

// Exact byte copy (HICCL_BYTES): one input, out = in[0] bit for bit.  The
// transport's batched data movement runs on the same tile engine.
struct OpRaw {
  static constexpr bool kWidens = false;
  static constexpr int kEsz = 1;
  typedef u32x4 acc_t;
  __device__ static acc_t zero() { return (u32x4)(0u); }
  __device__ static acc_t add(acc_t, u32x4 p) { return p; }
  __device__ static u32x4 pack(acc_t a) { return a; }
  typedef uint8_t sacc_t;
  __device__ static sacc_t szero() { return 0; }
  __device__ static sacc_t sadd(sacc_t, const char *p) { return gld<uint8_t>(p); }
  __device__ static void sstore(char *p, sacc_t a) { gst<uint8_t>(p, a); }
};

// ----------------------------------------------------------- tile engine --
//
// A compute is split as [head scalars | npkt 16-B packets | tail scalars],
// the packets 16-B aligned on the OUTPUT.  A tile = BLOCK*U packets; lane t
// of the workgroup owns packets u*BLOCK + t (u < U), so every load
// instruction of a wave covers 1 KiB contiguous bytes of one input.

constexpr int kMaxArgInputs = 64;  // kernarg pointer table (512 B)

struct SingleArgs {
  char *out;          // raw output pointer
  uint64_t npkt;      // body packets
  uint64_t ntiles;    // >= 1
  uint32_t n;         // inputs
  uint32_t head;      // scalar elements before the body
  uint32_t tail;      // scalar elements after the body
  uint32_t order;     // log2 of the tile-order segments (0: linear; tile_order)
  uint32_t *sched;    // dynamic unit counter {ticket, done}, or NULL: static grid-stride
  uint32_t grab;      // units per ticket (dynamic schedule), >= 1
  uint32_t drain;     // 1: wait for a unit's stores before the next unit's loads
  const char *in[kMaxArgInputs];
};

// Descriptor of one compute in a batched plan (device memory).
struct PlanDesc {
  char *out;
  uint64_t npkt;
  uint64_t tile_begin;  // first global unit of this compute
  uint32_t n, head, tail, pad;
};
static_assert(sizeof(PlanDesc) == 40, "PlanDesc layout");

// A plan launch.  One device block holds [desc | ptrs | unit_comp]:
//   desc[c]                  compute c
//   ptrs[c * stride + k]     input k of compute c (stride = the plan's max n)
//   unit_comp[t]             the compute owning global unit t (NULL: compute 0)
// so a workgroup reaches a unit's input pointers in two dependent scalar
// loads: unit_comp[t], then desc[c] and ptrs[c * stride ...] side by side.
struct PlanArgs {
  const PlanDesc *desc;
  const char *const *ptrs;
  const uint32_t *unit_comp;
  uint64_t t_begin, t_end;
  uint32_t *sched;  // dynamic unit counter, or NULL
  uint32_t stride, grab;
};

// Input pointer source: kernarg array or device table.
struct ArgInputs {
  const char *const *p;
  __device__ const char *operator()(int k) const { return p[k]; }
};

// Under the peer policies the plain scalar accesses are bracketed by
// system-scope fences instead (an acquire before the loads: this XCD's L2
// drops lines of peer memory; a release after the stores: its dirty lines
// are written back) -- only the workgroup owning a compute's first unit,
// and only when the compute has a head or a tail.
template <class Op, int POL = 11, class Inputs>
__device__ __forceinline__ void scalar_part(char *out, Inputs in, uint32_t n, uint32_t head,
                                            uint64_t npkt, uint32_t tail, int tid) {
  constexpr int V = kPacket / Op::kEsz;
  if (tid >= (int)(head + tail)) return;
  if constexpr (POL % 10 == kPolLoadSys) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  uint64_t e = (tid < (int)head) ? (uint64_t)tid : (uint64_t)head + npkt * V + (tid - head);
  uint64_t off = e * Op::kEsz;
  typename Op::sacc_t acc = Op::szero();
  for (uint32_t k = 0; k < n; k++) acc = Op::sadd(acc, in(k) + off);
  Op::sstore(out + off, acc);
  if constexpr (POL / 10 == kPolStoreSys) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// One group of G inputs (G static): G descriptor builds (scalar), then G*U
// independent 16-B buffer loads, then the G in-order adds per packet.
template <class Op, int U, int G, int POL, class Inputs>
__device__ __forceinline__ void group_at(typename Op::acc_t (&acc)[U], Inputs in, uint32_t g,
                                         uint64_t tile_off, uint32_t tile_bytes,
                                         const uint32_t (&voff)[U]) {
  rsrc_t r[G];
#pragma unroll
  for (int j = 0; j < G; j++) r[j] = make_rsrc(in(g + j) + tile_off, tile_bytes);
  u32x4 x[G][U];
  // Every load of the group is issued before the first add, input by input
  // (the barriers pin that order, so the adds -- input 0 first -- wait with
  // a vmcnt staircase instead of one vmcnt(0)).  Without them the scheduler
  // of the plan kernel (pointer table in memory) split an 8-input group into
  // 24 + 8 (f32) or 16 + 16 (bf16) loads with an s_waitcnt vmcnt(0) in
  // between: two memory round trips per tile.
#pragma unroll
  for (int j = 0; j < G; j++) {
#pragma unroll
    for (int u = 0; u < U; u++) x[j][u] = load_pkt<POL>(r[j], voff[u]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < G; j++) {
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = Op::add(acc[u], x[j][u]);
  }
}

// One tile: packets pkt0 + u*BLOCK + tid, tile_bytes = valid bytes of the
// tile (< the full tile only for the last one).  Inputs are consumed as full
// groups of 8 followed by one statically sized remainder group, so the adds
// happen in exactly the order k = 0, 1, ..., n-1.
// `before_store()` runs after the last add, before the stores (the unit
// scheduler publishes its next ticket there: every load has been waited for
// and no store is pending yet, so reading the atomic's result costs nothing).
struct NoHook {
  __device__ void operator()() const {}
};

template <class Op, int U, int POL, class Inputs, class Hook = NoHook>
__device__ __forceinline__ void tile_body(char *outb, Inputs in, uint32_t n, uint64_t tile_off,
                                          uint32_t tile_bytes, const uint32_t (&voff)[U],
                                          Hook before_store = Hook()) {
  typename Op::acc_t acc[U];
#pragma unroll
  for (int u = 0; u < U; u++) acc[u] = Op::zero();
  // groups of GM inputs: at most 32 packets per lane in flight (U = 8: 4
  // inputs, U = 16: 2), so wide tiles stay within the register file
  constexpr uint32_t GM = U >= 8 ? 32 / U : 8;
  uint32_t g = 0;
  for (; g + GM <= n; g += GM) group_at<Op, U, GM, POL>(acc, in, g, tile_off, tile_bytes, voff);
  switch (n - g) {  // wave-uniform
    case 1: group_at<Op, U, 1, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 2: if constexpr (GM > 2) group_at<Op, U, 2, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 3: if constexpr (GM > 3) group_at<Op, U, 3, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 4: if constexpr (GM > 4) group_at<Op, U, 4, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 5: if constexpr (GM > 5) group_at<Op, U, 5, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 6: if constexpr (GM > 6) group_at<Op, U, 6, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    case 7: if constexpr (GM > 7) group_at<Op, U, 7, POL>(acc, in, g, tile_off, tile_bytes, voff); break;
    default: break;
  }
  before_store();
  rsrc_t w = make_rsrc(outb + tile_off, tile_bytes);
#pragma unroll
  for (int u = 0; u < U; u++) store_pkt<POL>(w, voff[u], Op::pack(acc[u]));
}

// Input-phased chunk (the default engine for large buckets).  A chunk =
// BLOCK*P packets; lane t owns packets p*BLOCK + t.  The workgroup sweeps
// input 0 of the chunk, then input 1, ...: input j+1's P loads are in flight
// while input j is added, so chip-wide only ~2 input streams are open at a
// time and each is read as long contiguous runs (BLOCK*P*16 B per workgroup;
// 128 KiB at the default 512 x 16).  The per-element add order is unchanged
// (k = 0, 1, ..., n-1 from a zero accumulator).  Measured: the nine-stream
// tile order runs at 5.5-5.8 TB/s and depends on the physical placement of
// the buckets; the phased order at 6.0-6.4 TB/s.
// n is runtime: inputs are taken in pairs; the load that would read past
// input n-1 gets a zero-range descriptor (no memory traffic, reads 0, never
// added).
template <class Op, int P, int POL, class Inputs, class Hook = NoHook>
__device__ __forceinline__ void chunk_body(char *outb, Inputs in, uint32_t n, uint64_t off,
                                           uint32_t nbytes, const uint32_t (&voff)[P],
                                           Hook before_store = Hook()) {
  typename Op::acc_t acc[P];
#pragma unroll
  for (int p = 0; p < P; p++) acc[p] = Op::zero();
  if (n > 0) {
    u32x4 x[P], y[P];
    {
      rsrc_t r = make_rsrc(in(0) + off, nbytes);
#pragma unroll
      for (int p = 0; p < P; p++) x[p] = load_pkt<POL>(r, voff[p]);
    }
    uint32_t j = 0;
    for (; j + 2 <= n; j += 2) {  // x: input j in flight
      rsrc_t ry = make_rsrc(in(j + 1) + off, nbytes);
#pragma unroll
      for (int p = 0; p < P; p++) y[p] = load_pkt<POL>(ry, voff[p]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) {
        acc[p] = Op::add(acc[p], x[p]);
        if constexpr (Op::kWidens) __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      const bool more = j + 2 < n;
      rsrc_t rx = make_rsrc(in(more ? j + 2 : j + 1) + off, more ? nbytes : 0u);
#pragma unroll
      for (int p = 0; p < P; p++) x[p] = load_pkt<POL>(rx, voff[p]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int p = 0; p < P; p++) {
        acc[p] = Op::add(acc[p], y[p]);
        if constexpr (Op::kWidens) __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (n & 1) {
#pragma unroll
      for (int p = 0; p < P; p++) acc[p] = Op::add(acc[p], x[p]);
    }
  }
  before_store();
  rsrc_t w = make_rsrc(outb + off, nbytes);
#pragma unroll
  for (int p = 0; p < P; p++) store_pkt<POL>(w, voff[p], Op::pack(acc[p]));
}

// Engines: kTile = all n inputs of a BLOCK*U tile loaded together (small
// computes, many tiles); kPhase = chunk_body (large buckets).
constexpr int kTile = 0;
constexpr int kPhase = 1;

template <class Op, int U, int POL, int ENG, class Inputs, class Hook>
__device__ __forceinline__ void unit_body(char *outb, Inputs in, uint32_t n, uint64_t off,
                                          uint32_t nbytes, const uint32_t (&voff)[U], Hook hook) {
  if constexpr (ENG == kPhase)
    chunk_body<Op, U, POL>(outb, in, n, off, nbytes, voff, hook);
  else
    tile_body<Op, U, POL>(outb, in, n, off, nbytes, voff, hook);
}

// Body inputs shifted by the head: base(k) = in[k] + head*esz.
template <class Inner>
struct Shifted {
  Inner in;
  uint64_t shift;
  __device__ const char *operator()(int k) const { return in(k) + shift; }
};

// ---------------------------------------------------- unit scheduling ----
//
// Static: workgroup b takes units b, b + grid, ...  Dynamic (sched != NULL):
// every workgroup takes its next unit from a device counter, so the
// workgroups the memory system serves faster do more units and the launch's
// tail is one unit instead of the slowest workgroup's share (+1.6-2.1 % on
// C2: profiles/r01_phase_probe_dyn.jsonl).  The next ticket is fetched one
// unit ahead so the atomic's latency hides under the current unit.  The
// counter pair {ticket, done} is zero on entry; the last workgroup to finish
// resets it, so consecutive launches on one stream (or replays of a graph)
// reuse it without a memset.  The host gives every (device, stream) its own
// pair and never uses it during stream capture (unit_sched_for()).
__device__ __forceinline__ void drain_stores(uint32_t drain) {
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <class Body>
__device__ __forceinline__ void for_each_unit(uint32_t *sched, uint32_t grab, uint64_t t0, uint64_t t1,
                                              Body body, uint32_t drain = 0) {
  if (!sched) {
    for (uint64_t t = t0 + blockIdx.x; t < t1; t += gridDim.x) {
      body(t, [] {});
      drain_stores(drain);
    }
    return;
  }
  // a ticket k covers units [t0 + k*grab, t0 + (k+1)*grab)
  __shared__ uint32_t s_next[2];
  if (threadIdx.x == 0)
    s_next[0] = __hip_atomic_fetch_add(&sched[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  uint64_t t = t0 + (uint64_t)s_next[0] * grab;
  int slot = 1;
  while (t < t1) {
    // the next ticket is grabbed before this one's loads; its value is
    // published after the last unit's last add and before that unit's stores
    // (the body's hook), where every load has been waited for, so the wait
    // costs little (a wait with stores pending is vmcnt(0))
    uint32_t nxt;  // meaningful in lane 0 only; no merge value, so no wait at the branch join
    if (threadIdx.x == 0)
      nxt = __hip_atomic_fetch_add(&sched[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tend = (t + grab < t1) ? t + grab : t1;
    for (uint64_t u = t; u < tend; u++) {
      const bool last = u + 1 == tend;
      body(u, [&]() {
        if (last && threadIdx.x == 0) s_next[slot] = nxt;
      });
      drain_stores(drain);
    }
    __syncthreads();
    t = t0 + (uint64_t)s_next[slot] * grab;
    slot ^= 1;
  }
  if (threadIdx.x == 0) {
    // every ticket grab of this workgroup precedes its done increment
    const uint32_t prev = __hip_atomic_fetch_add(&sched[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // last workgroup: no grab is outstanding
      __hip_atomic_store(&sched[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sched[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Tile order: unit t of a launch of n units runs tile tile_order(t).  With
// 2^L segments the order interleaves them -- consecutive units (the ones in
// flight together across the chip) spread over 2^L equal stretches of every
// input instead of one contiguous window -- a bijection on [0, n) for any n
// (segment s holds q + (s < r) tiles, q = n >> L, r = n mod 2^L; the last r
// units are the long segments' extra tiles).  L = 0: linear.
__device__ __forceinline__ uint64_t tile_order(uint64_t t, uint64_t n, uint32_t L) {
  if (!L) return t;
  const uint64_t S = 1ull << L, q = n >> L, r = n & (S - 1);
  uint64_t seg, idx;
  if (t < (q << L)) {
    seg = t & (S - 1);
    idx = t >> L;
  } else {
    seg = t - (q << L);
    idx = q;
  }
  return seg * q + (seg < r ? seg : r) + idx;
}

// ------------------------------------------------------------ kernels ------

template <class Op, int BLOCK, int U, int POL, int ENG>
__global__ __launch_bounds__(BLOCK) void k_reduce_single(SingleArgs a) {
  const int tid = threadIdx.x;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * BLOCK + tid) * kPacket);
  ArgInputs raw{a.in};
  if (blockIdx.x == 0) scalar_part<Op>(a.out, raw, a.n, a.head, a.npkt, a.tail, tid);
  if (a.npkt == 0) return;  // (the host never passes a sched counter then)
  const uint64_t shift = (uint64_t)a.head * Op::kEsz;
  Shifted<ArgInputs> in{raw, shift};
  char *outb = a.out + shift;
  constexpr uint64_t TILE = (uint64_t)BLOCK * U;
  for_each_unit(a.sched, a.grab, 0, a.ntiles, [&](uint64_t u, auto hook) {
    const uint64_t t = tile_order(u, a.ntiles, a.order);
    const uint64_t pkt0 = t * TILE;
    const uint64_t left = a.npkt - pkt0;
    const uint32_t tile_bytes = (uint32_t)((left < TILE ? left : TILE) * kPacket);
    unit_body<Op, U, POL, ENG>(outb, in, a.n, pkt0 * kPacket, tile_bytes, voff, hook);
  }, a.drain);
}

// The plan's device pointer table is read through the constant address space
// (4): the loads are then scalar (s_load) and the pointers known uniform.
// Through a generic pointer the compiler emits a flat load -- whose
// s_waitcnt vmcnt(0) drains every buffer load in flight -- and a
// readfirstlane waterfall loop around every buffer load using the pointer.
typedef const char *const __attribute__((address_space(4))) ConstPtr;

struct TableInputs {
  const char *const *p;
  __device__ const char *operator()(int k) const { return ((ConstPtr *)p)[k]; }
};

typedef const PlanDesc __attribute__((address_space(4))) ConstDesc;
typedef const uint32_t __attribute__((address_space(4))) ConstU32;

__device__ __forceinline__ PlanDesc load_desc(const PlanDesc *desc, uint32_t c) {
  const ConstDesc *q = (const ConstDesc *)desc + c;  // scalar loads
  PlanDesc d;
  d.out = q->out;
  d.npkt = q->npkt;
  d.tile_begin = q->tile_begin;
  d.n = q->n;
  d.head = q->head;
  d.tail = q->tail;
  d.pad = 0;
  return d;
}

// All computes of a plan in one launch.  Global unit t belongs to compute
// unit_comp[t] (the host's table: one scalar load, instead of a search over
// the computes' first units whose dependent probes cost several
// microseconds in the first unit of every workgroup of a small plan).
template <class Op, int BLOCK, int U, int POL, int ENG>
__global__ __launch_bounds__(BLOCK) void k_reduce_plan(PlanArgs a) {
  const int tid = threadIdx.x;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * BLOCK + tid) * kPacket);
  constexpr uint64_t TILE = (uint64_t)BLOCK * U;
  for_each_unit(a.sched, a.grab, a.t_begin, a.t_end, [&](uint64_t t, auto hook) {
    const uint32_t c = a.unit_comp ? ((ConstU32 *)a.unit_comp)[t] : 0u;
    const PlanDesc d = load_desc(a.desc, c);
    const uint64_t lt = t - d.tile_begin;
    TableInputs raw{a.ptrs + (uint64_t)c * a.stride};
    if (lt == 0) scalar_part<Op, POL>(d.out, raw, d.n, d.head, d.npkt, d.tail, tid);
    const uint64_t pkt0 = lt * TILE;
    if (pkt0 >= d.npkt) {  // a scalar-only compute: nothing to load or store
      hook();
      return;
    }
    const uint64_t shift = (uint64_t)d.head * Op::kEsz;
    Shifted<TableInputs> in{raw, shift};
    const uint64_t left = d.npkt - pkt0;
    const uint32_t tile_bytes = (uint32_t)((left < TILE ? left : TILE) * kPacket);
    unit_body<Op, U, POL, ENG>(d.out + shift, in, d.n, pkt0 * kPacket, tile_bytes, voff, hook);
  });
}

// ------------------------------------------------------- synthetic inputs --

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float uniform_f32(uint64_t key, uint64_t i) {
  uint64_t h = splitmix64(key + i);
  return (float)(uint32_t)(h >> 40) * (1.0f / 8388608.0f) - 1.0f;
}

template <int DT>
__global__ __launch_bounds__(256) void k_fill(char *out, uint64_t count, uint64_t key,
                                              uint64_t first) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count;
       i += (uint64_t)gridDim.x * 256) {
    float v = uniform_f32(key, first + i);
    if constexpr (DT == HICCL_FLOAT32) ((float *)out)[i] = v;
    if constexpr (DT == HICCL_FLOAT64) ((double *)out)[i] = (double)v;
    if constexpr (DT == HICCL_BFLOAT16) ((uint16_t *)out)[i] = bf_round(v);
  }
}

__global__ __launch_bounds__(256) void k_copy(u32x4 *__restrict__ dst,
                                              const u32x4 *__restrict__ src, uint64_t npkt) {
  constexpr int U = 4;
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U; b < npkt; b += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t p = b + u * 256 + threadIdx.x;
      if (p < npkt) v[u] = src[p];
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t p = b + u * 256 + threadIdx.x;
      if (p < npkt) dst[p] = v[u];
    }
  }
}

__global__ void k_copy_bytes(char *dst, const char *src, uint64_t nbytes) {
  for (uint64_t i = threadIdx.x; i < nbytes; i += blockDim.x) dst[i] = src[i];
}

// ------------------------------------------------------ stream signalling --
// One wave: lanes < nsig publish `epoch` to (typically peer, IPC-mapped)
// flags with a system-scope release store; lanes < nwait spin on local flags
// with system-scope acquire loads until they reach `epoch`.  Every spin is
// bounded (s_memrealtime, 100 MHz): on timeout the lane records an error and
// exits, so a broken protocol can never hang the GPU.

constexpr int kMaxFlags = 64;  // signal and wait flags per launch (one per lane)

// Several signal/wait phases in ONE launch, executed in order: phase p
// stores its epoch to its flags (system-scope release), then waits for its
// flags (relaxed polls, then a system-scope acquire fence); phase
// p + 1 starts after every wait of phase p has finished.  The transport queues the consecutive signal/wait steps of
// a stream-ordered pipeline (a step's done tokens, the next step's readies)
// into one such launch instead of one launch each: same order of every
// operation on the stream, fewer kernel boundaries (~1.5-1.9 us each).
constexpr int kMaxPhases = 8;

struct SigPhaseArgs {
  uint32_t *sig[kMaxFlags];
  const uint32_t *wait[kMaxFlags];
  uint32_t *err;
  const uint32_t *epoch_dev;  // NULL, or a device word added to every epoch at run time (graph replays)
  uint64_t timeout_ticks;
  uint32_t nphase;
  uint32_t light;  // 1: relaxed stores and polls, no fences (HICCL_PROG_FENCES, as the programs' prologue)
  uint32_t sig_end[kMaxPhases];   // phase p signals sig[sig_end[p-1] .. sig_end[p])
  uint32_t wait_end[kMaxPhases];  // and waits for wait[wait_end[p-1] .. wait_end[p])
  uint32_t epoch[kMaxPhases];
};

__global__ __launch_bounds__(64) void k_sigwait_phases(SigPhaseArgs a) {
  const uint32_t lane = threadIdx.x;
  const uint32_t add = a.epoch_dev ? __hip_atomic_load(a.epoch_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  uint32_t s0 = 0, w0 = 0;
  for (uint32_t p = 0; p < a.nphase; p++) {
    const uint32_t epoch = a.epoch[p] + add;
    const uint32_t s1 = a.sig_end[p], w1 = a.wait_end[p];
    if (s0 + lane < s1) {
      if (a.light)
        __hip_atomic_store(a.sig[s0 + lane], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        __hip_atomic_store(a.sig[s0 + lane], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (w0 + lane < w1) {
      const uint32_t *f = a.wait[w0 + lane];
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      // relaxed polls in both modes (no cache invalidate per poll); in the
      // fenced mode the system-scope acquire fence below, executed by
      // this lane after its last poll, makes the load that saw the peer's
      // release store synchronise with it -- the fence form of an acquire
      // load, paid once per phase instead of once per poll
      auto poll = [&]() { return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
      while ((int32_t)(poll() - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (a.err && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
          if (a.err) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    // fenced mode: each lane's acquire half of its polls, sequenced after
    // its last poll; then every lane's waits (and acquires, carried to the
    // other lanes by the barrier's workgroup-scope fences) precede any store
    // of the next phase
    if (!a.light) __atomic_thread_fence(__ATOMIC_ACQUIRE);
    __syncthreads();
    s0 = s1;
    w0 = w1;
  }
}

// One lane adds v to a device counter (stream-ordered; graph replay number).
__global__ __launch_bounds__(64) void k_counter_add(uint32_t *ctr, uint32_t v) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------ step programs --
//
// A stream-ordered pipeline step is a short ordered list: ready-token phases,
// the transport's batched copies, done-token phases, the step's reductions,
// the fused transfers' done tokens.  Launched one by one that is a
// k_sigwait_phases before every copy or reduction kernel.  A PROGRAM folds
// the signal/wait phases that precede a batch of units into that batch's
// kernel as a PROLOGUE: workgroup 0's first wave runs the phases in order
// (system-scope release stores of the epochs, bounded acquire spins -- as
// k_sigwait_phases), then publishes the launch's sequence number in the
// program's gate word; every other workgroup waits for that word before its
// first unit.  The units are the tiles of the batch's computes (reductions in
// the program's type, or exact byte copies), statically interleaved over the
// grid like the plan kernel.
//
// Measured alternative (round 3, profiles/r03f_progstep_*.jsonl): running a
// whole step -- several unit batches with completion gates between them --
// in one launch.  Completions then need grid-wide counting (atomics on one
// line from every workgroup) and, MI355X's L2 being per XCD, a system-scope
// L2 writeback per workgroup before each count and an invalidate after each
// gate: 40-170 us per step against 18-22 us for the separate launches.  A
// kernel boundary does that cache maintenance once per XCD.  So units that
// depend on other units stay in separate launches; only the token phases
// move into the kernels.
//
// Coherence of the prologue: no unit of the launch touches its data before
// the gate opens, so the data the phases waited for (peers' writes over
// xGMI) is read after it arrived, as it is by a kernel launched after a
// separate k_sigwait_phases; the launch's own stores are released at its
// end like any kernel's.

constexpr int kProgMaxPhases = 64;
constexpr int kProgBlock = 256;
constexpr int kProgPol = 11;  // nt loads, nt stores (the library's default policy)

struct ProgPhase {
  uint32_t sig_begin, sig_end, wait_begin, wait_end;
};

struct ProgArgs {
  const PlanDesc *desc;  // computes of the unit batch; pad bit 0: exact byte copy, bits 1-2: peer flags
  const char *const *ptrs;
  const uint32_t *unit_comp;
  const ProgPhase *phase;
  uint32_t *const *sig;
  const uint32_t *const *wait;
  uint64_t *gate;  // workgroup 0 stores the launch's sequence number here after the phases
  uint32_t *err;
  const uint32_t *epoch_dev;
  uint64_t timeout_ticks;
  uint64_t nunits;
  uint32_t stride, nphase;
  uint64_t seq;  // this launch's gate value (+ *epoch_dev); never reused, see hiccl_program_launch
  uint32_t light;  // 1: relaxed token stores, no fences in the prologue (HICCL_PROG_FENCES, prog_light())
  uint32_t epoch[kProgMaxPhases];  // per launch: phase p stores / awaits epoch[p] (+ *epoch_dev)
};

// Phases [0, count) on one wave (lanes = flags), as k_sigwait_phases.
//
// `light` (opt-in, HICCL_PROG_FENCES=light): relaxed system-scope token stores
// and no fence after the waits.  A program's tokens never publish data of
// their own launch -- a done token follows the copies or reductions of an
// EARLIER launch (complete, and released, at that kernel's end; a peer's
// buffer written through with the peer policy), a ready token only says a
// buffer an earlier launch read is free -- and this launch's units start
// after the gate, on workgroups whose L1 holds none of their data (the
// kernel-start acquire invalidated it and nothing read it since).  The wave
// issues a phase's stores only after its polls of the previous phase have
// returned (the loop exits on the loaded value).  Fenced mode (the
// default: release stores, an acquire fence per phase after relaxed polls, a
// release gate store) orders workgroup 0 after the peers by the memory model,
// and the other workgroups after workgroup 0 by an agent-scope acquire after
// their gate polls (k_program); light mode leaves the gate hand-off relaxed.
__device__ __forceinline__ void prog_phases(const ProgArgs &a, uint32_t count, uint32_t lane, uint32_t add) {
  for (uint32_t p = 0; p < count; p++) {
    const ConstU32 *q = (const ConstU32 *)&a.phase[p];
    const uint32_t s0 = q[0], s1 = q[1], w0 = q[2], w1 = q[3];
    const uint32_t epoch = a.epoch[p] + add;
    for (uint32_t i = s0 + lane; i < s1; i += 64) {
      uint32_t *f = ((uint32_t *const __attribute__((address_space(4))) *)a.sig)[i];
      if (a.light)
        __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (uint32_t i = w0 + lane; i < w1; i += 64) {
      const uint32_t *f = ((const uint32_t *const __attribute__((address_space(4))) *)a.wait)[i];
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      // relaxed polls (no cache invalidate per poll); the fence below acquires
      while ((int32_t)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (a.err && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
          if (a.err) __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
    }
    // fenced mode: each lane's acquire half of its polls, after its last
    // poll; then every lane's waits (and acquires) precede any store of the
    // next phase -- a wave-level barrier whose wavefront-scope fences carry
    // the ordering from lane to lane (only this wave runs the phases, so no
    // workgroup barrier is available here)
    if (!a.light) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Bounded wait of one lane until the gate word holds this launch's `seq`;
// on a time-out or an error recorded by anyone it gives up (the grid drains,
// the host reports the error).  Relaxed polls with backoff: hundreds of
// workgroups poll one line.  Equality, not >=: the word holds the previous
// launch's value until workgroup 0 stores ours, and no two launches of a
// program share a value (64-bit, hiccl_program_launch), so a later eager
// launch's value can never open a replay's gate early.
__device__ __forceinline__ void prog_gate_wait(const ProgArgs &a, uint64_t seq) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nap = 1;
  while (__hip_atomic_load(a.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq) {
    for (uint32_t i = 0; i < nap; i++) __builtin_amdgcn_s_sleep(2);
    if (nap < 8) nap <<= 1;
    if (a.err && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
      if (a.err) __hip_atomic_store(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}

template <class Op, int U, int POL>
__device__ __forceinline__ void prog_unit_of(const PlanDesc &d, TableInputs raw, uint64_t lt, int tid,
                                             const uint32_t (&voff)[U]) {
  constexpr uint64_t TILE = (uint64_t)kProgBlock * U;
  if (lt == 0) scalar_part<Op, POL>(d.out, raw, d.n, d.head, d.npkt, d.tail, tid);
  const uint64_t pkt0 = lt * TILE;
  if (pkt0 >= d.npkt) return;
  const uint64_t shift = (uint64_t)d.head * Op::kEsz;
  Shifted<TableInputs> in{raw, shift};
  const uint64_t left = d.npkt - pkt0;
  const uint32_t tile_bytes = (uint32_t)((left < TILE ? left : TILE) * kPacket);
  tile_body<Op, U, POL>(d.out + shift, in, d.n, pkt0 * kPacket, tile_bytes, voff);
}

// A unit under its compute's peer policy (the plan's hiccl_reduce_plan_set_peer
// flags, kept in the descriptor: bit 0 stores, bit 1 loads; workgroup-uniform).
template <class Op, int U>
__device__ __forceinline__ void prog_unit_peer(uint32_t peer, const PlanDesc &d, TableInputs raw, uint64_t lt,
                                               int tid, const uint32_t (&voff)[U]) {
  constexpr int L = kProgPol % 10, S = kProgPol / 10;
  switch (peer & 3u) {
    case 0: prog_unit_of<Op, U, kProgPol>(d, raw, lt, tid, voff); break;
    case 1: prog_unit_of<Op, U, 10 * kPolStoreSys + L>(d, raw, lt, tid, voff); break;
    case 2: prog_unit_of<Op, U, 10 * S + kPolLoadSys>(d, raw, lt, tid, voff); break;
    default: prog_unit_of<Op, U, 10 * kPolStoreSys + kPolLoadSys>(d, raw, lt, tid, voff); break;
  }
}

template <class Op, int U>
__global__ __launch_bounds__(kProgBlock) void k_program(ProgArgs a) {
  const int tid = threadIdx.x;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (uint32_t)((u * kProgBlock + tid) * kPacket);
  if (a.nphase) {
    const uint32_t add = a.epoch_dev ? __hip_atomic_load(a.epoch_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const uint64_t seq = a.seq + add;
    if (blockIdx.x == 0) {
      if (tid < 64) {
        prog_phases(a, a.nphase, (uint32_t)tid, add);
        if (tid == 0) {
          if (a.light)
            __hip_atomic_store(a.gate, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else
            __hip_atomic_store(a.gate, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    } else if (tid == 0) {
      prog_gate_wait(a, seq);
      // Fenced mode: an agent-scope acquire closes the relaxed gate polls,
      // pairing with workgroup 0's agent-scope release store of the gate,
      // which follows workgroup 0's system-scope acquire of the peers'
      // tokens.  That orders this workgroup after the tokens for writes made
      // on THIS GPU.  It is not a guarantee for a peer GPU's writes: on a
      // part with several XCDs workgroup 0's system-scope acquire
      // invalidates only its own XCD's L2, and an agent-scope acquire on
      // another XCD does not drop non-coherent L2 lines there.  Peer data
      // stays visible because no L2 holds a line of it (peer puts store
      // write-through, HICCL_PEER_STORES; fused reads load system-scope,
      // HICCL_PEER_LOADS; and the kernel-start invalidate) -- the same
      // cache argument `light` rests on, and unconfirmed until a run with
      // one GPU per rank.  Agent scope, not system: a system-scope acquire
      // per workgroup (1,024 L2 invalidations per launch) cost ~8 us per
      // C5 step (profiles/r04f_progstep.jsonl).  The workgroup barrier
      // below carries it to the other lanes.
      if (!a.light) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
  for (uint64_t t = blockIdx.x; t < a.nunits; t += gridDim.x) {
    const uint32_t c = a.unit_comp ? ((ConstU32 *)a.unit_comp)[t] : 0u;
    const ConstDesc *q = (const ConstDesc *)a.desc + c;
    const PlanDesc d = load_desc(a.desc, c);
    const uint32_t flags = q->pad;  // bit 0: exact byte copy; bits 1-2: peer stores / peer loads
    TableInputs raw{a.ptrs + (uint64_t)c * a.stride};
    if (flags & 1u)
      prog_unit_peer<OpRaw, U>(flags >> 1, d, raw, t - d.tile_begin, tid, voff);
    else
      prog_unit_peer<Op, U>(flags >> 1, d, raw, t - d.tile_begin, tid, voff);
  }
}

// ------------------------------------------------------------ host side ----

// Token protocol of programs and of k_sigwait_phases (hiccl_token_mode).
// Default FENCED: release token stores, relaxed polls then an acquire
// fence per phase, a release gate store and an agent-scope acquire after
// each workgroup's gate polls -- the memory model's own guarantee.
// HICCL_PROG_FENCES=light: relaxed stores and polls, no fences (prog_phases'
// argument rests on kernel-boundary cache behaviour that only a run with one
// GPU per rank can confirm, so it is opt-in until one has).  Read at every
// launch (a capture keeps the value it was recorded with).
bool prog_light() {
  const char *e = std::getenv("HICCL_PROG_FENCES");
  return e && std::string(e) == "light";
}

struct DevInfo {
  int cus = 0;
};

std::mutex g_dev_mu;
DevInfo g_dev[64];

// hiccl_reduce_auto_choice: the CU count AUTO plans for, in place of a device's
thread_local int t_cus_override = 0;

int device_cus(int dev) {
  if (t_cus_override > 0) return t_cus_override;
  if (dev < 0 || dev >= 64) return 256;
  std::lock_guard<std::mutex> lk(g_dev_mu);
  if (g_dev[dev].cus == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    g_dev[dev].cus = cus;
  }
  return g_dev[dev].cus;
}

// Dynamic-scheduling counter pairs, one per (device, stream), allocated on
// first use (64 B apart) and zeroed once; the kernels leave them zero.
struct SchedKey {
  int dev;
  hipStream_t s;
  bool operator<(const SchedKey &o) const { return dev != o.dev ? dev < o.dev : s < o.s; }
};
std::mutex g_sched_mu;
std::map<SchedKey, uint32_t *> g_sched;

// Tickets per workgroup below which a dynamic schedule does not pay off
// (C4 at 16 / 64 MiB per input: 4 / 16 tickets per workgroup lose 33 / 14 %
// to the per-ticket barrier; 64 tickets at 256 MiB gain 3 %).
constexpr uint64_t kDynMinUnitsPerWG = 32;
// AUTO schedules dynamically from this many inputs on (TILE engine).
constexpr double kDynMinInputs = 5;
// A ticket should cover at least this many 16 KiB input tiles of traffic
// ((n + 1) per tile): one tile at n >= 8, two at n = 4..7, ... -- a ticket
// costs an atomic and a workgroup barrier (profiles/r01_schedsweep*.jsonl).
constexpr double kTicketTiles = 9;
// AUTO takes the tile engine (n >= kDynMinInputs) from this many tickets per
// workgroup on: below it the phased engine is ahead.
constexpr uint64_t kTileMinTicketsPerWG = 64;

// Wide tiles (TILE, 256 lanes x 8 packets = 32 KiB per input) on the
// dynamic schedule for few inputs (2..4) and large buckets: 32 packets per
// lane in flight over the n inputs at once.  From 128 tickets per workgroup
// (1 GiB per input) they lead the phased engine by 2-8 % (n = 2 / 3 / 4 at
// 1-4 GiB per input: 6.34-6.47 / 6.26-6.60 / 6.17-6.51 vs 5.77-6.25 TB/s);
// at 512 MiB they tie, at 256 MiB they lose (profiles/r02f_widetile_sweep.jsonl,
// r02f_widedyn_sweep.jsonl).  f32 and bf16 (native accumulation) only.
constexpr int kWideUnroll = 8;
constexpr uint64_t kWideMinTicketsPerWG = 128;

// Units per ticket of the dynamic schedule: one 128 KiB phased chunk or one
// wide tile; for 16 KiB tiles enough to cover kTicketTiles tile-loads.
uint32_t default_grab(int engine, double n, int unroll = 4 /* kDefUnroll */) {
  if (engine == HICCL_ENGINE_PHASE || unroll >= kWideUnroll) return 1u;
  const double g = kTicketTiles / (n + 1.0);
  return g <= 1.0 ? 1u : (uint32_t)(g + 0.999);
}

// Is `s` being captured into a graph?  `if_unknown` is the answer when the
// runtime cannot tell.
bool capturing(hipStream_t s, bool if_unknown) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess) {
    (void)hipGetLastError();
    return if_unknown;
  }
  return cap != hipStreamCaptureStatusNone;
}

// hipStreamPerThread is one handle value for a different stream on every
// host thread: two threads could run kernels on one counter at once (units
// skipped, wrong sums), so it takes the static schedule.  The null stream is
// the legacy stream here (this library is built without per-thread default
// streams): launches on it serialise, one counter is safe.
bool per_thread_stream(hipStream_t s) { return s == hipStreamPerThread; }

// The counter pair for a launch of `units` work units (n inputs, packet-
// weighted mean for a plan) on `grid` workgroups on (dev, s), or NULL for a
// static schedule: AUTO is dynamic for the TILE engine from kDynMinInputs
// inputs or with wide tiles (with the static grid-stride each workgroup is
// bound to the same addresses mod grid x 16 KiB, i.e. to a fixed subset of
// DRAM channels, and the ones on slow channels straggle: 5.6-5.7 vs
// 6.3-6.7 TB/s on C2); never during stream capture (a replayed graph could
// run beside other work on the same stream's counter) nor on
// hipStreamPerThread; NULL also on any allocation failure.
// The schedule rule itself (stream aside).
bool wants_dynamic(int engine, double n, uint64_t units, uint64_t grid, int schedule, uint32_t grab, int unroll) {
  if (schedule == HICCL_SCHED_STATIC) return false;
  if (schedule == HICCL_SCHED_AUTO && (engine != HICCL_ENGINE_TILE || (n < kDynMinInputs && unroll < kWideUnroll)))
    return false;
  if (!grab) grab = default_grab(engine, n, unroll);
  return (units + grab - 1) / grab >= kDynMinUnitsPerWG * grid;
}

uint32_t *unit_sched_for(int engine, double n, uint64_t units, uint64_t grid, int dev, hipStream_t s,
                         int schedule = HICCL_SCHED_AUTO, uint32_t grab = 0, int unroll = 4 /* kDefUnroll */) {
  if (!wants_dynamic(engine, n, units, grid, schedule, grab, unroll)) return nullptr;
  if (per_thread_stream(s) || capturing(s, true)) return nullptr;
  std::lock_guard<std::mutex> lk(g_sched_mu);
  auto it = g_sched.find(SchedKey{dev, s});
  if (it != g_sched.end()) return it->second;
  uint32_t *p = nullptr;
  if (hipMalloc((void **)&p, 64) != hipSuccess) return nullptr;
  // zeroed in order on `s` (a null-stream memset does not order a
  // non-blocking stream's first kernel after it)
  if (hipMemsetAsync(p, 0, 64, s) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  g_sched[SchedKey{dev, s}] = p;
  return p;
}

int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) d = 0;
  return d;
}

size_t esize(int dtype) {
  switch (dtype) {
    case HICCL_FLOAT32: return 4;
    case HICCL_FLOAT64: return 8;
    case HICCL_BFLOAT16: return 2;
    case HICCL_UINT64: return 8;
    case HICCL_INT32: return 4;
    case HICCL_BYTES: return 1;
    default: return 0;
  }
}

struct Split {
  uint32_t head, tail;
  uint64_t npkt;
};

// [head | npkt packets | tail] with the packets 16-B aligned on `out`.
Split split_on(const void *out, size_t count, size_t esz) {
  const size_t V = kPacket / esz;
  const uintptr_t mis = (uintptr_t)out % kPacket;
  size_t head = mis ? (kPacket - mis) / esz : 0;
  if (head > count) head = count;
  Split s;
  s.head = (uint32_t)head;
  s.npkt = (count - head) / V;
  s.tail = (uint32_t)(count - head - s.npkt * V);
  return s;
}

// Validate pointers: element alignment, no partial overlap with the output.
int check_buffers(void *out, const void *const *in, int n, size_t count, size_t esz) {
  if (!out) return fail(hipErrorInvalidValue, "hiccl_reduce: out is NULL");
  if ((uintptr_t)out % esz)
    return fail(hipErrorInvalidValue, "hiccl_reduce: out is not element-aligned");
  if (n < 0) return fail(hipErrorInvalidValue, "hiccl_reduce: n < 0");
  if (n > 0 && !in) return fail(hipErrorInvalidValue, "hiccl_reduce: in is NULL");
  const uintptr_t o0 = (uintptr_t)out, o1 = o0 + count * esz;
  for (int k = 0; k < n; k++) {
    const uintptr_t p = (uintptr_t)in[k];
    if (!p) return fail(hipErrorInvalidValue, "hiccl_reduce: in[" + std::to_string(k) + "] is NULL");
    if (p % esz)
      return fail(hipErrorInvalidValue,
                  "hiccl_reduce: in[" + std::to_string(k) + "] is not element-aligned");
    const uintptr_t p1 = p + count * esz;
    if (p != o0 && p < o1 && o0 < p1)
      return fail(hipErrorInvalidValue, "hiccl_reduce: in[" + std::to_string(k) +
                                            "] partially overlaps out (only exact aliasing is allowed)");
  }
  return 0;
}

// Engine shapes, chosen from on-device sweeps:
//  tile   256 lanes x 4 packets (16 KiB per input per tile), for computes too
//         small to give every CU several phased chunks;
//  phase  512 lanes x P packets (P = 16, or 8 where the accumulator of a
//         packet takes 8 VGPRs -- bf16 WIDE -- or the adds get reassociated:
//         int32) -- 128 KiB per input per chunk (64 KiB at P = 8).
// Both: nt loads and nt stores, one workgroup per CU, grid-stride.
constexpr int kDefBlock = 256;
constexpr int kDefUnroll = 4;
static_assert(kDefUnroll == 4, "default_grab / unit_sched_for default their unroll to 4");
constexpr int kDefPol = 11;  // nt loads, nt stores
// A launch that writes at most this many bytes stores write-through (system
// scope, sc0 sc1) unless its config names a store form: see plan_store_peer.
// Copies (one input) up to 32 MiB; reductions (two or more inputs per
// output, packet-weighted for a plan) up to 256 MiB.
constexpr uint64_t kWtMaxBytes = 32ull << 20;
constexpr uint64_t kWtMaxBytesReduce = 256ull << 20;
inline uint64_t wt_cap(double n) { return n >= 1.5 ? kWtMaxBytesReduce : kWtMaxBytes; }
constexpr int kDefBpc = 1;
constexpr int kSmallBpc = 4;
constexpr int kPhBlock = 512;
// auto engine: with >= 5 inputs the TILE engine on the dynamic schedule;
// with fewer, PHASE (static) when every CU gets a chunk, else TILE
// (profiles/r01_schedsweep*.jsonl, r01_crossover.jsonl).
constexpr uint64_t kPhaseMinChunksPerCU = 1;

// P of the phased engine: 16 packets per lane (acc + two in-flight loads =
// 3 x 64 VGPRs at 512 lanes) unless the accumulator is wider than a packet
// (bf16: f32x8) or the compiler reassociates the adds and holds more
// registers (int32: exact, so it may) -- then 8.
template <class Op>
constexpr int phase_p() {
  return (sizeof(typename Op::acc_t) > 16 || std::is_same<Op, OpI32>::value) ? 8 : 16;
}

int phase_p_dtype(int dtype, int acc) {
  if (dtype == HICCL_BFLOAT16) return acc == HICCL_ACC_WIDE ? 8 : 16;
  return dtype == HICCL_INT32 ? 8 : 16;
}

struct Cfg {
  int block, unroll, bpc, nt, acc, grid, store, engine, schedule, grab, drain;
  bool store_auto;  // store_policy 0: the store form follows the launch's size (wt_cap)
  bool wt;          // the launch stores write-through by size: decided BEFORE the engine
                    // (oneshot_cfg, plan_cfg), since AUTO's engine rules differ under it
  int order;        // tile-order segments (hiccl_reduce_config_t.order; 0/1 linear)
};

// Raw config: zero block/unroll stay zero until the engine is known.
Cfg resolve(const hiccl_reduce_config_t *c) {
  Cfg r{0, 0, 0, kDefPol % 10, HICCL_ACC_NATIVE, 0, kDefPol / 10, HICCL_ENGINE_AUTO, HICCL_SCHED_AUTO, 0, 0, true,
        false, 0};
  if (c) {
    r.block = c->block;
    r.unroll = c->unroll;
    if (c->blocks_per_cu) r.bpc = c->blocks_per_cu;
    if (c->nontemporal) r.nt = c->nontemporal - 1;
    r.acc = c->acc;
    r.grid = c->grid;
    if (c->store_policy) r.store = c->store_policy - 1;
    r.store_auto = c->store_policy == 0;
    r.engine = c->engine;
    r.schedule = c->schedule;
    r.grab = c->grab;
    r.drain = c->drain;
    r.order = c->order;
  }
  return r;
}

// Wide tiles for this launch: the unroll (16 for two inputs, 8 for three or
// four: n = 2 at 1-2 GiB per input 6.50-6.66 vs 6.33-6.46 TB/s at 8; n = 3 / 4
// lead at 8, profiles/r02g_wideverify.jsonl), or 0.  f32 / bf16 native only,
// from kWideMinTicketsPerWG 8-packet tiles per workgroup (1 GiB per input).
// Wide tiles exist only at block 256 with nt loads and nt stores (pick_u):
// a caller that asks for another block or cache policy keeps the u4 / PHASE
// choice instead of an unsupported shape.
int auto_wide_unroll(uint64_t npkt, double n, int dtype, const Cfg &c, int dev) {
  const bool tuned = dtype == HICCL_FLOAT32 || (dtype == HICCL_BFLOAT16 && c.acc == HICCL_ACC_NATIVE);
  if (!tuned || n < 1.5 || n >= kDynMinInputs) return 0;
  if ((c.block && c.block != kDefBlock) || c.nt != kDefPol % 10 || c.store != kDefPol / 10) return 0;
  if (npkt / ((uint64_t)kDefBlock * kWideUnroll) < kWideMinTicketsPerWG * (uint64_t)device_cus(dev)) return 0;
  return n < 2.5 ? 2 * kWideUnroll : kWideUnroll;
}

// Auto engine from the packets per input of a launch (summed over its
// computes) and the number of inputs (packet-weighted mean for a plan).
// Interleaved engine x schedule sweeps, n = 5 / 8 / 16 x 32 MiB-1 GiB per
// input (profiles/r01g_xover.jsonl; bf16: r01g_bf16_crossover.jsonl): the
// tile engine on the dynamic schedule leads from 64 tickets per workgroup
// (n = 8, 1 GiB: 6.71 vs 6.32 TB/s phased), the phased engine below it
// (n = 8, 128 MiB = 32 tickets: 6.41 vs 5.94); with <= 4 inputs the phased
// engine leads at every size with a chunk per CU (r01_schedsweep.jsonl) --
// except from 1 GiB per input, where wide tiles lead (auto_wide_unroll).
int auto_engine(uint64_t npkt, double n, int dtype, const Cfg &c, int dev) {
  const int acc = c.acc;
  if (auto_wide_unroll(npkt, n, dtype, c, dev)) return HICCL_ENGINE_TILE;
  const bool packed_ok = !(dtype == HICCL_BFLOAT16 && acc == HICCL_ACC_WIDE);
  // Round 5: a launch that stores write-through (store form left to size, at
  // most wt_cap written; f32, bf16) runs faster on the phased engine wherever the
  // dynamic tiles would otherwise take it -- 256 MiB per input, n = 8 / 16 /
  // 32 / 64: 6.49 / 6.45 / 6.71 / 6.59 vs 6.37-6.40 TB/s interleaved
  // (profiles/r05ab_c3_engines_many.jsonl; n = 8 on another box 6.50 vs
  // 6.42, r05v_c3_engines.jsonl), config 4's 256 MiB plan 6.60 vs 6.44
  // (r05aa_c4_engines.jsonl; bf16 6.62 vs 6.33, r05ad_c4_engines_bf16.jsonl);
  // at 1 GiB (nt) the tiles keep their lead.  `c.wt` is the store form the
  // launch actually takes (by size, where a write-through kernel exists).
  const bool wt = c.wt;
  const bool wt_f32 = wt && dtype == HICCL_FLOAT32;
  const bool wt_many = wt && (dtype == HICCL_FLOAT32 || (dtype == HICCL_BFLOAT16 && acc == HICCL_ACC_NATIVE));
  if (n >= kDynMinInputs && packed_ok && !wt_many) {
    const uint64_t tickets = npkt / ((uint64_t)kDefBlock * kDefUnroll) / default_grab(HICCL_ENGINE_TILE, n);
    if (tickets >= kTileMinTicketsPerWG * (uint64_t)device_cus(dev)) return HICCL_ENGINE_TILE;
  }
  const uint64_t chunk = (uint64_t)kPhBlock * phase_p_dtype(dtype, acc);
  const uint64_t cus = (uint64_t)device_cus(dev);
  const uint64_t per_cu = npkt / (cus * chunk);  // phased chunks per CU
  // Round 3, on the round-2 kernels (interleaved one-shot sweeps of n = 2 /
  // 3 / 4 / 8 at 1-4.5 chunks per CU: f32 profiles/r03n_midsize.jsonl, bf16
  // r03o_midsize_bf16.jsonl, f64 r03x_midsize_f64.jsonl, int32 and bf16 with
  // the f32 accumulator -- 64 KiB chunks -- r03ze_midsize_i32.jsonl /
  // r03ze_midsize_bf16wide.jsonl; the C5 step shape scaled up,
  // r03n_stepscale.jsonl): the phased engine needs both several chunks per
  // CU and whole rounds of them -- one chunk per workgroup (a CU per
  // workgroup) is a single memory round trip with no overlap, and a last
  // round that only part of the grid works on (1.25 / 1.5 / 2.5 chunks per
  // CU) idles the rest: PHASE lost 3-20 % to static tiles there (f32 n = 3
  // at 40 MiB: 5.08 vs 6.15 TB/s; the C5 step at 8 x 2^18: 29.6 vs 23.2
  // us).  `round_eff` = chunks / (whole rounds x CUs).
  const bool big_chunk = chunk >= 8192;  // 128 KiB per input (P = 16)
  const uint64_t chunks = (npkt + chunk - 1) / chunk;
  const double round_eff = chunks ? (double)chunks / (double)(((chunks + cus - 1) / cus) * cus) : 0.0;
  if (n < 2.5) return per_cu > 16 && round_eff >= 0.89 ? HICCL_ENGINE_PHASE : HICCL_ENGINE_TILE;
  // Round 5: with the write-through stores a launch of this size takes
  // (store form left to size, at most wt_cap written; f32), static tiles lead
  // the phased engine at three inputs: 6.80 vs 6.62 TB/s interleaved at
  // 3 x 256 MiB (profiles/r05v_c3_engines.jsonl; 6.86 vs 6.63 on another
  // box, r05r_nway.jsonl); at two and four inputs the nt table holds.
  if (n >= 2.5 && n < 3.5 && wt_f32) return HICCL_ENGINE_TILE;
  if (n < kDynMinInputs) return per_cu >= 4 && round_eff >= 0.89 ? HICCL_ENGINE_PHASE : HICCL_ENGINE_TILE;
  // many inputs, under the dynamic tiles' ticket count: PHASE from one
  // whole chunk per CU unless too much of the last round idles (f32 n = 8 at
  // 40 MiB, 1.25 per CU: tiles 6.03 vs 5.45; at 48 / 80 MiB PHASE holds:
  // 6.08 / 6.25; with 64 KiB chunks PHASE needs 80 %: int32 / bf16-wide n =
  // 8 at 1.5 per CU: tiles 5.84 / 5.94 vs 5.58 / 5.68); from 16 inputs a
  // 128 KiB chunk is >= 2 MiB of reads, and PHASE leads already with 70 %
  // of the CUs holding one (24 MiB per input, 0.75 chunks per CU: n = 16 /
  // 32 PHASE 6.56 / 6.34 vs tiles 6.15-6.25; at 0.5 per CU tiles lead:
  // 6.21 / 6.25 vs 5.43 / 5.61; profiles/r03q_sweep_manyn.jsonl)
  const bool enough = per_cu >= 1 || (n >= 16 && big_chunk);
  return enough && round_eff >= (big_chunk ? 0.7 : 0.8) ? HICCL_ENGINE_PHASE : HICCL_ENGINE_TILE;
}

// Workgroups per CU: a tile launch too small for a phased chunk per CU has
// few tiles per workgroup and is latency-bound -- four workgroups per CU
// keep more of it in flight (n = 8, 16 MiB per input: 6.31 vs 6.01 TB/s,
// 32 MiB: 6.27-6.40 vs 5.97-6.13; profiles/r01g_small_sweep.jsonl).
int auto_bpc(int engine, uint64_t npkt, int dtype, int acc, int dev) {
  const uint64_t chunk = (uint64_t)kPhBlock * phase_p_dtype(dtype, acc);
  return engine == HICCL_ENGINE_TILE && npkt < kPhaseMinChunksPerCU * (uint64_t)device_cus(dev) * chunk
             ? kSmallBpc
             : kDefBpc;
}

// Packets per lane of the TILE engine: a launch with fewer than two 16 KiB
// tiles per CU is pure latency (one round trip per workgroup) -- half-size
// tiles on twice the workgroups finish it sooner (the C5 step, four n = 2
// and one n = 4 computes of 2^18 f32: 4.75 vs 5.32 us queued,
// profiles/r02c_plan_sweep.jsonl); 2 exists for the headline types only.
int auto_unroll(uint64_t npkt, int dtype, int acc, int dev) {
  const bool tuned = dtype == HICCL_FLOAT32 || (dtype == HICCL_BFLOAT16 && acc == HICCL_ACC_NATIVE);
  return tuned && npkt < 2ull * device_cus(dev) * kDefBlock * kDefUnroll ? 2 : kDefUnroll;
}

// Fill in the engine and its default shape (n: inputs, or a plan's
// packet-weighted mean).
void finish_cfg(Cfg &c, uint64_t npkt, double n, int dtype, int dev) {
  if (c.engine == HICCL_ENGINE_AUTO)
    c.engine = (c.block || c.unroll) ? HICCL_ENGINE_TILE : auto_engine(npkt, n, dtype, c, dev);
  if (c.engine == HICCL_ENGINE_PHASE) {
    if (!c.block) c.block = kPhBlock;
    if (!c.unroll) c.unroll = phase_p_dtype(dtype, c.acc);
  } else {
    if (!c.block) c.block = kDefBlock;
    if (!c.unroll) {
      const int wide = auto_wide_unroll(npkt, n, dtype, c, dev);
      c.unroll = wide ? wide : auto_unroll(npkt, dtype, c.acc, dev);
    }
  }
  if (!c.bpc) c.bpc = auto_bpc(c.engine, npkt, dtype, c.acc, dev);
}

// ---- single-compute dispatch (template instantiation table)

typedef void (*single_fn)(SingleArgs, dim3, hipStream_t);

template <class Op, int B, int U, int POL, int ENG = kTile>
void launch_single_t(SingleArgs a, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((k_reduce_single<Op, B, U, POL, ENG>), grid, dim3(B), 0, s, a);
}

template <class Op, int B, int U>
single_fn pick_nt(int pol) {
  switch (pol) {
    case 0: return launch_single_t<Op, B, U, 0>;
    case 1: return launch_single_t<Op, B, U, 1>;
    case 10: return launch_single_t<Op, B, U, 10>;
    case 11: return launch_single_t<Op, B, U, 11>;
    case 20: return launch_single_t<Op, B, U, 20>;
    case 21: return launch_single_t<Op, B, U, 21>;
    case 10 * kPolStoreSys + 1: return launch_single_t<Op, B, U, 10 * kPolStoreSys + 1>;
    default: return nullptr;
  }
}

template <class Op, int B>
single_fn pick_u(int u, int pol) {
  switch (u) {
    case 1: return pick_nt<Op, B, 1>(pol);
    case 2: return pick_nt<Op, B, 2>(pol);
    case 4: return pick_nt<Op, B, 4>(pol);
    // wide tiles for few inputs (32 packets per lane in flight at n = 4 / 2)
    case 8: return pol == kDefPol && B == 256 ? launch_single_t<Op, B, 8, kDefPol> : nullptr;
    case 16: return pol == kDefPol && B == 256 ? launch_single_t<Op, B, 16, kDefPol> : nullptr;
    default: return nullptr;
  }
}

// Phased engine: the default shape for every type; the headline types also
// get the sweep shapes (chunk 64-128 KiB) and cache-policy variants.
template <class Op, bool TUNED>
single_fn pick_phase(const Cfg &c) {
  constexpr int PD = phase_p<Op>();
  const int pol = c.store * 10 + c.nt;
  if (c.block == kPhBlock && c.unroll == PD) {
    switch (pol) {
      case 11: return launch_single_t<Op, kPhBlock, PD, 11, kPhase>;
      case 10 * kPolStoreSys + 1: return launch_single_t<Op, kPhBlock, PD, 10 * kPolStoreSys + 1, kPhase>;
      case 1: if constexpr (TUNED) return launch_single_t<Op, kPhBlock, PD, 1, kPhase>; break;
      case 10: if constexpr (TUNED) return launch_single_t<Op, kPhBlock, PD, 10, kPhase>; break;
      case 21: if constexpr (TUNED) return launch_single_t<Op, kPhBlock, PD, 21, kPhase>; break;
      case 0: if constexpr (TUNED) return launch_single_t<Op, kPhBlock, PD, 0, kPhase>; break;
      default: break;
    }
    return nullptr;
  }
  if constexpr (TUNED) {
    if (pol != kDefPol) return nullptr;
    if (c.block == 1024 && c.unroll == 4) return launch_single_t<Op, 1024, 4, 11, kPhase>;
    if constexpr (PD == 16) {
      if (c.block == 512 && c.unroll == 8) return launch_single_t<Op, 512, 8, 11, kPhase>;
      if (c.block == 1024 && c.unroll == 8) return launch_single_t<Op, 1024, 8, 11, kPhase>;
      if (c.block == 256 && c.unroll == 16) return launch_single_t<Op, 256, 16, 11, kPhase>;
    } else {
      if (c.block == 512 && c.unroll == 4) return launch_single_t<Op, 512, 4, 11, kPhase>;
    }
  }
  return nullptr;
}

// Full tuning table for the headline types; default shape for the rest.
template <class Op, bool TUNED>
single_fn pick_single(const Cfg &c) {
  if (c.engine == HICCL_ENGINE_PHASE) return pick_phase<Op, TUNED>(c);
  const int pol = c.store * 10 + c.nt;
  if constexpr (TUNED) {
    if (c.block == 256) return pick_u<Op, 256>(c.unroll, pol);
    if (c.block == 512) return pick_u<Op, 512>(c.unroll, pol);
    return nullptr;
  } else {
    if (c.block != kDefBlock || c.unroll != kDefUnroll) return nullptr;
    if (pol == 10 * kPolStoreSys + 1) return launch_single_t<Op, kDefBlock, kDefUnroll, 10 * kPolStoreSys + 1>;
    return pol == kDefPol ? launch_single_t<Op, kDefBlock, kDefUnroll, kDefPol> : nullptr;
  }
}

single_fn pick_single_dtype(int dtype, const Cfg &c) {
  switch (dtype) {
    case HICCL_FLOAT32: return pick_single<OpF32, true>(c);
    case HICCL_BFLOAT16:
      return c.acc == HICCL_ACC_WIDE ? pick_single<OpBF16Wide, false>(c)
                                     : pick_single<OpBF16, true>(c);
    case HICCL_FLOAT64: return pick_single<OpF64, false>(c);
    case HICCL_UINT64: return pick_single<OpU64, false>(c);
    case HICCL_INT32: return pick_single<OpI32, false>(c);
    case HICCL_BYTES: return pick_single<OpRaw, false>(c);
    default: return nullptr;
  }
}

// ---- plan dispatch
//
// Plan kernels (and one-shot calls with > 64 inputs, which run as a
// one-compute plan) come in the PHASE engine's default shape and the TILE
// engine at 256 lanes x U packets, U = 4 for every type and also 1 or 2 for
// the headline types (f32, bf16 native).  Cache policy: nt loads and stores.

constexpr int kPlanBlock = kDefBlock;
static_assert(kPlanBlock == kDefBlock, "plan_cfg shapes plans with finish_cfg");

// Packets per work unit (tile or chunk) of a plan kernel.
uint64_t unit_pkts(int engine, int dtype, int acc, int unroll) {
  return engine == HICCL_ENGINE_PHASE ? (uint64_t)kPhBlock * phase_p_dtype(dtype, acc)
                                      : (uint64_t)kPlanBlock * (unroll ? unroll : kDefUnroll);
}

typedef void (*plan_fn)(const PlanArgs &, dim3, hipStream_t);

template <class Op, int ENG, int U, int POL = kDefPol>
void launch_plan_t(const PlanArgs &a, dim3 grid, hipStream_t s) {
  constexpr int B = ENG == kPhase ? kPhBlock : kPlanBlock;
  hipLaunchKernelGGL((k_reduce_plan<Op, B, U, POL, ENG>), grid, dim3(B), 0, s, a);
}

// The plan kernels' cache policy: nt loads and stores, or a plan's peer
// policy (hiccl_reduce_plan_set_peer: system-scope stores and/or loads) --
// those in the PHASE engine's default shape and TILE at U = 4 (and 2 for the
// headline types: a pipeline step's small batches).
int plan_pol(int peer) {
  return 10 * ((peer & HICCL_PEER_STORES) ? kPolStoreSys : kDefPol / 10) +
         ((peer & HICCL_PEER_LOADS) ? kPolLoadSys : kDefPol % 10);
}

template <class Op, bool TUNED, int POL>
plan_fn pick_plan_pol(int engine, int unroll) {
  constexpr bool DEF = POL == kDefPol;
  if (engine == HICCL_ENGINE_PHASE) return launch_plan_t<Op, kPhase, phase_p<Op>(), POL>;
  switch (unroll) {
    case 0:
    case 4: return launch_plan_t<Op, kTile, 4, POL>;
    case 2: if constexpr (TUNED) return launch_plan_t<Op, kTile, 2, POL>; break;
    case 8: if constexpr (TUNED && DEF) return launch_plan_t<Op, kTile, 8>; break;
    case 16: if constexpr (TUNED && DEF) return launch_plan_t<Op, kTile, 16>; break;
    case 1: if constexpr (TUNED && DEF) return launch_plan_t<Op, kTile, 1>; break;
    default: break;
  }
  return nullptr;
}

template <class Op, bool TUNED>
plan_fn pick_plan_eng(int engine, int unroll, int pol) {
  constexpr int L = kDefPol % 10, S = kDefPol / 10;
  switch (pol) {
    case kDefPol: return pick_plan_pol<Op, TUNED, kDefPol>(engine, unroll);
    case 10 * kPolStoreSys + L: return pick_plan_pol<Op, TUNED, 10 * kPolStoreSys + L>(engine, unroll);
    case 10 * S + kPolLoadSys: return pick_plan_pol<Op, TUNED, 10 * S + kPolLoadSys>(engine, unroll);
    case 10 * kPolStoreSys + kPolLoadSys:
      return pick_plan_pol<Op, TUNED, 10 * kPolStoreSys + kPolLoadSys>(engine, unroll);
    default: return nullptr;
  }
}

plan_fn pick_plan(int dtype, int acc, int engine, int unroll, int pol = kDefPol) {
  switch (dtype) {
    case HICCL_FLOAT32: return pick_plan_eng<OpF32, true>(engine, unroll, pol);
    case HICCL_BFLOAT16:
      return acc == HICCL_ACC_WIDE ? pick_plan_eng<OpBF16Wide, false>(engine, unroll, pol)
                                   : pick_plan_eng<OpBF16, true>(engine, unroll, pol);
    case HICCL_FLOAT64: return pick_plan_eng<OpF64, false>(engine, unroll, pol);
    case HICCL_UINT64: return pick_plan_eng<OpU64, false>(engine, unroll, pol);
    case HICCL_INT32: return pick_plan_eng<OpI32, false>(engine, unroll, pol);
    case HICCL_BYTES: return pick_plan_eng<OpRaw, false>(engine, unroll, pol);
    default: return nullptr;
  }
}

// Is `c` (engine resolved, shape filled in by finish_cfg) a shape the plan
// kernels have?  Empty string if so, else why not.
std::string plan_shape_error(const Cfg &c, int dtype) {
  if (c.nt != kDefPol % 10 || (c.store != kDefPol / 10 && c.store != kPolStoreSys))
    return "plan kernels load nt (nontemporal 2) and store nt (store_policy 2), system-scope write-through "
           "(store_policy 4) or either by the launch's size (store_policy 0)";
  if (c.drain) return "plan kernels do not support drain";
  if (c.order != 0 && c.order != 1) return "plan kernels run their units in linear order (order 0)";
  if (c.engine == HICCL_ENGINE_PHASE) {
    if (c.block != kPhBlock || c.unroll != phase_p_dtype(dtype, c.acc))
      return "plan kernels run the PHASE engine in its default shape only (block 512, unroll " +
             std::to_string(phase_p_dtype(dtype, c.acc)) + ")";
    return "";
  }
  if (c.block != kPlanBlock) return "plan kernels run the TILE engine at block 256 only";
  if (c.store == kPolStoreSys) {
    if (!pick_plan(dtype, c.acc, HICCL_ENGINE_TILE, c.unroll, plan_pol(HICCL_PEER_STORES)))
      return "write-through plan kernels (store_policy 4) run the TILE engine at unroll 4 (f32 / bf16: 2 or 4) only";
    return "";
  }
  if (!pick_plan(dtype, c.acc, HICCL_ENGINE_TILE, c.unroll))
    return "plan kernels run the TILE engine at unroll 4 (f32 / bf16: 1, 2, 4, 8 or 16) only";
  return "";
}

// The one-shot call's configuration, engine and store form resolved.  The
// store form is decided first: write-through (system scope) by size -- at
// most wt_cap written -- when the config leaves it open, loads are nt (the
// only write-through kernels) and an explicit TILE unroll is 2 or 4 (the
// plan's rule, plan_store_peer: one rule for both), since AUTO's engine rules
// differ under it (auto_engine).  If the shape finish_cfg then picks lacks a
// write-through kernel, the call keeps nt stores and its engine is chosen
// again for them.  n > 64 inputs run on the plan kernel (reduce_via_table),
// whose kernels decide.  hiccl_reduce_ex and hiccl_reduce_auto_choice_ex
// share it.
Cfg oneshot_cfg(int dtype, const hiccl_reduce_config_t *cfg, uint64_t npkt, uint64_t out_bytes, double n,
                int dev) {
  const Cfg raw = resolve(cfg);
  Cfg c = raw;
  const bool u_ok = !raw.unroll || raw.unroll == 2 || raw.unroll == kDefUnroll || raw.engine == HICCL_ENGINE_PHASE;
  c.wt = raw.store_auto && raw.nt == kDefPol % 10 && u_ok && out_bytes <= wt_cap(dtype == HICCL_BYTES ? 1.0 : n);
  finish_cfg(c, npkt, n, dtype, dev);
  if (!c.wt) return c;
  Cfg w = c;
  w.store = kPolStoreSys;
  if (n > kMaxArgInputs ? pick_plan(dtype, w.acc, w.engine, w.unroll, plan_pol(HICCL_PEER_STORES)) != nullptr
                        : pick_single_dtype(dtype, w) != nullptr)
    return w;
  c = raw;
  finish_cfg(c, npkt, n, dtype, dev);
  return c;
}

// The enumerated fields of a one-shot config (before finish_cfg).
int check_cfg_fields(const Cfg &c, const std::string &who) {
  if (c.acc != HICCL_ACC_NATIVE && c.acc != HICCL_ACC_WIDE) return fail(hipErrorInvalidValue, who + ": bad acc mode");
  if (c.engine < HICCL_ENGINE_AUTO || c.engine > HICCL_ENGINE_PHASE)
    return fail(hipErrorInvalidValue, who + ": bad engine");
  if (c.schedule < HICCL_SCHED_AUTO || c.schedule > HICCL_SCHED_DYNAMIC)
    return fail(hipErrorInvalidValue, who + ": bad schedule");
  if (c.grab < 0 || c.grab > 4096) return fail(hipErrorInvalidValue, who + ": bad grab");
  if (c.order < 0 || c.order > 4096 || (c.order & (c.order - 1)))
    return fail(hipErrorInvalidValue, who + ": order must be 0 or a power of two <= 4096");
  return 0;
}

uint32_t log2u(int v) {
  uint32_t l = 0;
  while (v > 1) {
    v >>= 1;
    l++;
  }
  return l;
}

uint64_t tiles_for(uint64_t npkt, uint64_t tile) {
  uint64_t t = (npkt + tile - 1) / tile;
  return t ? t : 1;  // a compute with only scalars still owns one tile
}

// Large-n one-shot path: stage the pointer table in stream-ordered device
// memory and run it as a one-compute plan.
int reduce_via_table(int dtype, const Cfg &c, void *out, const void *const *in, int n, size_t count,
                     hipStream_t s);


}  // namespace

// ======================================================================
// C ABI
// ======================================================================

extern "C" {

size_t hiccl_dtype_size(int dtype) { return esize(dtype); }

const char *hiccl_last_error(void) { return g_last_error.c_str(); }

int hiccl_version(void) { return HICCL_VERSION_INT; }

int hiccl_reduce_ex(int dtype, void *out, const void *const *in, int n, size_t count,
                    void *stream, const hiccl_reduce_config_t *cfg) {
  const size_t esz = esize(dtype);
  if (!esz) return fail(hipErrorInvalidValue, "hiccl_reduce: unknown dtype " + std::to_string(dtype));
  if (count == 0) return 0;
  if (dtype == HICCL_BYTES && n != 1) return fail(hipErrorInvalidValue, "hiccl_reduce: HICCL_BYTES copies need n == 1");
  if (int e = check_buffers(out, in, n, count, esz)) return e;
  if (int e = check_cfg_fields(resolve(cfg), "hiccl_reduce")) return e;
  hipStream_t s = (hipStream_t)stream;
  const int dev = current_device();
  Split sp = split_on(out, count, esz);
  // engine, shape and store form (write-through by size, as a plan's:
  // plan_store_peer)
  Cfg c = oneshot_cfg(dtype, cfg, sp.npkt, (uint64_t)count * esz, n, dev);
  if (c.bpc < 1 || c.bpc > 64) return fail(hipErrorInvalidValue, "hiccl_reduce_ex: blocks_per_cu");
  if (c.grid < 0) return fail(hipErrorInvalidValue, "hiccl_reduce_ex: grid < 0");
  if (n > kMaxArgInputs) {
    const std::string why = plan_shape_error(c, dtype);
    if (!why.empty()) return fail(hipErrorInvalidValue, "hiccl_reduce_ex: n > 64 inputs run on the plan kernel: " + why);
    // the > 64-input pointer table is uploaded from host memory per call: a
    // captured graph would replay a copy from a freed host buffer
    if (capturing(s, false))
      return fail(hipErrorStreamCaptureUnsupported,
                  "hiccl_reduce: n > 64 inputs cannot be captured into a graph (use a plan)");
    return reduce_via_table(dtype, c, out, in, n, count, s);
  }

  single_fn fn = pick_single_dtype(dtype, c);
  if (!fn)
    return fail(hipErrorInvalidValue, "hiccl_reduce_ex: unsupported config (block " +
                                          std::to_string(c.block) + ", unroll " +
                                          std::to_string(c.unroll) + ", nt " +
                                          std::to_string(c.nt) + ", store " +
                                          std::to_string(c.store) + ", engine " +
                                          std::to_string(c.engine) + ") for this dtype");

  SingleArgs a;
  memset(&a, 0, sizeof(a));
  a.out = (char *)out;
  a.npkt = sp.npkt;
  a.head = sp.head;
  a.tail = sp.tail;
  a.n = (uint32_t)n;
  const uint64_t tile = (uint64_t)c.block * c.unroll;
  a.ntiles = tiles_for(sp.npkt, tile);
  for (int k = 0; k < n; k++) a.in[k] = (const char *)in[k];

  uint64_t grid = c.grid > 0 ? (uint64_t)c.grid : (uint64_t)device_cus(dev) * c.bpc;
  if (grid > a.ntiles) grid = a.ntiles;
  a.grab = c.grab > 0 ? (uint32_t)c.grab : default_grab(c.engine, n, c.unroll);
  a.drain = (uint32_t)c.drain;
  a.order = log2u(c.order);
  a.sched = unit_sched_for(c.engine, n, a.ntiles, grid, dev, s, c.schedule, a.grab, c.unroll);
  fn(a, dim3((unsigned)grid), s);
  return check_hip(hipGetLastError(), "hiccl_reduce: launch");
}

int hiccl_reduce(int dtype, void *out, const void *const *in, int n, size_t count, void *stream) {
  return hiccl_reduce_ex(dtype, out, in, n, count, stream, nullptr);
}

int hiccl_reduce_f32(float *out, const float *const *in, int n, size_t count, void *stream) {
  return hiccl_reduce_ex(HICCL_FLOAT32, out, (const void *const *)in, n, count, stream, nullptr);
}

int hiccl_reduce_bf16(uint16_t *out, const uint16_t *const *in, int n, size_t count,
                      void *stream) {
  return hiccl_reduce_ex(HICCL_BFLOAT16, out, (const void *const *)in, n, count, stream, nullptr);
}

int hiccl_reduce_auto_choice_ex(int dtype, const hiccl_reduce_config_t *cfg, size_t count, double n, int cus,
                                int *engine, int *unroll, int *blocks_per_cu, int *dynamic, int *store_policy) {
  const size_t esz = esize(dtype);
  if (!esz) return fail(hipErrorInvalidValue, "auto_choice: unknown dtype");
  if (cus <= 0 || n < 0) return fail(hipErrorInvalidValue, "auto_choice: cus must be > 0 and n >= 0");
  if (int e = check_cfg_fields(resolve(cfg), "auto_choice")) return e;
  struct CusOverride {  // no device query: the choice for `cus` CUs (reset on every exit)
    explicit CusOverride(int c) { t_cus_override = c; }
    ~CusOverride() { t_cus_override = 0; }
  } scoped(cus);
  const uint64_t npkt = (uint64_t)count * esz / kPacket;
  const Cfg c = oneshot_cfg(dtype, cfg, npkt, (uint64_t)count * esz, n, -1);
  // the same refusals as hiccl_reduce_ex: a shape no kernel has is an error
  const bool has = n > kMaxArgInputs ? plan_shape_error(c, dtype).empty() : pick_single_dtype(dtype, c) != nullptr;
  if (!has) return fail(hipErrorInvalidValue, "auto_choice: no kernel for this config and dtype");
  if (c.bpc < 1 || c.bpc > 64) return fail(hipErrorInvalidValue, "auto_choice: blocks_per_cu");
  if (c.grid < 0) return fail(hipErrorInvalidValue, "auto_choice: grid < 0");
  const uint64_t units = tiles_for(npkt, (uint64_t)c.block * c.unroll);  // tiles or phased chunks
  const uint64_t grid = std::min<uint64_t>(c.grid > 0 ? (uint64_t)c.grid : (uint64_t)cus * c.bpc, units);
  const bool dyn = wants_dynamic(c.engine, n, units, grid, c.schedule, (uint32_t)c.grab, c.unroll);
  if (engine) *engine = c.engine;
  if (unroll) *unroll = c.unroll;
  if (blocks_per_cu) *blocks_per_cu = c.bpc;
  if (dynamic) *dynamic = dyn ? 1 : 0;
  if (store_policy) *store_policy = c.store + 1;
  return 0;
}

int hiccl_reduce_auto_choice(int dtype, int acc, size_t count, double n, int cus, int *engine, int *unroll,
                             int *blocks_per_cu, int *dynamic) {
  hiccl_reduce_config_t z;
  memset(&z, 0, sizeof(z));
  z.acc = acc;
  return hiccl_reduce_auto_choice_ex(dtype, &z, count, n, cus, engine, unroll, blocks_per_cu, dynamic, nullptr);
}

// ---------------------------------------------------------------- plan ----

}  // extern "C"

struct hiccl_reduce_plan {
  int dtype = 0;
  int device = 0;
  hiccl_reduce_config_t req;      // hiccl_reduce_plan_set_config / _set_engine / _set_acc (0 = default)
  int engine = HICCL_ENGINE_TILE;  // resolved at upload
  int unroll = kDefUnroll;         // TILE packets per lane, resolved at upload
  double mean_n = 0;               // packet-weighted inputs per compute
  int bpc = 1;                     // workgroups per CU, resolved at upload
  int peer = 0;                    // hiccl_reduce_plan_set_peer flags
  int eff_peer = 0;                // peer | the store form plan_store_peer picks, resolved at upload
  size_t esz = 0;
  struct Comp {
    void *out;
    std::vector<const void *> in;
    size_t count;
  };
  std::vector<Comp> comps;
  int maxn = 0;
  bool dirty = true;
  char *d_block = nullptr;  // [desc | ptrs | unit_comp] (PlanArgs)
  PlanArgs args;            // pointers into d_block
  uint64_t total_tiles = 0;
  hipStream_t own = nullptr;
  hipStream_t last = nullptr;  // stream of the last launch (plan_sync synchronises it)
  bool launched = false;
  std::atomic<bool> enqueued{false};  // some launch went out (on a stream not remembered)
};

namespace {
// Before the plan's device block is freed: no launch may still read it.
void plan_quiesce(hiccl_reduce_plan *p) {
  if (p->enqueued.load(std::memory_order_relaxed)) {
    (void)hipDeviceSynchronize();
    p->enqueued.store(false, std::memory_order_relaxed);
  } else if (p->launched) {
    (void)hipStreamSynchronize(p->last);
  }
}
}  // namespace

namespace {

// Store form of a plan's launches.  nt stores are not write-through: a
// launch's output lines may sit dirty in the XCD L2s until the end-of-kernel
// release writes them back, on the critical path of the next kernel on the
// stream (MI355X_MICROARCH.md "boundary": + B / 6 TB/s for B dirty bytes).
// So a plan that writes at most wt_cap(n) bytes per launch stores with
// system-scope write-through (sc0 sc1, the peer-store form) instead, when its
// config leaves the store form to size (store_policy 0).  Measured on the C5
// step (4 x n = 2 + 1 x n = 4 computes of 2^18 f32, 5 MiB written, plus its
// five 1 MiB byte copies; tools/step_store_probe.py,
// profiles/r05d_step_store.jsonl): the reduction 4.52 -> 3.53 us per eager
// launch (0.49 -> 0.63 of 8 TB/s), 3.01 -> 2.91 us under graph replay, the
// copies 3.53 -> 3.28 us; 10-20 MiB written 20-38 % faster.  Byte copies
// lose from 48 MiB written (1-4 %); reductions keep gaining up to 256 MiB
// (tools/store_threshold_probe.py: 8 inputs writing 32-256 MiB 1.6-3 %
// faster, config 3's buckets -- n x 256 MiB -- 1.2-9.2 %, n = 2 reaching
// 7.02 TB/s; profiles/r05o_store_threshold.jsonl, r05p_store_c3.jsonl) and
// stop at 512 MiB and 1 GiB (-0.7 / -0.6 % on the TILE engine, config 2 no
// gain; r05q_store_big.jsonl, r05j_c2_store_ab.jsonl): hence the two caps
// (wt_cap; one-shot calls follow the same rule, hiccl_reduce_ex).
int plan_store_peer(const hiccl_reduce_plan *p) {
  const int req = p->req.store_policy;  // 0: by size; 2: nt; 4: write-through (plan_set_config checked it)
  if (req == kPolStoreSys + 1) return HICCL_PEER_STORES;
  if (req != 0) return 0;
  // by size only where a write-through kernel of the plan's shape exists: an
  // explicit TILE unroll other than 2 / 4 keeps nt stores
  const int u = p->req.unroll;
  if (u && u != 2 && u != kDefUnroll && p->req.engine != HICCL_ENGINE_PHASE) return 0;
  uint64_t out = 0;
  double weighted_n = 0;
  for (auto &c : p->comps) {
    out += (uint64_t)c.count * p->esz;
    weighted_n += (double)c.count * (double)c.in.size();
  }
  const double n = out ? weighted_n * (double)p->esz / (double)out : 0.0;
  return out <= wt_cap(p->dtype == HICCL_BYTES ? 1.0 : n) ? HICCL_PEER_STORES : 0;
}

int plan_eff_peer(const hiccl_reduce_plan *p) { return p->peer | plan_store_peer(p); }

// The plan's configuration with its engine and shape resolved for `npkt`
// packets of packet-weighted mean `mean_n` inputs.
Cfg plan_cfg(const hiccl_reduce_plan *p, uint64_t npkt, double mean_n) {
  Cfg c = resolve(&p->req);
  const bool auto_unroll = !c.unroll;
  // AUTO's engine rules follow the store form the launches take by size
  // (plan_store_peer already checked the shape has a write-through kernel)
  c.wt = c.store_auto && (plan_store_peer(p) & HICCL_PEER_STORES);
  finish_cfg(c, npkt, mean_n, p->dtype, p->device);  // (kPlanBlock == kDefBlock)
  // peer and write-through policies exist at TILE U = 4 / 2 only: wide tiles
  // become U = 4
  if (p->eff_peer && c.engine == HICCL_ENGINE_TILE && auto_unroll && c.unroll != 2) c.unroll = kDefUnroll;
  return c;
}

// Lay out [desc (ncomp) | ptrs (ncomp x stride) | unit_comp (units)] on the
// host, 8-B aligned pieces; returns the byte size, fills the offsets.
struct BlockLayout {
  size_t desc, ptrs, unit_comp, bytes;
};
BlockLayout block_layout(size_t ncomp, size_t stride, size_t units) {
  BlockLayout L;
  L.desc = 0;
  L.ptrs = ncomp * sizeof(PlanDesc);
  L.unit_comp = L.ptrs + ncomp * stride * sizeof(void *);
  L.bytes = L.unit_comp + ((units * sizeof(uint32_t) + 7) & ~(size_t)7);
  return L;
}

int plan_upload(hiccl_reduce_plan *p, hipStream_t s) {
  if (!p->dirty) return 0;
  // synchronous allocation + copy: not allowed inside a stream capture
  // (capture a plan only after a launch outside the capture uploaded it)
  if (capturing(s, false))
    return fail(hipErrorStreamCaptureUnsupported,
                "plan: the first launch after an add or a config change uploads the plan and cannot be captured");
  if (p->d_block) {
    plan_quiesce(p);  // a running launch still reads it
    (void)hipFree(p->d_block);
    p->d_block = nullptr;
  }
  const size_t nc = p->comps.size();
  uint64_t total_pkt = 0;
  double weighted_n = 0;
  p->maxn = 0;
  for (auto &c : p->comps) {
    const uint64_t k = split_on(c.out, c.count, p->esz).npkt;
    total_pkt += k;
    weighted_n += (double)k * c.in.size();
    if ((int)c.in.size() > p->maxn) p->maxn = (int)c.in.size();
  }
  const double mean_n = total_pkt ? weighted_n / total_pkt : 0;
  p->mean_n = mean_n;
  p->eff_peer = plan_eff_peer(p);
  const Cfg c = plan_cfg(p, total_pkt, mean_n);
  p->engine = c.engine;
  p->unroll = c.unroll;
  p->bpc = c.bpc;
  const uint64_t unit = unit_pkts(p->engine, p->dtype, c.acc, p->unroll);
  uint64_t units = 0;
  for (auto &cp : p->comps) units += tiles_for(split_on(cp.out, cp.count, p->esz).npkt, unit);
  const size_t stride = p->maxn > 0 ? (size_t)p->maxn : 1;
  const BlockLayout L = block_layout(nc, stride, units);
  std::vector<char> host(L.bytes, 0);
  PlanDesc *hd = (PlanDesc *)(host.data() + L.desc);
  const void **hp = (const void **)(host.data() + L.ptrs);
  uint32_t *hu = (uint32_t *)(host.data() + L.unit_comp);
  uint64_t tile = 0;
  for (size_t i = 0; i < nc; i++) {
    auto &cp = p->comps[i];
    Split sp = split_on(cp.out, cp.count, p->esz);
    PlanDesc &d = hd[i];
    d.out = (char *)cp.out;
    d.npkt = sp.npkt;
    d.head = sp.head;
    d.tail = sp.tail;
    d.n = (uint32_t)cp.in.size();
    d.tile_begin = tile;
    for (size_t k = 0; k < cp.in.size(); k++) hp[i * stride + k] = cp.in[k];
    const uint64_t nt = tiles_for(sp.npkt, unit);
    for (uint64_t t = 0; t < nt; t++) hu[tile + t] = (uint32_t)i;
    tile += nt;
  }
  p->total_tiles = tile;
  if (int e = check_hip(hipMalloc((void **)&p->d_block, L.bytes), "plan: hipMalloc")) return e;
  if (int e = check_hip(hipMemcpy(p->d_block, host.data(), L.bytes, hipMemcpyHostToDevice), "plan: upload"))
    return e;
  memset(&p->args, 0, sizeof(p->args));
  p->args.desc = (const PlanDesc *)(p->d_block + L.desc);
  p->args.ptrs = (const char *const *)(p->d_block + L.ptrs);
  p->args.unit_comp = nc > 1 ? (const uint32_t *)(p->d_block + L.unit_comp) : nullptr;
  p->args.stride = (uint32_t)stride;
  p->args.t_begin = 0;
  p->args.t_end = tile;
  p->dirty = false;
  return 0;
}

// One plan-kernel launch of `a` (desc, ptrs, unit_comp, units, stride set),
// shaped by `c` (engine and shape resolved).
int launch_plan(PlanArgs a, int dtype, const Cfg &c, double mean_n, int dev, hipStream_t s, int pol = kDefPol) {
  plan_fn fn = pick_plan(dtype, c.acc, c.engine, c.unroll, pol);
  if (!fn)
    return fail(hipErrorInvalidValue, pol == kDefPol ? "plan: unsupported dtype / shape"
                                                     : "plan: no peer-policy kernel for this shape (PHASE default, "
                                                       "TILE unroll 4, f32 / bf16 also 2)");
  const uint64_t units = a.t_end - a.t_begin;
  uint64_t grid = c.grid > 0 ? (uint64_t)c.grid : (uint64_t)device_cus(dev) * c.bpc;
  if (grid > units) grid = units;
  a.grab = c.grab > 0 ? (uint32_t)c.grab : default_grab(c.engine, mean_n, c.unroll);
  a.sched = unit_sched_for(c.engine, mean_n, units, grid, dev, s, c.schedule, a.grab, c.unroll);
  fn(a, dim3((unsigned)grid), s);
  return check_hip(hipGetLastError(), "plan: launch");
}

int plan_kernel(hiccl_reduce_plan *p, hipStream_t s) {
  Cfg c = resolve(&p->req);
  c.engine = p->engine;
  c.unroll = p->unroll;
  c.block = p->engine == HICCL_ENGINE_PHASE ? kPhBlock : kPlanBlock;
  c.bpc = p->bpc;
  return launch_plan(p->args, p->dtype, c, p->mean_n, p->device, s, plan_pol(p->eff_peer));
}

int reduce_via_table(int dtype, const Cfg &c, void *out, const void *const *in, int n, size_t count,
                     hipStream_t s) {
  const size_t esz = esize(dtype);
  Split sp = split_on(out, count, esz);
  const BlockLayout L = block_layout(1, (size_t)n, 0);
  std::vector<char> host(L.bytes, 0);
  PlanDesc *hd = (PlanDesc *)(host.data() + L.desc);
  const void **hp = (const void **)(host.data() + L.ptrs);
  for (int k = 0; k < n; k++) hp[k] = in[k];
  hd->out = (char *)out;
  hd->npkt = sp.npkt;
  hd->head = sp.head;
  hd->tail = sp.tail;
  hd->n = (uint32_t)n;
  hd->tile_begin = 0;
  char *dmem = nullptr;
  if (int e = check_hip(hipMallocAsync((void **)&dmem, L.bytes, s), "hiccl_reduce: hipMallocAsync")) return e;
  // hipMemcpyAsync from pageable memory returns once the source is consumed,
  // so `host` may go out of scope (never under capture: refused by the caller)
  if (int e = check_hip(hipMemcpyAsync(dmem, host.data(), L.bytes, hipMemcpyHostToDevice, s),
                        "hiccl_reduce: table upload")) {
    (void)hipFreeAsync(dmem, s);
    return e;
  }
  PlanArgs a;
  memset(&a, 0, sizeof(a));
  a.desc = (const PlanDesc *)(dmem + L.desc);
  a.ptrs = (const char *const *)(dmem + L.ptrs);
  a.unit_comp = nullptr;
  a.stride = (uint32_t)n;
  a.t_begin = 0;
  a.t_end = tiles_for(sp.npkt, unit_pkts(c.engine, dtype, c.acc, c.unroll));
  // the store form oneshot_cfg decided: write-through by size or on request
  // (store_policy 4), else nt
  const int pol = c.store == kPolStoreSys ? plan_pol(HICCL_PEER_STORES) : kDefPol;
  if (int e = launch_plan(a, dtype, c, n, current_device(), s, pol)) {
    (void)hipFreeAsync(dmem, s);  // nothing launched reads it
    return e;
  }
  return check_hip(hipFreeAsync(dmem, s), "hiccl_reduce: hipFreeAsync");
}

}  // namespace

extern "C" {

int hiccl_reduce_plan_create(hiccl_reduce_plan_t **plan, int dtype, int device) {
  if (!plan) return fail(hipErrorInvalidValue, "plan_create: plan is NULL");
  *plan = nullptr;
  if (!esize(dtype)) return fail(hipErrorInvalidValue, "plan_create: unknown dtype");
  int ndev = 0;
  if (int e = check_hip(hipGetDeviceCount(&ndev), "plan_create: hipGetDeviceCount")) return e;
  if (device < 0 || device >= ndev) return fail(hipErrorInvalidDevice, "plan_create: bad device");
  if (int e = check_hip(hipSetDevice(device), "plan_create: hipSetDevice")) return e;
  auto *p = new hiccl_reduce_plan;
  memset(&p->req, 0, sizeof(p->req));
  p->dtype = dtype;
  p->device = device;
  p->esz = esize(dtype);
  // the plan's own stream is created on first request (hiccl_reduce_plan_stream):
  // callers that launch on a shared stream never pay for one
  *plan = p;
  return 0;
}

int hiccl_reduce_plan_set_acc(hiccl_reduce_plan_t *p, int acc) {
  if (!p) return fail(hipErrorInvalidValue, "plan_set_acc: plan is NULL");
  if (acc != HICCL_ACC_NATIVE && acc != HICCL_ACC_WIDE)
    return fail(hipErrorInvalidValue, "plan_set_acc: bad mode");
  p->req.acc = acc;
  p->dirty = true;  // the auto engine's chunk size depends on the accumulator
  return 0;
}

int hiccl_reduce_plan_set_engine(hiccl_reduce_plan_t *p, int engine) {
  if (!p) return fail(hipErrorInvalidValue, "plan_set_engine: plan is NULL");
  if (engine < HICCL_ENGINE_AUTO || engine > HICCL_ENGINE_PHASE)
    return fail(hipErrorInvalidValue, "plan_set_engine: bad engine");
  p->req.engine = engine;
  p->dirty = true;
  return 0;
}

int hiccl_reduce_plan_set_peer(hiccl_reduce_plan_t *p, int flags) {
  if (!p) return fail(hipErrorInvalidValue, "plan_set_peer: plan is NULL");
  if (flags & ~(HICCL_PEER_STORES | HICCL_PEER_LOADS))
    return fail(hipErrorInvalidValue, "plan_set_peer: flags must be a combination of HICCL_PEER_STORES and HICCL_PEER_LOADS");
  p->peer = flags;
  p->dirty = true;
  return 0;
}

int hiccl_reduce_plan_peer(const hiccl_reduce_plan_t *p) { return p ? p->peer : -1; }

int hiccl_reduce_plan_store_policy(const hiccl_reduce_plan_t *p) {
  if (!p) return -1;
  return (plan_eff_peer(p) & HICCL_PEER_STORES) ? kPolStoreSys + 1 : kDefPol / 10 + 1;
}

int hiccl_reduce_plan_set_config(hiccl_reduce_plan_t *p, const hiccl_reduce_config_t *cfg) {
  if (!p) return fail(hipErrorInvalidValue, "plan_set_config: plan is NULL");
  hiccl_reduce_config_t z;
  memset(&z, 0, sizeof(z));
  const hiccl_reduce_config_t &c = cfg ? *cfg : z;
  if (c.acc != HICCL_ACC_NATIVE && c.acc != HICCL_ACC_WIDE) return fail(hipErrorInvalidValue, "plan_set_config: bad acc");
  if (c.engine < HICCL_ENGINE_AUTO || c.engine > HICCL_ENGINE_PHASE)
    return fail(hipErrorInvalidValue, "plan_set_config: bad engine");
  if (c.schedule < HICCL_SCHED_AUTO || c.schedule > HICCL_SCHED_DYNAMIC)
    return fail(hipErrorInvalidValue, "plan_set_config: bad schedule");
  if (c.grab < 0 || c.grab > 4096) return fail(hipErrorInvalidValue, "plan_set_config: bad grab");
  if (c.blocks_per_cu < 0 || c.blocks_per_cu > 64) return fail(hipErrorInvalidValue, "plan_set_config: blocks_per_cu");
  if (c.grid < 0) return fail(hipErrorInvalidValue, "plan_set_config: grid < 0");
  // the shape must be one the plan kernels have, whatever engine AUTO picks
  Cfg r = resolve(&c);
  const bool shape = c.block || c.unroll;
  if (shape && r.engine == HICCL_ENGINE_AUTO) r.engine = HICCL_ENGINE_TILE;
  const int engines[2] = {HICCL_ENGINE_TILE, HICCL_ENGINE_PHASE};
  for (int eng : engines) {
    if (r.engine != HICCL_ENGINE_AUTO && r.engine != eng) continue;
    Cfg t = r;
    t.engine = eng;
    if (!t.block) t.block = eng == HICCL_ENGINE_PHASE ? kPhBlock : kPlanBlock;
    if (!t.unroll) t.unroll = eng == HICCL_ENGINE_PHASE ? phase_p_dtype(p->dtype, t.acc) : kDefUnroll;
    const std::string why = plan_shape_error(t, p->dtype);
    if (!why.empty()) return fail(hipErrorInvalidValue, "plan_set_config: " + why);
  }
  p->req = c;
  p->dirty = true;
  return 0;
}

int hiccl_reduce_plan_engine(const hiccl_reduce_plan_t *p) { return p ? p->engine : -1; }

int hiccl_reduce_plan_add(hiccl_reduce_plan_t *p, void *out, const void *const *in, int n,
                          size_t count) {
  if (!p) return fail(hipErrorInvalidValue, "plan_add: plan is NULL");
  if (p->dtype == HICCL_BYTES && n != 1) return fail(hipErrorInvalidValue, "plan_add: HICCL_BYTES copies need n == 1");
  if (int e = check_buffers(out, in, n, count, p->esz)) return e;
  if (count == 0) return 0;
  hiccl_reduce_plan::Comp c;
  c.out = out;
  c.in.assign(in, in + n);
  c.count = count;
  p->comps.push_back(std::move(c));
  p->dirty = true;
  return 0;
}

}  // extern "C"

namespace {
// Upload (if needed) and launch, no bookkeeping of where the launch went.
int plan_enqueue_impl(hiccl_reduce_plan_t *p, hipStream_t s, const char *what) {
  if (!p) return fail(hipErrorInvalidValue, std::string(what) + ": plan is NULL");
  if (int e = check_hip(hipSetDevice(p->device), (std::string(what) + ": hipSetDevice").c_str())) return e;
  if (p->comps.empty()) return 0;
  if (int e = plan_upload(p, s)) return e;
  return plan_kernel(p, s);
}
}  // namespace

extern "C" {

int hiccl_reduce_plan_enqueue(hiccl_reduce_plan_t *p, void *stream) {
  if (int e = plan_enqueue_impl(p, (hipStream_t)stream, "plan_enqueue")) return e;
  // no stream bookkeeping (callers on several threads and streams); a
  // re-upload or destroy then synchronises the device before it frees the
  // block a launch may still read
  if (!p->comps.empty()) p->enqueued.store(true, std::memory_order_relaxed);
  return 0;
}

int hiccl_reduce_plan_launch(hiccl_reduce_plan_t *p, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  if (int e = plan_enqueue_impl(p, s, "plan_launch")) return e;
  if (p->comps.empty()) return 0;
  // a capturing stream is not remembered (plan_sync does not apply to graph
  // replays: synchronise the stream the graph runs on); a re-upload or
  // destroy of a plan captured into a graph synchronises the device
  if (capturing(s, false)) {
    p->enqueued.store(true, std::memory_order_relaxed);
    return 0;
  }
  p->launched = true;
  p->last = s;
  return 0;
}

int hiccl_reduce_plan_launch_each(hiccl_reduce_plan_t *p, void *stream) {
  if (!p) return fail(hipErrorInvalidValue, "plan_launch_each: plan is NULL");
  if (int e = check_hip(hipSetDevice(p->device), "plan_launch_each: hipSetDevice")) return e;
  if (p->comps.empty()) return 0;
  // One one-shot launch per compute, each with the engine AUTO picks for that
  // compute alone (the reference's structure, compute.h:88-91).
  for (auto &c : p->comps)
    if (int e = hiccl_reduce_ex(p->dtype, c.out, c.in.data(), (int)c.in.size(), c.count, stream, &p->req))
      return e;
  p->launched = true;
  p->last = (hipStream_t)stream;
  return 0;
}

int hiccl_reduce_plan_sync(hiccl_reduce_plan_t *p) {
  if (!p) return fail(hipErrorInvalidValue, "plan_sync: plan is NULL");
  if (!p->launched) return 0;
  if (int e = check_hip(hipSetDevice(p->device), "plan_sync: hipSetDevice")) return e;
  // the reference's wait(): hipStreamSynchronize of the compute's stream
  // (compute.h:107-117) -- no completion event per launch (an event record
  // after every kernel costs the queue ~3 us per step on MI355X)
  if (int e = check_hip(hipStreamSynchronize(p->last), "plan_sync")) return e;
  // nothing of this plan is pending on that stream any more: a later
  // re-upload or destroy does not touch it (the caller may destroy it)
  p->launched = false;
  return 0;
}

int hiccl_reduce_plan_numcomp(const hiccl_reduce_plan_t *p) { return p ? (int)p->comps.size() : 0; }

void *hiccl_reduce_plan_stream(hiccl_reduce_plan_t *p) {
  if (!p) return nullptr;
  if (!p->own) {
    if (check_hip(hipSetDevice(p->device), "plan_stream: hipSetDevice")) return nullptr;
    if (check_hip(hipStreamCreateWithFlags(&p->own, hipStreamNonBlocking), "plan_stream: create")) return nullptr;
  }
  return (void *)p->own;
}

size_t hiccl_reduce_plan_bytes(const hiccl_reduce_plan_t *p) {
  if (!p) return 0;
  size_t b = 0;
  for (auto &c : p->comps) b += c.count * (c.in.size() + 1) * p->esz;
  return b;
}

void hiccl_reduce_plan_destroy(hiccl_reduce_plan_t *p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->d_block) plan_quiesce(p);
  else if (p->launched) (void)hipStreamSynchronize(p->last);
  if (p->d_block) (void)hipFree(p->d_block);
  if (p->own) (void)hipStreamDestroy(p->own);
  delete p;
}

// -------------------------------------------------- host-resident buckets --

}  // extern "C"

struct hiccl_host_pipe {
  int dtype = 0;
  int device = 0;
  size_t esz = 0;
  size_t chunk = 0;  // elements per input per chunk
  int depth = 0;
  int cap_n = 0;     // staging slots hold this many inputs
  std::vector<hipStream_t> streams;
  std::vector<char *> stage;  // per slot: max(cap_n, 1) x chunk elements
};

namespace {

constexpr size_t kPipeChunkBytes = 64ull << 20;
constexpr int kPipeDepth = 3;

int pipe_stage_for(hiccl_host_pipe *p, int n) {
  const int need = n > 0 ? n : 1;
  if (need <= p->cap_n) return 0;
  for (auto &b : p->stage)
    if (b) { (void)hipFree(b); b = nullptr; }
  p->cap_n = 0;
  for (auto &b : p->stage)
    if (int e = check_hip(hipMalloc((void **)&b, (size_t)need * p->chunk * p->esz), "host_pipe: hipMalloc staging"))
      return e;
  p->cap_n = need;
  return 0;
}

}  // namespace

extern "C" {

int hiccl_host_pipe_create(hiccl_host_pipe_t **pipe, int dtype, int device, size_t chunk_bytes,
                           int depth) {
  if (!pipe) return fail(hipErrorInvalidValue, "host_pipe_create: pipe is NULL");
  *pipe = nullptr;
  const size_t esz = esize(dtype);
  if (!esz) return fail(hipErrorInvalidValue, "host_pipe_create: unknown dtype");
  if (depth < 0 || depth > 8) return fail(hipErrorInvalidValue, "host_pipe_create: depth must be 0..8");
  if (!chunk_bytes) chunk_bytes = kPipeChunkBytes;
  if (chunk_bytes < esz) return fail(hipErrorInvalidValue, "host_pipe_create: chunk_bytes below one element");
  int ndev = 0;
  if (int e = check_hip(hipGetDeviceCount(&ndev), "host_pipe_create: hipGetDeviceCount")) return e;
  if (device < 0 || device >= ndev) return fail(hipErrorInvalidDevice, "host_pipe_create: bad device");
  if (int e = check_hip(hipSetDevice(device), "host_pipe_create: hipSetDevice")) return e;
  auto *p = new hiccl_host_pipe;
  p->dtype = dtype;
  p->device = device;
  p->esz = esz;
  p->chunk = chunk_bytes / esz;
  p->depth = depth ? depth : kPipeDepth;
  p->stage.assign(p->depth, nullptr);
  for (int i = 0; i < p->depth; i++) {
    hipStream_t s = nullptr;
    if (int e = check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "host_pipe_create: stream")) {
      hiccl_host_pipe_destroy(p);
      return e;
    }
    p->streams.push_back(s);
  }
  *pipe = p;
  return 0;
}

int hiccl_host_pipe_reduce(hiccl_host_pipe_t *p, void *out, const void *const *in, int n, size_t count) {
  if (!p) return fail(hipErrorInvalidValue, "host_pipe_reduce: pipe is NULL");
  if (p->dtype == HICCL_BYTES && n != 1) return fail(hipErrorInvalidValue, "host_pipe_reduce: HICCL_BYTES copies need n == 1");
  if (int e = check_buffers(out, in, n, count, p->esz)) return e;
  if (count == 0) return 0;
  if (int e = check_hip(hipSetDevice(p->device), "host_pipe_reduce: hipSetDevice")) return e;
  if (int e = pipe_stage_for(p, n)) return e;
  const size_t slot_in = p->chunk * p->esz;  // bytes between staged inputs
  std::vector<const void *> dev_in((size_t)(n > 0 ? n : 1));
  int err = 0;
  size_t c = 0;
  for (size_t lo = 0; lo < count && !err; lo += p->chunk, c++) {
    const size_t len = count - lo < p->chunk ? count - lo : p->chunk;
    const int slot = (int)(c % (size_t)p->depth);
    hipStream_t s = p->streams[slot];
    char *stage = p->stage[slot];
    for (int k = 0; k < n && !err; k++) {
      dev_in[k] = stage + (size_t)k * slot_in;
      err = check_hip(hipMemcpyAsync(stage + (size_t)k * slot_in, (const char *)in[k] + lo * p->esz,
                                     len * p->esz, hipMemcpyHostToDevice, s),
                      "host_pipe_reduce: H2D");
    }
    // in place into staged input 0 (exact aliasing is element-wise safe)
    if (!err) err = hiccl_reduce_ex(p->dtype, stage, dev_in.data(), n, len, s, nullptr);
    if (!err)
      err = check_hip(hipMemcpyAsync((char *)out + lo * p->esz, stage, len * p->esz, hipMemcpyDeviceToHost, s),
                      "host_pipe_reduce: D2H");
  }
  for (hipStream_t s : p->streams) {  // drain every slot, even after an error
    int e = check_hip(hipStreamSynchronize(s), "host_pipe_reduce: sync");
    if (!err) err = e;
  }
  return err;
}

void hiccl_host_pipe_destroy(hiccl_host_pipe_t *p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  for (hipStream_t s : p->streams) (void)hipStreamSynchronize(s);
  for (char *b : p->stage)
    if (b) (void)hipFree(b);
  for (hipStream_t s : p->streams) (void)hipStreamDestroy(s);
  delete p;
}

// ---------------------------------------------------- stream signalling --

int hiccl_signal_wait(uint32_t *const *sig, int nsig, const uint32_t *const *wait, int nwait,
                      uint32_t epoch, uint32_t *err, double timeout_s, void *stream) {
  return hiccl_signal_wait_dev(sig, nsig, wait, nwait, epoch, nullptr, err, timeout_s, stream);
}

int hiccl_counter_add(uint32_t *ctr, uint32_t v, void *stream) {
  if (!ctr) return fail(hipErrorInvalidValue, "counter_add: ctr is NULL");
  hipLaunchKernelGGL(k_counter_add, dim3(1), dim3(64), 0, (hipStream_t)stream, ctr, v);
  return check_hip(hipGetLastError(), "counter_add: launch");
}

int hiccl_signal_wait_dev(uint32_t *const *sig, int nsig, const uint32_t *const *wait, int nwait,
                          uint32_t epoch, const uint32_t *epoch_dev, uint32_t *err, double timeout_s,
                          void *stream) {
  hiccl_signal_phase_t ph;
  ph.sig = sig;
  ph.nsig = nsig;
  ph.wait = wait;
  ph.nwait = nwait;
  ph.epoch = epoch;
  return hiccl_signal_wait_phases(&ph, 1, epoch_dev, err, timeout_s, stream);
}

int hiccl_signal_wait_phases(const hiccl_signal_phase_t *ph, int nph, const uint32_t *epoch_dev, uint32_t *err,
                             double timeout_s, void *stream) {
  if (nph < 0 || (nph && !ph)) return fail(hipErrorInvalidValue, "signal_wait: bad phase list");
  for (int p = 0; p < nph; p++) {
    const hiccl_signal_phase_t &q = ph[p];
    if (q.nsig < 0 || q.nwait < 0 || (q.nsig && !q.sig) || (q.nwait && !q.wait))
      return fail(hipErrorInvalidValue, "signal_wait: bad flag lists");
    for (int i = 0; i < q.nsig; i++)
      if (!q.sig[i]) return fail(hipErrorInvalidValue, "signal_wait: NULL signal flag");
    for (int i = 0; i < q.nwait; i++)
      if (!q.wait[i]) return fail(hipErrorInvalidValue, "signal_wait: NULL wait flag");
  }
  const uint64_t ticks = (uint64_t)((timeout_s > 0 ? timeout_s : 30.0) * 1e8);  // s_memrealtime: 100 MHz
  hipStream_t s = (hipStream_t)stream;
  SigPhaseArgs a;
  const uint32_t light = prog_light() ? 1u : 0u;
  auto reset = [&]() {
    memset(&a, 0, sizeof(a));
    a.err = err;
    a.epoch_dev = epoch_dev;
    a.timeout_ticks = ticks;
    a.light = light;
  };
  auto launch = [&]() -> int {
    if (!a.nphase) return 0;
    hipLaunchKernelGGL(k_sigwait_phases, dim3(1), dim3(64), 0, s, a);
    int e = check_hip(hipGetLastError(), "signal_wait: launch");
    reset();
    return e;
  };
  // Append (sig[0..ns), wait[0..nw)) with `epoch` as one sub-phase, starting
  // a new launch when the kernel's arrays or phase slots are full.
  auto push = [&](uint32_t *const *sg, int ns, const uint32_t *const *wt, int nw, uint32_t epoch) -> int {
    if (a.nphase == (uint32_t)kMaxPhases ||
        (a.nphase ? a.sig_end[a.nphase - 1] : 0) + ns > (uint32_t)kMaxFlags ||
        (a.nphase ? a.wait_end[a.nphase - 1] : 0) + nw > (uint32_t)kMaxFlags)
      if (int e = launch()) return e;
    const uint32_t s0 = a.nphase ? a.sig_end[a.nphase - 1] : 0, w0 = a.nphase ? a.wait_end[a.nphase - 1] : 0;
    for (int i = 0; i < ns; i++) a.sig[s0 + i] = sg[i];
    for (int i = 0; i < nw; i++) a.wait[w0 + i] = wt[i];
    a.sig_end[a.nphase] = s0 + ns;
    a.wait_end[a.nphase] = w0 + nw;
    a.epoch[a.nphase] = epoch;
    a.nphase++;
    return 0;
  };
  reset();
  for (int p = 0; p < nph; p++) {
    const hiccl_signal_phase_t &q = ph[p];
    if (q.nsig + q.nwait == 0) continue;
    if (q.nsig <= kMaxFlags && q.nwait <= kMaxFlags) {
      if (int e = push(q.sig, q.nsig, q.wait, q.nwait, q.epoch)) return e;
      continue;
    }
    // a phase above kMaxFlags: every signal first, then the waits, in
    // kMaxFlags pieces (a wait must never precede a signal of its phase)
    for (int i = 0; i < q.nsig; i += kMaxFlags)
      if (int e = push(q.sig + i, q.nsig - i < kMaxFlags ? q.nsig - i : kMaxFlags, nullptr, 0, q.epoch)) return e;
    for (int i = 0; i < q.nwait; i += kMaxFlags)
      if (int e = push(nullptr, 0, q.wait + i, q.nwait - i < kMaxFlags ? q.nwait - i : kMaxFlags, q.epoch))
        return e;
  }
  return launch();
}

}  // extern "C"

// ------------------------------------------------------------ step programs --

struct hiccl_program {
  int dtype = 0;
  int device = 0;
  struct Unit {
    void *out;
    std::vector<const void *> in;
    size_t count;
    bool bytes;  // exact byte copy (a HICCL_BYTES plan's compute)
    int peer;    // the plan's hiccl_reduce_plan_set_peer flags
  };
  std::vector<Unit> units;  // the unit batch (after the phases)
  struct Phase {
    std::vector<uint32_t *> sig;
    std::vector<const uint32_t *> wait;
  };
  std::vector<Phase> phases;  // the prologue
  bool dirty = true;
  char *d_block = nullptr;
  uint64_t *d_gate = nullptr;
  uint64_t seq = 0;  // last sequence number used (eager launches; captures reserve a range)
  ProgArgs args;
  int unroll = 4;
  uint32_t grid = 0;
  uint32_t max_wg = 0;  // hiccl_program_set_max_workgroups (0: default)
  std::atomic<bool> enqueued{false};
};

namespace {

// Workgroups per CU of a program launch: a small batch (under one 16 KiB
// tile per lane-group per CU, the C5 step) takes 4 like the plan kernel's
// small launches, larger ones 2.
constexpr int kProgSmallBpc = 4;
constexpr int kProgBpc = 2;

typedef void (*prog_fn)(const ProgArgs &, dim3, hipStream_t);

template <class Op, int U>
void launch_prog_t(const ProgArgs &a, dim3 grid, hipStream_t s) {
  hipLaunchKernelGGL((k_program<Op, U>), grid, dim3(kProgBlock), 0, s, a);
}

prog_fn pick_prog(int dtype, int unroll) {
  const bool u2 = unroll == 2;
  switch (dtype) {
    case HICCL_FLOAT32: return u2 ? launch_prog_t<OpF32, 2> : launch_prog_t<OpF32, 4>;
    case HICCL_BFLOAT16: return u2 ? launch_prog_t<OpBF16, 2> : launch_prog_t<OpBF16, 4>;
    case HICCL_FLOAT64: return u2 ? nullptr : launch_prog_t<OpF64, 4>;
    case HICCL_UINT64: return u2 ? nullptr : launch_prog_t<OpU64, 4>;
    case HICCL_INT32: return u2 ? nullptr : launch_prog_t<OpI32, 4>;
    case HICCL_BYTES: return u2 ? nullptr : launch_prog_t<OpRaw, 4>;
    default: return nullptr;
  }
}

void prog_quiesce(hiccl_program *p) {
  if (p->enqueued.load(std::memory_order_relaxed)) {
    (void)hipDeviceSynchronize();
    p->enqueued.store(false, std::memory_order_relaxed);
  }
}

int prog_upload(hiccl_program *p, hipStream_t s) {
  if (!p->dirty) return 0;
  if (capturing(s, false))
    return fail(hipErrorStreamCaptureUnsupported,
                "program: the first launch after a change uploads the program and cannot be captured");
  prog_quiesce(p);
  if (p->d_block) {
    (void)hipFree(p->d_block);
    p->d_block = nullptr;
  }
  if (!p->d_gate) {
    if (int e = check_hip(hipMalloc((void **)&p->d_gate, 256), "program: hipMalloc(gate)")) return e;
    if (int e = check_hip(hipMemset(p->d_gate, 0, 256), "program: hipMemset(gate)")) return e;
    p->seq = 0;
  }
  const int cus = device_cus(p->device);
  const size_t tesz = esize(p->dtype);
  auto esz_of = [&](const hiccl_program::Unit &u) { return u.bytes ? (size_t)1 : tesz; };
  uint64_t total_pkt = 0;
  size_t maxn = 1;
  for (auto &u : p->units) {
    total_pkt += split_on(u.out, u.count, esz_of(u)).npkt;
    if (u.in.size() > maxn) maxn = u.in.size();
  }
  // half-size tiles when the batch has under two 16 KiB tiles per CU (auto_unroll)
  const bool small = total_pkt < 2ull * cus * kProgBlock * 4;
  p->unroll = pick_prog(p->dtype, 2) && small ? 2 : 4;
  const uint64_t unit = (uint64_t)kProgBlock * p->unroll;
  const size_t ncomp = p->units.size();
  std::vector<uint32_t> unit_comp;
  std::vector<PlanDesc> desc(ncomp);
  std::vector<const void *> ptrs(ncomp * maxn, nullptr);
  for (size_t c = 0; c < ncomp; c++) {
    auto &u = p->units[c];
    const Split sp = split_on(u.out, u.count, esz_of(u));
    PlanDesc &d = desc[c];
    d.out = (char *)u.out;
    d.npkt = sp.npkt;
    d.head = sp.head;
    d.tail = sp.tail;
    d.n = (uint32_t)u.in.size();
    d.pad = (u.bytes ? 1u : 0u) | ((uint32_t)u.peer << 1);
    d.tile_begin = unit_comp.size();
    for (size_t k = 0; k < u.in.size(); k++) ptrs[c * maxn + k] = u.in[k];
    const uint64_t nt = tiles_for(sp.npkt, unit);
    for (uint64_t t = 0; t < nt; t++) unit_comp.push_back((uint32_t)c);
  }
  if (unit_comp.size() > 0xffffffffull) return fail(hipErrorInvalidValue, "program: more than 2^32 tiles");
  ProgArgs &a = p->args;
  memset(&a, 0, sizeof(a));
  a.nunits = unit_comp.size();
  a.nphase = (uint32_t)p->phases.size();
  a.stride = (uint32_t)maxn;
  uint64_t grid = (uint64_t)cus * (small ? kProgSmallBpc : kProgBpc);
  if (p->max_wg && p->max_wg < grid) grid = p->max_wg;
  if (grid > a.nunits) grid = a.nunits;
  p->grid = (uint32_t)(grid ? grid : 1);  // a phases-only program: workgroup 0 alone
  // device block: [desc | ptrs | unit_comp | phases | sig | wait]
  size_t nsig = 0, nwait = 0;
  for (auto &ph : p->phases) {
    nsig += ph.sig.size();
    nwait += ph.wait.size();
  }
  auto al8 = [](size_t x) { return (x + 7) & ~(size_t)7; };
  const size_t o_desc = 0, o_ptrs = al8(o_desc + ncomp * sizeof(PlanDesc));
  const size_t o_uc = al8(o_ptrs + ptrs.size() * sizeof(void *));
  const size_t o_ph = al8(o_uc + unit_comp.size() * sizeof(uint32_t));
  const size_t o_sig = al8(o_ph + p->phases.size() * sizeof(ProgPhase));
  const size_t o_wait = al8(o_sig + nsig * sizeof(void *));
  const size_t bytes = al8(o_wait + nwait * sizeof(void *)) + 8;
  std::vector<char> host(bytes, 0);
  if (ncomp) memcpy(host.data() + o_desc, desc.data(), ncomp * sizeof(PlanDesc));
  if (!ptrs.empty()) memcpy(host.data() + o_ptrs, ptrs.data(), ptrs.size() * sizeof(void *));
  if (!unit_comp.empty()) memcpy(host.data() + o_uc, unit_comp.data(), unit_comp.size() * sizeof(uint32_t));
  {
    ProgPhase *hp = (ProgPhase *)(host.data() + o_ph);
    uint32_t **hs = (uint32_t **)(host.data() + o_sig);
    const uint32_t **hw = (const uint32_t **)(host.data() + o_wait);
    uint32_t si = 0, wi = 0;
    for (size_t i = 0; i < p->phases.size(); i++) {
      auto &ph = p->phases[i];
      hp[i].sig_begin = si;
      for (auto *f : ph.sig) hs[si++] = f;
      hp[i].sig_end = si;
      hp[i].wait_begin = wi;
      for (auto *f : ph.wait) hw[wi++] = f;
      hp[i].wait_end = wi;
    }
  }
  if (int e = check_hip(hipMalloc((void **)&p->d_block, bytes), "program: hipMalloc")) return e;
  if (int e = check_hip(hipMemcpy(p->d_block, host.data(), bytes, hipMemcpyHostToDevice), "program: upload"))
    return e;
  a.desc = (const PlanDesc *)(p->d_block + o_desc);
  a.ptrs = (const char *const *)(p->d_block + o_ptrs);
  a.unit_comp = ncomp > 1 ? (const uint32_t *)(p->d_block + o_uc) : nullptr;
  a.phase = (const ProgPhase *)(p->d_block + o_ph);
  a.sig = (uint32_t *const *)(p->d_block + o_sig);
  a.wait = (const uint32_t *const *)(p->d_block + o_wait);
  a.gate = p->d_gate;
  p->dirty = false;
  return 0;
}

}  // namespace

extern "C" {

int hiccl_program_create(hiccl_program_t **prog, int dtype, int device) {
  if (!prog) return fail(hipErrorInvalidValue, "program_create: prog is NULL");
  *prog = nullptr;
  if (!pick_prog(dtype, 4)) return fail(hipErrorInvalidValue, "program_create: unsupported dtype");
  int ndev = 0;
  if (int e = check_hip(hipGetDeviceCount(&ndev), "program_create: hipGetDeviceCount")) return e;
  if (device < 0 || device >= ndev) return fail(hipErrorInvalidDevice, "program_create: bad device");
  auto *p = new hiccl_program;
  p->dtype = dtype;
  p->device = device;
  *prog = p;
  return 0;
}

int hiccl_program_add_signal(hiccl_program_t *p, uint32_t *const *sig, int nsig, const uint32_t *const *wait,
                             int nwait) {
  if (!p) return fail(hipErrorInvalidValue, "program_add_signal: prog is NULL");
  if (nsig < 0 || nwait < 0 || (nsig && !sig) || (nwait && !wait))
    return fail(hipErrorInvalidValue, "program_add_signal: bad flag lists");
  for (int i = 0; i < nsig; i++)
    if (!sig[i]) return fail(hipErrorInvalidValue, "program_add_signal: NULL signal flag");
  for (int i = 0; i < nwait; i++)
    if (!wait[i]) return fail(hipErrorInvalidValue, "program_add_signal: NULL wait flag");
  if (!p->units.empty())
    return fail(hipErrorInvalidValue, "program_add_signal: phases precede the program's units (start a new program)");
  if (p->phases.size() >= (size_t)kProgMaxPhases)
    return fail(hipErrorInvalidValue, "program_add_signal: more than 64 phases in one program");
  hiccl_program::Phase ph;
  ph.sig.assign(sig, sig + nsig);
  ph.wait.assign(wait, wait + nwait);
  p->phases.push_back(std::move(ph));
  p->dirty = true;
  return 0;
}

int hiccl_program_add_plan(hiccl_program_t *p, const hiccl_reduce_plan_t *plan) {
  if (!p || !plan) return fail(hipErrorInvalidValue, "program_add_plan: NULL argument");
  const bool bytes = plan->dtype == HICCL_BYTES;
  if (!bytes && plan->dtype != p->dtype)
    return fail(hipErrorInvalidValue, "program_add_plan: the plan's dtype is neither the program's nor HICCL_BYTES");
  if (plan->req.acc == HICCL_ACC_WIDE)
    return fail(hipErrorInvalidValue, "program_add_plan: programs accumulate natively (HICCL_ACC_NATIVE) only");
  const int peer = plan_eff_peer(plan);  // the plan's own store form (plan_store_peer) carries over
  for (auto &c : plan->comps) p->units.push_back(hiccl_program::Unit{c.out, c.in, c.count, bytes, peer});
  p->dirty = true;
  return 0;
}

int hiccl_program_set_max_workgroups(hiccl_program_t *p, int max_wg) {
  if (!p) return fail(hipErrorInvalidValue, "program_set_max_workgroups: prog is NULL");
  if (max_wg < 0) return fail(hipErrorInvalidValue, "program_set_max_workgroups: max_wg < 0");
  p->max_wg = (uint32_t)max_wg;
  p->dirty = true;
  return 0;
}

int hiccl_program_num_units(const hiccl_program_t *p) { return p ? (int)p->units.size() : 0; }
int hiccl_program_num_phases(const hiccl_program_t *p) { return p ? (int)p->phases.size() : 0; }

int hiccl_program_launch(hiccl_program_t *p, const uint32_t *epochs, const uint32_t *epoch_dev, uint32_t *err,
                         double timeout_s, void *stream) {
  if (!p) return fail(hipErrorInvalidValue, "program_launch: prog is NULL");
  if (!p->phases.empty() && !epochs) return fail(hipErrorInvalidValue, "program_launch: epochs is NULL");
  if (int e = check_hip(hipSetDevice(p->device), "program_launch: hipSetDevice")) return e;
  if (p->phases.empty() && p->units.empty()) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (int e = prog_upload(p, s)) return e;
  prog_fn fn = pick_prog(p->dtype, p->unroll);
  if (!fn) return fail(hipErrorInvalidValue, "program_launch: no kernel for this dtype / shape");
  ProgArgs a = p->args;
  a.err = err;
  a.epoch_dev = epoch_dev;
  a.timeout_ticks = (uint64_t)((timeout_s > 0 ? timeout_s : 30.0) * 1e8);  // s_memrealtime: 100 MHz
  for (uint32_t i = 0; i < a.nphase; i++) a.epoch[i] = epochs[i];
  a.light = prog_light() ? 1u : 0u;
  // the gate's sequence number: one per eager launch; a captured launch
  // uses seq + *epoch_dev (replay r: seq + r) and reserves every value a
  // 32-bit *epoch_dev can add, so no later launch or re-capture of this
  // program reuses a value one of its replays stores (64-bit: no wrap)
  a.seq = ++p->seq;
  if (epoch_dev) p->seq += (1ull << 32);
  fn(a, dim3(p->grid), s);
  p->enqueued.store(true, std::memory_order_relaxed);
  return check_hip(hipGetLastError(), "program_launch: launch");
}

void hiccl_program_destroy(hiccl_program_t *p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  prog_quiesce(p);
  if (p->d_block) (void)hipFree(p->d_block);
  if (p->d_gate) (void)hipFree(p->d_gate);
  delete p;
}

int hiccl_token_mode(void) { return prog_light() ? HICCL_TOKENS_LIGHT : HICCL_TOKENS_FENCED; }

// "1" / yes / on / true (any case) opt in; "0" / no / off / false / unset
// keep the default (off).  Round 3 read any value but "0" as on: a value
// that is neither spelling is read as off and named once on stderr, so a job
// script's protocol never changes without a word.
int hiccl_step_program_default(void) {
  const char *e = std::getenv("HICCL_STEP_PROGRAM");
  if (!e) return 0;
  std::string v(e);
  for (auto &ch : v) ch = (char)std::tolower((unsigned char)ch);
  if (v == "1" || v == "yes" || v == "on" || v == "true") return 1;
  if (!(v.empty() || v == "0" || v == "no" || v == "off" || v == "false")) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      std::fprintf(stderr, "HiCCL: HICCL_STEP_PROGRAM=%s not recognised (1/yes/on/true or 0/no/off/false); "
                           "step programs stay off\n", e);
  }
  return 0;
}

// ---------------------------------------------------------- measurement --

int hiccl_fill_uniform(int dtype, void *out, size_t count, uint64_t seed, uint32_t k, size_t first,
                       void *stream) {
  if (count == 0) return 0;
  if (!out) return fail(hipErrorInvalidValue, "fill_uniform: out is NULL");
  // Same key derivation as oracle/reduce_oracle.c hash3(): splitmix64(seed ^ k<<48) + i.
  uint64_t z = seed ^ ((uint64_t)k << 48);
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  const uint64_t key = z ^ (z >> 31);
  uint64_t blocks = (count + 255) / 256;
  const uint64_t cap = (uint64_t)device_cus(current_device()) * 16;
  if (blocks > cap) blocks = cap;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case HICCL_FLOAT32:
      hipLaunchKernelGGL(k_fill<HICCL_FLOAT32>, dim3((unsigned)blocks), dim3(256), 0, s, (char *)out,
                         (uint64_t)count, key, (uint64_t)first);
      break;
    case HICCL_FLOAT64:
      hipLaunchKernelGGL(k_fill<HICCL_FLOAT64>, dim3((unsigned)blocks), dim3(256), 0, s, (char *)out,
                         (uint64_t)count, key, (uint64_t)first);
      break;
    case HICCL_BFLOAT16:
      hipLaunchKernelGGL(k_fill<HICCL_BFLOAT16>, dim3((unsigned)blocks), dim3(256), 0, s, (char *)out,
                         (uint64_t)count, key, (uint64_t)first);
      break;
    default: return fail(hipErrorInvalidValue, "fill_uniform: dtype must be FLOAT32/FLOAT64/BFLOAT16");
  }
  return check_hip(hipGetLastError(), "fill_uniform: launch");
}

int hiccl_device_info(int device, int *cus, int *mem_clock_khz, int *bus_width_bits) {
  int v = 0;
  if (cus) {
    if (int e = check_hip(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, device), "device_info: CUs"))
      return e;
    *cus = v;
  }
  if (mem_clock_khz) {
    if (int e = check_hip(hipDeviceGetAttribute(&v, hipDeviceAttributeMemoryClockRate, device), "device_info: clock"))
      return e;
    *mem_clock_khz = v;
  }
  if (bus_width_bits) {
    if (int e = check_hip(hipDeviceGetAttribute(&v, hipDeviceAttributeMemoryBusWidth, device), "device_info: bus"))
      return e;
    *bus_width_bits = v;
  }
  return 0;
}

int hiccl_stream_copy(void *dst, const void *src, size_t bytes, void *stream) {
  if (bytes == 0) return 0;
  if (!dst || !src) return fail(hipErrorInvalidValue, "stream_copy: NULL pointer");
  if ((uintptr_t)dst % 16 || (uintptr_t)src % 16)
    return fail(hipErrorInvalidValue, "stream_copy: pointers must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  const uint64_t npkt = bytes / 16;
  if (npkt) {
    uint64_t blocks = (npkt + 1023) / 1024;
    const uint64_t cap = (uint64_t)device_cus(current_device()) * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, s, (u32x4 *)dst,
                       (const u32x4 *)src, npkt);
  }
  if (bytes % 16)
    hipLaunchKernelGGL(k_copy_bytes, dim3(1), dim3(64), 0, s, (char *)dst + npkt * 16,
                       (const char *)src + npkt * 16, (uint64_t)(bytes % 16));
  return check_hip(hipGetLastError(), "stream_copy: launch");
}

// ---- bucket layout
//
// A reduction bucket -- n inputs and the output of one compute -- in ONE
// device allocation, buffer j (inputs 0..n-1, then the output) at
// j x stride, stride = the buffer rounded up to 64 KiB plus 64 KiB.  Measured
// on config 2 (tools/alloc_probe.py; profiles/r06d_alloc.jsonl, r06e_, r06f_,
// r06h_): the same kernel on nine separate hipMalloc'd buffers (torch.empty,
// hipMalloc, hipDeviceMallocContiguous) runs 1.43-1.56 ms depending on the
// allocation -- up to 9 % apart in one process, although every buffer alone
// reads and writes at the same rate -- while buckets in one allocation at
// 1 GiB + 0-4 MiB strides ran 1.424-1.462 ms, every one of 28 instances on
// fresh devices (the 64-128 KiB staggers fastest).  Separate allocations
// leave the streams' relative physical placement to chance; one allocation
// fixes it.  Which physical memory the allocation gets still matters: on a
// device whose free memory was fragmented first, later buckets can be as
// slow as separate buffers (r06l_alloc.jsonl).
static uint64_t bucket_stride(size_t bytes) {
  const uint64_t g = 64ull << 10;
  return (((uint64_t)bytes + g - 1) / g) * g + g;
}

size_t hiccl_bucket_stride(int dtype, size_t count) {
  const size_t esz = esize(dtype);
  return esz && count ? (size_t)bucket_stride(count * esz) : 0;
}

int hiccl_bucket_alloc(int dtype, int n, size_t count, int device, void **base, void **in, void **out) {
  const size_t esz = esize(dtype);
  if (!esz) return fail(hipErrorInvalidValue, "bucket_alloc: unknown dtype");
  if (n < 0 || n > (1 << 20)) return fail(hipErrorInvalidValue, "bucket_alloc: n out of range");
  if (!count) return fail(hipErrorInvalidValue, "bucket_alloc: count must be > 0");
  if (!base || !out || (n > 0 && !in)) return fail(hipErrorInvalidValue, "bucket_alloc: NULL output argument");
  *base = nullptr;
  int prev = 0;
  if (int e = check_hip(hipGetDevice(&prev), "bucket_alloc: hipGetDevice")) return e;
  if (int e = check_hip(hipSetDevice(device), "bucket_alloc: hipSetDevice")) return e;
  const uint64_t stride = bucket_stride(count * esz);
  char *b = nullptr;
  const int e = check_hip(hipMalloc((void **)&b, (size_t)(stride * (uint64_t)(n + 1))), "bucket_alloc: hipMalloc");
  (void)hipSetDevice(prev);  // the caller's current device is left as it was
  if (e) return e;
  for (int k = 0; k < n; k++) in[k] = b + (uint64_t)k * stride;
  *out = b + (uint64_t)n * stride;
  *base = b;
  return 0;
}

int hiccl_bucket_free(void *base) {
  if (!base) return 0;
  return check_hip(hipFree(base), "bucket_free: hipFree");
}

}  // extern "C"
