// tools/hbm_probe.hip -- bench-only HBM micro-probes (not part of the product).
//
// Measures what the MI355X memory system delivers for the access mixes the
// reduction stage is made of, so the reduction kernel can be judged against
// an achievable ceiling and not only the 8 TB/s spec:
//   read   : N streams read, nothing written (one dword per workgroup)
//   write  : one stream written
//   mix    : N streams read + 1 written (the reduction's traffic, no adds)
// Each in several forms: global_load (flat 64-bit), buffer_load (SGPR
// descriptor), nt / default policy, block and unroll variants, LDS-DMA.
//
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libhbm_probe.so tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t mk(const void *p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)n, 0x00020000);
}

struct Ptrs {
  const char *in[64];
  char *out;
  uint64_t bytes;  // per stream
  int n;
};

// Mix kernel: N reads + 1 write per packet (XOR instead of add: no FP cost).
// AUXL / AUXS: cache-policy bits of loads / stores (gfx950: 1 sc0, 2 nt, 16 sc1).
// ORDER 0: loads issued input-major (all U packets of input j, then j+1);
// ORDER 1: packet-major.
template <int B, int U, int AUXL, int AUXS, int ORDER, bool WRITE, bool READ>
__global__ __launch_bounds__(B) void k_mix(Ptrs p) {
  const uint64_t tile = (uint64_t)B * U * 16;
  const uint64_t ntiles = p.bytes / tile;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (u * B + threadIdx.x) * 16;
  u32x4 sink = (u32x4)(0u);
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t off = t * tile;
    u32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) acc[u] = (u32x4)(0u);
    if (READ) {
      for (int g = 0; g < p.n; g += 8) {
        u32x4 x[8][U];
        rsrc_t r[8];
#pragma unroll
        for (int j = 0; j < 8; j++)
          r[j] = mk(p.in[(g + j) < p.n ? g + j : 0] + off, (g + j) < p.n ? (uint32_t)tile : 0u);
        if (ORDER != 1) {
#pragma unroll
          for (int j = 0; j < 8; j++)
#pragma unroll
            for (int u = 0; u < U; u++) x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r[j], voff[u], 0, AUXL);
        } else {
#pragma unroll
          for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < 8; j++) x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r[j], voff[u], 0, AUXL);
        }
        if (ORDER == 2) __builtin_amdgcn_sched_barrier(0);  // all loads before any use
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
          for (int u = 0; u < U; u++) acc[u] ^= x[j][u];
      }
    }
    if (WRITE) {
      rsrc_t w = mk(p.out + off, (uint32_t)tile);
#pragma unroll
      for (int u = 0; u < U; u++) {
        u32x4 v = READ ? acc[u] : (u32x4)((uint32_t)(off + voff[u]));
        __builtin_amdgcn_raw_buffer_store_b128(v, w, voff[u], 0, AUXS);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) sink ^= acc[u];
    }
  }
  if (!WRITE && sink.x == 0x12345678u && sink.y == 0x9abcdef0u) p.out[threadIdx.x] = 1;
}

// LDS-DMA mix: each wave streams its inputs into LDS with global_load_lds
// (16 B/lane), then reads them back (ds_read_b128) and writes the XOR.
template <int B, int AUX>
__global__ __launch_bounds__(B) void k_mix_lds(Ptrs p) {
  constexpr int W = B / 64;
  __shared__ u32x4 lds[8][B];  // one 16-B packet per lane per input
  const uint64_t tile = (uint64_t)B * 16;
  const uint64_t ntiles = p.bytes / tile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  (void)W;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t off = t * tile;
    for (int j = 0; j < p.n && j < 8; j++) {
      const char *src = p.in[j] + off + (uint64_t)threadIdx.x * 16;
      __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)&lds[j][wave * 64], 16, 0, AUX);
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) & lgkmcnt(0)
    u32x4 acc = (u32x4)(0u);
    for (int j = 0; j < p.n && j < 8; j++) acc ^= lds[j][threadIdx.x];
    rsrc_t w = mk(p.out + off, (uint32_t)tile);
    __builtin_amdgcn_raw_buffer_store_b128(acc, w, threadIdx.x * 16, 0, 0);
  }
}

// Grouped mix (mode 4, n <= 8): a workgroup reads G consecutive tiles (all
// n inputs of a tile in flight, XOR into acc[g]) and stores the G tiles
// together after the last one's reads, so its writes come in bursts of
// G tiles.  G = 1 is the plain mix order.  nt loads and nt stores.
template <int B, int U, int G>
__global__ __launch_bounds__(B) void k_mix_grp(Ptrs p) {
  const uint64_t tile = (uint64_t)B * U * 16;
  const uint64_t ntiles = p.bytes / tile;
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; u++) voff[u] = (u * B + threadIdx.x) * 16;
  for (uint64_t t0 = (uint64_t)blockIdx.x * G; t0 < ntiles; t0 += (uint64_t)gridDim.x * G) {
    u32x4 acc[G][U];
#pragma unroll
    for (int g = 0; g < G; g++) {
      const uint64_t off = (t0 + g) * tile;
      const bool live = t0 + g < ntiles;
      u32x4 x[8][U];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        rsrc_t r = mk(p.in[j < p.n ? j : 0] + (live ? off : 0), (live && j < p.n) ? (uint32_t)tile : 0u);
#pragma unroll
        for (int u = 0; u < U; u++) x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r, voff[u], 0, 2);
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc[g][u] = x[0][u];
#pragma unroll
        for (int j = 1; j < 8; j++) acc[g][u] ^= x[j][u];
      }
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
      const bool live = t0 + g < ntiles;
      rsrc_t w = mk(p.out + (live ? (t0 + g) * tile : 0), live ? (uint32_t)tile : 0u);
#pragma unroll
      for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(acc[g][u], w, voff[u], 0, 2);
    }
  }
}

template <class K>
static int launch(K kern, int grid, int block, Ptrs p, hipStream_t s) {
  hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, s, p);
  return (int)hipGetLastError();
}

template <int B, int U, int AL, int AS, int O>
static int run_mix(int mode, int grid, Ptrs p, hipStream_t s) {
  if (mode == 0) return launch(k_mix<B, U, AL, AS, O, true, true>, grid, B, p, s);
  if (mode == 1) return launch(k_mix<B, U, AL, AS, O, false, true>, grid, B, p, s);
  if (mode == 2) return launch(k_mix<B, U, AL, AS, O, true, false>, grid, B, p, s);
  return -1;
}

template <int B, int U, int AL, int AS>
static int run_o(int o, int mode, int grid, Ptrs p, hipStream_t s) {
  if (o == 2) return run_mix<B, U, AL, AS, 2>(mode, grid, p, s);
  return o ? run_mix<B, U, AL, AS, 1>(mode, grid, p, s) : run_mix<B, U, AL, AS, 0>(mode, grid, p, s);
}

template <int B, int U, int AL>
static int run_as(int as, int o, int mode, int grid, Ptrs p, hipStream_t s) {
  switch (as) {
    case 0: return run_o<B, U, AL, 0>(o, mode, grid, p, s);
    case 2: return run_o<B, U, AL, 2>(o, mode, grid, p, s);
    case 16: return run_o<B, U, AL, 16>(o, mode, grid, p, s);
    case 17: return run_o<B, U, AL, 17>(o, mode, grid, p, s);
  }
  return -1;
}

template <int B, int U>
static int run_al(int al, int as, int o, int mode, int grid, Ptrs p, hipStream_t s) {
  switch (al) {
    case 0: return run_as<B, U, 0>(as, o, mode, grid, p, s);
    case 2: return run_as<B, U, 2>(as, o, mode, grid, p, s);
    case 16: return run_as<B, U, 16>(as, o, mode, grid, p, s);
  }
  return -1;
}

template <int B>
static int run_u(int u, int al, int as, int o, int mode, int grid, Ptrs p, hipStream_t s) {
  switch (u) {
    case 1: return run_al<B, 1>(al, as, o, mode, grid, p, s);
    case 2: return run_al<B, 2>(al, as, o, mode, grid, p, s);
    case 4: return run_al<B, 4>(al, as, o, mode, grid, p, s);
    case 8: return run_al<B, 8>(al, as, o, mode, grid, p, s);
  }
  return -1;
}

extern "C" {
// mode: 0 mix (N reads + 1 write), 1 read-only, 2 write-only, 3 LDS-DMA mix
int probe_run(int mode, int block, int unroll, int aux_load, int aux_store, int order, int grid,
              const void *const *in, int n, void *out, uint64_t bytes, void *stream) {
  // the kernels read p.in[0..n): at most 64 streams (at most 8 for the LDS
  // and grouped mixes, whose loads are unrolled over 8 inputs; fewer read
  // zeros through empty descriptors), as many as config 3's largest bucket
  if (n < 1 || n > 64 || ((mode == 3 || mode == 4) && n > 8)) return -1;
  Ptrs p;
  for (int k = 0; k < 64; k++) p.in[k] = (const char *)(k < n ? in[k] : in[0]);
  p.out = (char *)out;
  p.bytes = bytes;
  p.n = n;
  hipStream_t s = (hipStream_t)stream;
  if (mode == 4) {  // grouped mix: unroll = U, order = G
    if (block != 256) return -1;
    const int key = unroll * 10 + order;
    switch (key) {
      case 41: return launch(k_mix_grp<256, 4, 1>, grid, 256, p, s);
      case 42: return launch(k_mix_grp<256, 4, 2>, grid, 256, p, s);
      case 22: return launch(k_mix_grp<256, 2, 2>, grid, 256, p, s);
      case 24: return launch(k_mix_grp<256, 2, 4>, grid, 256, p, s);
      case 14: return launch(k_mix_grp<256, 1, 4>, grid, 256, p, s);
      case 18: return launch(k_mix_grp<256, 1, 8>, grid, 256, p, s);
    }
    return -1;
  }
  if (mode == 3) {
    if (block == 256) return aux_load ? launch(k_mix_lds<256, 2>, grid, 256, p, s)
                                      : launch(k_mix_lds<256, 0>, grid, 256, p, s);
    return launch(k_mix_lds<512, 0>, grid, 512, p, s);
  }
  switch (block) {
    case 256: return run_u<256>(unroll, aux_load, aux_store, order, mode, grid, p, s);
    case 512: return run_u<512>(unroll, aux_load, aux_store, order, mode, grid, p, s);
    case 1024: return run_u<1024>(unroll, aux_load, aux_store, order, mode, grid, p, s);
  }
  return -1;
}
}
