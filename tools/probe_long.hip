// probe_long.hip - memory ceiling of the long-frame (C4) byte pattern for
// three read decompositions (diagnostic, NOT product code). Every kernel
// reads every byte of n frames of L bytes at stride S and writes one 16-byte
// record per frame. Persistent grid, wave per chunk of 64 frames.
//   span:   the wave reads the chunk's contiguous 64*S bytes, 16 B per lane per
//           load, U loads in flight (fully coalesced), then per-frame sums via LDS
//   group:  16 lanes per frame, 4 frames per round, 16 B per lane per load
//   prefix: lane per frame reads bytes 0..95 first (the product's pass A),
//           then the group rounds stream [96, L)
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
  if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4_a4*>(p);
}

__device__ __forceinline__ uint32_t hsum(u32x4 v) { return v.x + v.y + v.z + v.w; }

template <int U, bool NT, bool ATOM = true>
__global__ void __launch_bounds__(256) k_span(const uint8_t* base, u32x4* out, uint32_t n, uint32_t L, uint32_t S) {
  __shared__ uint32_t acc[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  for (uint32_t c = blockIdx.x * 4 + wv; c < nch; c += nw) {
    acc[wv][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    const uint32_t f0 = c * 64, nf = n - f0 < 64 ? n - f0 : 64;
    const uint64_t s0 = (uint64_t)f0 * S, bytes = (uint64_t)(nf - 1) * S + L;
    const uint32_t npc = (uint32_t)((bytes + 15) / 16);
    uint32_t mine = 0;
    for (uint32_t q0 = 0; q0 < npc; q0 += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q = q0 + 64 * u + lane;
        v[u] = ld<NT>(base + s0 + 16ull * (q < npc ? q : npc - 1));
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q = q0 + 64 * u + lane;
        const uint32_t fr = (16 * q) / S;  // owning frame (pieces straddling go to the first)
        if (!ATOM) mine += hsum(v[u]);
        else if (q < npc) atomicAdd(&acc[wv][fr < 64 ? fr : 63], hsum(v[u]));
      }
    }
    __builtin_amdgcn_wave_barrier();
    if ((uint32_t)lane < nf) out[f0 + lane] = u32x4{acc[wv][lane] + mine, f0 + lane, 0u, 0u};
    __builtin_amdgcn_wave_barrier();
  }
}

// group: pieces from byte B0; PRE: lane-per-frame prefix load of 0..95 first
template <int T, bool PRE>
__global__ void __launch_bounds__(256) k_group(const uint8_t* base, u32x4* out, uint32_t n, uint32_t L, uint32_t S) {
  __shared__ uint32_t sm[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane / 16, gl = lane % 16;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  const uint32_t B0 = PRE ? 96u : 0u;
  for (uint32_t c = blockIdx.x * 4 + wv; c < nch; c += nw) {
    const uint32_t f0 = c * 64;
    uint32_t pre = 0;
    if (PRE) {
      const uint32_t i = f0 + lane < n ? f0 + lane : n - 1;
      const uint8_t* f = base + (uint64_t)i * S;
      u32x4 a = ld<false>(f) ^ ld<false>(f + 16) ^ ld<false>(f + 32);
      a ^= ld<false>(f + 48) ^ ld<false>(f + 64) ^ ld<false>(f + 80);
      pre = hsum(a);
    }
    for (uint32_t r = 0; r < 16; r++) {
      const uint32_t fi = f0 + r * 4 + g;
      const uint8_t* f = base + (uint64_t)(fi < n ? fi : n - 1) * S;
      uint32_t a = 0;
      for (uint32_t p0 = B0; p0 < L; p0 += 16 * 16 * T) {
        u32x4 v[T];
#pragma unroll
        for (int t = 0; t < T; t++) {
          const uint32_t pos = p0 + 16 * gl + 256 * t;
          v[t] = ld<false>(f + (pos < L ? pos : 0));
        }
#pragma unroll
        for (int t = 0; t < T; t++) a += hsum(v[t]);
      }
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) a += __shfl_xor(a, m, 16);
      if (gl == 0) sm[wv][r * 4 + g] = a;
    }
    __builtin_amdgcn_wave_barrier();
    if (f0 + lane < n) out[f0 + lane] = u32x4{sm[wv][lane] + pre, f0 + lane, 0u, 0u};
    __builtin_amdgcn_wave_barrier();
  }
}

typedef void (*kfn)(const uint8_t*, u32x4*, uint32_t, uint32_t, uint32_t);
static const kfn k_tab[] = {k_span<4, false>, k_span<8, false>, k_span<8, true>, k_span<16, false>, k_span<8, false, false>,
                            k_group<8, false>, k_group<8, true>, k_group<4, false>};
extern "C" const char* pl_name(int w) {
  static const char* nm[] = {"span_u4", "span_u8", "span_u8_nt", "span_u16", "span_u8_noatom", "group_t8", "prefix_group_t8",
                             "group_t4"};
  return nm[w];
}
extern "C" int pl_count(void) { return 8; }
extern "C" int pl_launch(int which, const void* base, void* out, uint32_t n, uint32_t L, uint32_t S, uint32_t grid,
                         void* stream) {
  hipLaunchKernelGGL(k_tab[which], dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)base, (u32x4*)out,
                     n, L, S);
  return (int)hipGetLastError();
}
