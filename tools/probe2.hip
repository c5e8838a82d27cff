// probe2.hip - HBM ceiling for read/write mixes (diagnostic, NOT product code).
// All kernels: persistent grid-stride over items, 256 threads per block.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

// plain float4 copy, U items per thread per iteration (loads first)
template <int U>
__global__ void __launch_bounds__(256) k_copy(const u32x4* in, u32x4* out, uint32_t n) {
  const uint32_t T = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += T * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = (i + u * T < n) ? in[i + u * T] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; u++)
      if (i + u * T < n) out[i + u * T] = v[u];
  }
}

// C2 mix: item = S-byte frame (4-aligned) read as 4 x 16 B, + 16-B record written
template <int U>
__global__ void __launch_bounds__(256) k_mix(const uint8_t* base, u32x4* out, uint32_t n, uint32_t S) {
  const uint32_t T = gridDim.x * 256;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += T * U) {
    u32x4 a[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t k = i + u * T < n ? i + u * T : n - 1;
      const u32x4_a4* f = (const u32x4_a4*)(base + (uint64_t)k * S);
      a[u] = f[0] ^ f[1] ^ f[2] ^ f[3];
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (i + u * T < n) out[i + u * T] = a[u];
  }
}

// C2 mix, wave-coalesced: a wave owns 64 consecutive frames; reads their
// contiguous 64*S bytes with aligned 16-B lane loads, writes 64 records
template <int S>
__global__ void __launch_bounds__(256) k_mixw(const uint8_t* base, u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = n / 64;
  constexpr int P = (64 * S) / 1024;  // full 1 KiB wave pieces
  constexpr int R = (64 * S) % 1024;
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += nw) {
    const u32x4* f = (const u32x4*)(base + (uint64_t)c * 64 * S);
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < P; k++) acc ^= f[k * 64 + lane];
    if (R && lane * 16 < R) acc ^= f[P * 64 + lane];
    out[(uint64_t)c * 64 + lane] = acc;
  }
}

typedef void (*launch_fn)(const void*, void*, uint32_t, uint32_t, uint32_t, hipStream_t);
static void copy1(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_copy<1>, dim3(g), dim3(256), 0, s, (const u32x4*)a, (u32x4*)b, n); }
static void copy4(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_copy<4>, dim3(g), dim3(256), 0, s, (const u32x4*)a, (u32x4*)b, n); }
static void mix1(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mix<1>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (u32x4*)b, n, S); }
static void mix2(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mix<2>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (u32x4*)b, n, S); }
static void mixw60(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mixw<60>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (u32x4*)b, n); }
static void mixw64(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mixw<64>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (u32x4*)b, n); }

// mixw60 + per-frame u16 length load (the descriptor)
__global__ void __launch_bounds__(256) k_mixw_len(const uint8_t* base, const uint16_t* len, u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = n / 64;
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += nw) {
    const u32x4* f = (const u32x4*)(base + (uint64_t)c * 64 * 60);
    u32x4 acc = {len[c * 64 + lane], 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 3; k++) acc ^= f[k * 64 + lane];
    if (lane < 48) acc ^= f[3 * 64 + lane];
    out[(uint64_t)c * 64 + lane] = acc;
  }
}

// + LDS transpose: each lane reads its frame's dwords 3..15 back
template <bool PF>
__global__ void __launch_bounds__(256) k_mixw_lds(const uint8_t* base, const uint16_t* len, u32x4* out, uint32_t n) {
  __shared__ uint32_t buf[4][1024];
  const int lane = threadIdx.x & 63;
  uint32_t* b = buf[threadIdx.x >> 6];
  const uint32_t nw = gridDim.x * 4, nch = n / 64;
  uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nch) return;
  u32x4 v[4];
  uint32_t L;
  auto issue = [&](uint32_t cc, u32x4 (&w)[4], uint32_t& l) {
    const uint32_t ck = cc < nch ? cc : nch - 1;
    const u32x4* f = (const u32x4*)(base + (uint64_t)ck * 64 * 60);
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = f[k * 64 + lane];
    l = len[ck * 64 + lane];
  };
  issue(c, v, L);
  for (;;) {
    u32x4 nv[4];
    uint32_t nL = 0;
    if (PF) issue(c + nw, nv, nL);
#pragma unroll
    for (int k = 0; k < 4; k++) *(u32x4*)(b + 4 * (lane + 64 * k)) = v[k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    u32x4 acc = {L, 0, 0, 0};
#pragma unroll
    for (int j = 3; j < 16; j++) acc.x ^= b[lane * 15 + j] << (j & 7);
    out[(uint64_t)c * 64 + lane] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    c += nw;
    if (c >= nch) break;
    if (PF) {
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = nv[k];
      L = nL;
    } else {
      issue(c, v, L);
    }
  }
}
static void mixwlen(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mixw_len, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (const uint16_t*)a, (u32x4*)b, n); }
static void mixwlds(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mixw_lds<false>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (const uint16_t*)a, (u32x4*)b, n); }
static void mixwldspf(const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, hipStream_t s) {
  hipLaunchKernelGGL(k_mixw_lds<true>, dim3(g), dim3(256), 0, s, (const uint8_t*)a, (const uint16_t*)a, (u32x4*)b, n); }

static const launch_fn tab[] = {copy1, copy4, mix1, mix2, mixw60, mixw64, mixwlen, mixwlds, mixwldspf};
static const char* names[] = {"copy1", "copy4", "mix1", "mix2", "mixw60", "mixw64", "mxlen60", "mxlds60", "mxldspf60"};
extern "C" int p2_count(void) { return 9; }
extern "C" const char* p2_name(int w) { return names[w]; }
extern "C" int p2_launch(int w, const void* a, void* b, uint32_t n, uint32_t S, uint32_t g, void* s) {
  tab[w](a, b, n, S, g, (hipStream_t)s);
  return (int)hipGetLastError();
}
