// probe_c2mem.hip - the C2 memory pattern alone (diagnostic, NOT product
// code): per 64-frame chunk a wave reads the chunk's 3840 contiguous bytes
// (4 non-temporal 16-byte loads per lane) and its 64 lengths, and writes 64
// 16-byte records (non-temporal), with no parse. AHEAD chunks are in flight
// per wave (register ring), grid-stride over a persistent grid of G blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// RUN: the wave's k-th chunk is ((k / RUN) nw + w) RUN + k % RUN (the
// product's coalesced kernel uses RUN = 2)
template <int AHEAD, int RUN = 1>
__global__ void __launch_bounds__(256) k_c2(const uint8_t* base, const uint16_t* len, u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = n / 64;
  const uint32_t w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
  auto chunk_of = [&](uint32_t k) -> uint32_t {
    const uint64_t c = ((uint64_t)(k / RUN) * nw + w0) * RUN + k % RUN;
    return c < nch ? (uint32_t)c : nch;
  };
  uint32_t kk = 0, c = chunk_of(0);
  if (c >= nch) return;
  u32x4 v[AHEAD + 1][4];
  uint32_t L[AHEAD + 1];
  auto issue = [&](uint32_t cc, u32x4 (&w)[4], uint32_t& l) {
    const uint32_t ck = cc < nch ? cc : nch - 1;
    const uint8_t* f = base + (uint64_t)ck * 3840u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t o = 16u * (uint32_t)(lane + 64 * k);
      w[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(f + (o < 3824u ? o : 3824u)));
    }
    l = len[ck * 64u + lane];
  };
#pragma unroll
  for (int a = 0; a <= AHEAD; a++) issue(chunk_of(a), v[a], L[a]);
  for (;;) {
    u32x4 acc = v[0][0] ^ v[0][1] ^ v[0][2] ^ v[0][3];
    acc.x ^= L[0];
    __builtin_nontemporal_store(acc, out + (uint64_t)c * 64u + lane);
    c = chunk_of(++kk);
    if (c >= nch) break;
#pragma unroll
    for (int a = 0; a < AHEAD; a++) {
#pragma unroll
      for (int k = 0; k < 4; k++) v[a][k] = v[a + 1][k];
      L[a] = L[a + 1];
    }
    issue(chunk_of(kk + AHEAD), v[AHEAD], L[AHEAD]);
  }
}

extern "C" int pm_count(void) { return 7; }
extern "C" int pm_launch(int w, const void* base, const void* len, void* out, uint32_t n, uint32_t grid, void* s) {
  const uint8_t* b = (const uint8_t*)base;
  const uint16_t* l = (const uint16_t*)len;
  u32x4* o = (u32x4*)out;
  hipStream_t st = (hipStream_t)s;
  if (w == 0) hipLaunchKernelGGL(k_c2<0>, dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 1) hipLaunchKernelGGL(k_c2<1>, dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 2) hipLaunchKernelGGL(k_c2<2>, dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 3) hipLaunchKernelGGL(k_c2<3>, dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 4) hipLaunchKernelGGL((k_c2<1, 2>), dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 5) hipLaunchKernelGGL((k_c2<2, 2>), dim3(grid), dim3(256), 0, st, b, l, o, n);
  if (w == 6) hipLaunchKernelGGL((k_c2<3, 2>), dim3(grid), dim3(256), 0, st, b, l, o, n);
  return (int)hipGetLastError();
}
