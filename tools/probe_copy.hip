// probe_copy.hip - ceiling of a plain HBM -> HBM copy (diagnostic, NOT product
// code): the bound of the TX build of 1514-B frames, which is a copy plus
// header writes. Grid-stride loops over 16-byte pieces, U pieces per lane in
// flight, default or non-temporal loads / stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = i0 + 256ull * u;
      v[u] = i < n ? (NTL ? __builtin_nontemporal_load(a + i) : a[i]) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = i0 + 256ull * u;
      if (i < n) {
        if (NTS) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

typedef void (*kfn)(const u32x4*, u32x4*, uint64_t);
static const kfn k_tab[] = {k_copy<1, false, false>, k_copy<4, false, false>, k_copy<4, false, true>,
                            k_copy<4, true, true>, k_copy<8, false, true>, k_copy<8, true, false>,
                            k_copy<2, false, true>};
extern "C" const char* pc_name(int w) {
  static const char* nm[] = {"u1", "u4", "u4_nts", "u4_ntl_nts", "u8_nts", "u8_ntl", "u2_nts"};
  return nm[w];
}
extern "C" int pc_count(void) { return 7; }
extern "C" int pc_launch(int w, const void* a, void* b, uint64_t n16, uint32_t grid, void* stream) {
  hipLaunchKernelGGL(k_tab[w], dim3(grid), dim3(256), 0, (hipStream_t)stream, (const u32x4*)a, (u32x4*)b, n16);
  return (int)hipGetLastError();
}
