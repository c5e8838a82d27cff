// probe_stream.hip - calibration kernels for the memory ceiling of the RX
// byte pattern (diagnostic, NOT product code). Persistent grid-stride loops.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT_LD, bool NT_ST>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if (NT_LD) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT_ST>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if (NT_ST) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// mode bits: 1 = read frames, 2 = write records, 4 = read len
template <bool NT_LD, bool NT_ST, int MODE>
__global__ void __launch_bounds__(256) probe_lane(const uint8_t* base, const uint16_t* len, u32x4* out, uint32_t n,
                                                  uint32_t S) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    u32x4 a = {i, 0u, 0u, 0u};
    if (MODE & 1) {
      const u32x4* f = (const u32x4*)(base + (uint64_t)i * S);
      a = ld<NT_LD, NT_ST>(f) ^ ld<NT_LD, NT_ST>(f + 1) ^ ld<NT_LD, NT_ST>(f + 2) ^ ld<NT_LD, NT_ST>(f + 3);
    }
    if (MODE & 4) a.x += len[i];
    if (MODE & 2) st<NT_ST>(out + i, a);
    else if (a.x == 0x12345678u && a.y == 0x9abcdefu) out[0] = a;
  }
}

typedef void (*kfn)(const uint8_t*, const uint16_t*, u32x4*, uint32_t, uint32_t);
static const kfn k_tab[] = {
    probe_lane<false, false, 7>, probe_lane<true, false, 7>, probe_lane<false, true, 7>, probe_lane<true, true, 7>,
    probe_lane<false, false, 1>, probe_lane<true, false, 1>, probe_lane<false, false, 2>, probe_lane<false, true, 2>,
};
extern "C" const char* probe_name(int w) {
  static const char* nm[] = {"rw", "rw_ntld", "rw_ntst", "rw_ntboth", "read_only", "read_only_nt", "write_only",
                             "write_only_nt"};
  return nm[w];
}
extern "C" int probe_count(void) { return 8; }
extern "C" int probe_launch(int which, const void* base, const void* len, void* out, uint32_t n, uint32_t S,
                            uint32_t grid, void* stream) {
  hipLaunchKernelGGL(k_tab[which], dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint8_t*)base,
                     (const uint16_t*)len, (u32x4*)out, n, S);
  return (int)hipGetLastError();
}
