// probe_c3.hip - memory ceiling of C3's byte pattern (packed IMIX frames,
// u64 offsets) for two whole-span read decompositions (diagnostic, NOT
// product code). A wave takes a chunk of 64 frames and reads the chunk's
// contiguous span [off[f0] & ~15, off[f0 + 63] + len[f0 + 63]):
//   reg:  16 B per lane per load, U loads in flight, summed in registers
//   lds:  staged HBM -> LDS with global_load_lds in 4 KiB windows, two
//         buffers per wave (window w + 1 in flight while w is read), each
//         lane reading its own 64 contiguous bytes of the window from LDS
// Both write one 16-byte record per frame. Times are compared with the
// product's C3 launch by tools/probe_c3.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint32_t hsum(u32x4 v) { return v.x + v.y + v.z + v.w; }

__device__ __forceinline__ void span_of(const uint64_t* off, const uint16_t* len, uint32_t n, uint32_t c,
                                        uint64_t& b, uint32_t& bytes) {
  const uint32_t f0 = c * 64, fl = f0 + 63 < n ? f0 + 63 : n - 1;
  b = off[f0] & ~15ull;
  bytes = (uint32_t)(off[fl] + len[fl] - b);
}

template <int U>
__global__ void __launch_bounds__(256) k_reg(const uint8_t* base, const uint64_t* off, const uint16_t* len,
                                             u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nch; c += nw) {
    uint64_t b;
    uint32_t bytes;
    span_of(off, len, n, c, b, bytes);
    const uint32_t npc = (bytes + 15) / 16;
    uint32_t a = 0;
    for (uint32_t q0 = 0; q0 < npc; q0 += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q = q0 + 64 * u + lane;
        v[u] = *reinterpret_cast<const u32x4*>(base + b + 16ull * (q < npc ? q : npc - 1));
      }
#pragma unroll
      for (int u = 0; u < U; u++) a += hsum(v[u]);
    }
    const uint32_t i = c * 64 + lane;
    if (i < n) out[i] = u32x4{a, i, 0u, 0u};
  }
}

// reg with the next chunk's span descriptors loaded one chunk ahead
template <int U>
__global__ void __launch_bounds__(256) k_reg2(const uint8_t* base, const uint64_t* off, const uint16_t* len,
                                              u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nch) return;
  uint64_t b;
  uint32_t bytes;
  span_of(off, len, n, c, b, bytes);
  for (;;) {
    const uint32_t cn = c + nw;
    uint64_t bn = 0;
    uint32_t bytesn = 0;
    if (cn < nch) span_of(off, len, n, cn, bn, bytesn);
    const uint32_t npc = (bytes + 15) / 16;
    uint32_t a = 0;
    for (uint32_t q0 = 0; q0 < npc; q0 += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q = q0 + 64 * u + lane;
        v[u] = *reinterpret_cast<const u32x4*>(base + b + 16ull * (q < npc ? q : npc - 1));
      }
#pragma unroll
      for (int u = 0; u < U; u++) a += hsum(v[u]);
    }
    const uint32_t i = c * 64 + lane;
    if (i < n) out[i] = u32x4{a, i, 0u, 0u};
    if (cn >= nch) break;
    c = cn;
    b = bn;
    bytes = bytesn;
  }
}

// reg over spans of CPW consecutive chunks (one contiguous span for packed
// frames), the waves' spans strided by CPW * nw chunks
template <int U, int CPW>
__global__ void __launch_bounds__(256) k_reg3(const uint8_t* base, const uint64_t* off, const uint16_t* len,
                                              u32x4* out, uint32_t n) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  for (uint32_t c = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CPW; c < nch; c += nw * CPW) {
    const uint32_t f0 = c * 64, fe = (c + CPW) * 64 < n ? (c + CPW) * 64 : n;
    const uint64_t b = off[f0] & ~15ull;
    const uint32_t bytes = (uint32_t)(off[fe - 1] + len[fe - 1] - b);
    const uint32_t npc = (bytes + 15) / 16;
    uint32_t a = 0;
    for (uint32_t q0 = 0; q0 < npc; q0 += 64 * U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t q = q0 + 64 * u + lane;
        v[u] = *reinterpret_cast<const u32x4*>(base + b + 16ull * (q < npc ? q : npc - 1));
      }
#pragma unroll
      for (int u = 0; u < U; u++) a += hsum(v[u]);
    }
    for (uint32_t f = f0 + lane; f < fe; f += 64) out[f] = u32x4{a, f, 0u, 0u};
  }
}

constexpr uint32_t kWin = 4096;  // bytes per window (4 glds per lane)
__global__ void __launch_bounds__(256) k_lds(const uint8_t* base, const uint64_t* off, const uint16_t* len,
                                             u32x4* out, uint32_t n, const uint8_t* zero) {
  __shared__ uint32_t buf[4][2][kWin / 4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4, nch = (n + 63) / 64;
  uint32_t c = blockIdx.x * 4 + wv;
  if (c >= nch) return;
  uint64_t b;
  uint32_t bytes;
  span_of(off, len, n, c, b, bytes);
  uint32_t nwin = (bytes + kWin - 1) / kWin, w = 0, slot = 0;
  auto issue = [&](uint64_t sb, uint32_t sbytes, uint32_t win, uint32_t s) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t o = win * kWin + 1024u * k + 16u * lane;
      const uint8_t* src = o < sbytes ? base + sb + o : zero + 16 * lane;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)((lds_u32*)&buf[wv][s][0] + 256u * k),
                                       16, 0, 0);
    }
  };
  issue(b, bytes, 0, 0);
  uint32_t a = 0;
  for (;;) {
    // the next window: this chunk's, else the next chunk's first
    uint32_t cn = c, wn = w + 1;
    uint64_t bn = b;
    uint32_t bytesn = bytes, nwinn = nwin;
    if (wn >= nwin) {
      cn = c + nw;
      wn = 0;
      if (cn < nch) {
        span_of(off, len, n, cn, bn, bytesn);
        nwinn = (bytesn + kWin - 1) / kWin;
      }
    }
    const bool more = cn < nch;
    if (more) {
      issue(bn, bytesn, wn, slot ^ 1u);
      __builtin_amdgcn_s_waitcnt(0x0F74);  // vmcnt(4): all but the 4 just issued
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    __builtin_amdgcn_wave_barrier();
    const lds_u32* q = (const lds_u32*)&buf[wv][slot][0] + 16u * lane;
#pragma unroll
    for (int k = 0; k < 4; k++) a += q[4 * k] + q[4 * k + 1] + q[4 * k + 2] + q[4 * k + 3];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): read before the buffer is refilled
    __builtin_amdgcn_wave_barrier();
    if (wn == 0) {  // chunk c done
      const uint32_t i = c * 64 + lane;
      if (i < n) out[i] = u32x4{a, i, 0u, 0u};
      a = 0;
    }
    if (!more) break;
    c = cn;
    w = wn;
    b = bn;
    bytes = bytesn;
    nwin = nwinn;
    slot ^= 1u;
  }
}

extern "C" const char* p3_name(int w) {
  static const char* nm[] = {"reg_u4", "reg_u8", "reg_u16", "lds_4k", "reg2_u8", "reg2_u16", "reg2_u24",
                             "reg3_u16_c4", "reg3_u16_c16", "reg3_u16_c64", "reg3_u8_c4", "reg3_u8_c1", "reg3_u8_c2"};
  return nm[w];
}
extern "C" int p3_count(void) { return 13; }
extern "C" int p3_launch(int which, const void* base, const void* off, const void* len, void* out, uint32_t n,
                         const void* zero, uint32_t grid, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* bp = (const uint8_t*)base;
  const uint64_t* op = (const uint64_t*)off;
  const uint16_t* lp = (const uint16_t*)len;
  u32x4* o = (u32x4*)out;
  if (which == 0) hipLaunchKernelGGL(k_reg<4>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 1) hipLaunchKernelGGL(k_reg<8>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 2) hipLaunchKernelGGL(k_reg<16>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 4) hipLaunchKernelGGL(k_reg2<8>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 5) hipLaunchKernelGGL(k_reg2<16>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 6) hipLaunchKernelGGL(k_reg2<24>, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 7) hipLaunchKernelGGL((k_reg3<16, 4>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 11) hipLaunchKernelGGL((k_reg3<8, 1>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 12) hipLaunchKernelGGL((k_reg3<8, 2>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 8) hipLaunchKernelGGL((k_reg3<16, 16>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 9) hipLaunchKernelGGL((k_reg3<16, 64>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 10) hipLaunchKernelGGL((k_reg3<8, 4>), dim3(grid), dim3(256), 0, s, bp, op, lp, o, n);
  if (which == 3) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, s, bp, op, lp, o, n, (const uint8_t*)zero);
  return (int)hipGetLastError();
}
