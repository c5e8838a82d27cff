// ixgrx_tcpx.hip - MI355X (gfx950) kernel for the rest of the tcp_input head
// (dp/net/tcp_in.c:230-241): for every IXG_V_TCP (or IXG_V_TCP6) record,
// the header fields tcp_input converts to host order and keeps in its
// LWIP_Context (ports, seqno, ackno, wnd) and tcplen, as one 16-byte
// struct ixg_tcp_ext per frame; optionally the in-place conversion itself.
//
// One lane per frame, one wave per 64 frames, no loop: the work per frame is
// a 16-byte record load, two loads from the frame's first 52 bytes and a
// 16-byte store, so the kernel is bound by HBM and needs only many waves in
// flight. The frame loads are issued together with the record load, for the
// common geometry (IPv4, ihl 5: TCP header at 34); a lane whose record says
// otherwise (IP options, the IPv6 extension) loads its header again at the
// right offset. Non-TCP lanes store zeros.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_tcpx.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

// 20 header bytes from the dword boundary 2 bytes before the TCP header
// (frame starts are 4-aligned and the header sits at 14 + 4*ihl or 54)
struct Hdr {
  u32x4 d;     // header bytes -2..13
  uint32_t e;  // header bytes 14..17
};

DEV Hdr load_hdr(const uint8_t* t) {
  Hdr h;
  h.d = *reinterpret_cast<const u32x4_a4*>(t - 2);
  h.e = *reinterpret_cast<const uint32_t*>(t + 14);
  return h;
}

template <bool OFFS>
DEV void tcpx(const ixg_xparams& p) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= p.n) return;
  uint8_t* f = p.base + (OFFS ? p.off[i] : i * (uint64_t)p.stride);
  const u32x4 r = reinterpret_cast<const u32x4*>(p.rec)[i];
  const uint32_t w12 = *reinterpret_cast<const uint32_t*>(f + 12);  // ethertype, version/ihl
  Hdr h = load_hdr(f + 34);
  const uint32_t verdict = (r.x >> 16) & 0xffu;
  const bool v4 = verdict == IXG_V_TCP, v6 = verdict == IXG_V_TCP6;
  u32x4 x = {0u, 0u, 0u, 0u};
  if (v4 || v6) {
    const uint32_t l4 = v6 ? 54u : 14u + 4u * ((w12 >> 16) & 15u);
    if (l4 != 34u) h = load_hdr(f + l4);  // IP options / IPv6: rare
    const uint32_t D0 = h.d.x, D1 = h.d.y, D2 = h.d.z, D3 = h.d.w, D4 = h.e;
    const ixgx_ext e = ixgx_make(D0, D1, D2, D3, D4, r.y, r.w);
    x = u32x4{e.x, e.y, e.z, e.w};
    if (p.flags & IXG_TCPX_INPLACE) ixgx_inplace(reinterpret_cast<uint32_t*>(f + l4 - 2), D0, D3, D4, e);
  }
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p.ext) + i);
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock) ixg_tcpx_s(ixg_xparams p) { tcpx<false>(p); }
extern "C" __global__ void __launch_bounds__(kBlock) ixg_tcpx_o(ixg_xparams p) { tcpx<true>(p); }

extern "C" int ixgrx_tcpx_launch(const void* params, void* stream) {
  const ixg_xparams& p = *static_cast<const ixg_xparams*>(params);
  const uint64_t grid = ((uint64_t)p.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(p.off ? ixg_tcpx_o : ixg_tcpx_s, dim3((uint32_t)grid), dim3(kBlock), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}
