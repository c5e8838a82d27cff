// ixgrx_icmp.hip - MI355X (gfx950) kernel for ICMP echo reflect
// (dp/net/icmp.c:44-71,88-91): every frame whose record is IXG_V_ICMP_ECHO
// becomes its echo reply in place, as icmp_input leaves it in the mbuf for
// eth_send_one: ICMP type 0; Ethernet destination = the old source, source
// = CFG.mac; IP destination = the old source, source = hton32(CFG.host_addr)
// (the IP checksum is not recomputed: the reference sends with ol_flags 0);
// the ICMP checksum = chksum_internet over the message with type and
// checksum zero.
//
// One wave per 64 records. The record reads are the kernel's traffic when
// echo requests are rare (IX's case). A message of at most kLaneMax bytes
// (a default 64-byte ping is 64) is rewritten by its own lane: every such
// lane sums its message's dwords at once, so a flood of small pings costs
// one pass. Longer messages are taken one at a time by the whole wave: all
// 64 lanes sum the message's dwords (a 1472-byte ping is 6 dwords per
// lane), a cross-lane one's-complement reduction gives the checksum, and 23
// lanes write one rewritten header byte each. Frames may have any
// alignment: a message that starts at an odd address sums byte-swapped
// 16-bit words, and the folded sum is swapped back (RFC 1071 byte-order
// independence).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_icmp.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

DEV uint32_t add1c(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return s + (s < a ? 1u : 0u);
}

DEV uint32_t fold16(uint32_t s) {
  s = (s & 0xffffu) + (s >> 16);
  return (s & 0xffffu) + (s >> 16);
}

constexpr uint32_t kLaneMax = 128;  // messages a lane rewrites on its own

// dword j of the message's aligned dwords (s: the message's start & 3),
// with the bytes that do not count zeroed: before the message, the type
// (message byte 0: becomes 0), the checksum field (bytes 2, 3), past len
DEV uint32_t msg_word(const uint32_t* w, uint32_t j, uint32_t nd, uint32_t s, uint32_t len) {
  uint32_t v = w[j];
  if (j == 0u || j == 1u || j + 1u == nd) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int t = (int)(4u * j) + k - (int)s;
      const bool keep = t == 1 || (t >= 4 && t < (int)len);
      if (!keep) v &= ~(0xffu << (8 * k));
    }
  }
  return v;
}

// chksum_internet of the folded sum (the swap for an odd start)
DEV uint32_t icmp_ck(uint32_t acc, uint32_t s) {
  uint32_t sum = fold16(acc);
  if (s & 1u) sum = ((sum & 0xffu) << 8) | (sum >> 8);
  return (~sum) & 0xffffu;
}

// header byte k (0..22) of the reply: Ethernet dhost = shost, shost =
// CFG.mac (icmp.c:50-51); IP dst = src, src = CFG.host_addr (:54-55);
// type = ICMP_ECHOREPLY (:89), checksum (:57-58): where it goes (at) and
// its value. Lanes 0-5 and 12-15 read bytes that lanes 6-11 and 16-19
// write: every lane takes its value here, the wave joins a barrier, and
// only then does any lane store (reply_store).
DEV uint32_t reply_byte(const ixg_iparams& p, const uint8_t* f, uint32_t off, uint32_t ck, int k, uint32_t& at) {
  uint32_t val;
  if (k < 6) {
    at = (uint32_t)k;
    val = f[6 + k];
  } else if (k < 12) {
    at = (uint32_t)k;
    val = p.mac[k - 6];
  } else if (k < 16) {
    at = 30u + (uint32_t)(k - 12);
    val = f[26 + (k - 12)];
  } else if (k < 20) {
    at = 26u + (uint32_t)(k - 16);
    val = p.host[k - 16];
  } else if (k == 20) {
    at = off;
    val = 0u;
  } else {
    at = off + 2u + (uint32_t)(k - 21);
    val = k == 21 ? (ck & 0xffu) : (ck >> 8);
  }
  return val;
}

// the record of item j (and where its frame is)
template <bool OFFS>
DEV uint8_t* item_frame(const ixg_iparams& p, uint64_t j) {
  return reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(p.base) + (OFFS ? p.off[j] : j * (uint64_t)p.stride));
}
DEV uint64_t item_rec(const ixg_iparams& p, uint64_t j) { return p.idx ? (uint64_t)p.idx[j] : j; }

// a reflected record: IXG_RF_REPLY (the asynchronous path's candidates)
DEV void mark_reply(const ixg_iparams& p, uint64_t r) {
  if (!p.mark) return;
  uint8_t* fl = reinterpret_cast<uint8_t*>(p.rec + r) + 3;
  *fl = (uint8_t)(*fl | IXG_RF_REPLY);
}

template <bool OFFS>
DEV void reflect(const ixg_iparams& p) {
  const int lane = threadIdx.x & 63;
  const uint64_t c = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t i = c * 64u + (uint64_t)lane;
  bool echo = false;
  uint32_t meta = 0;  // l4_off | l4_len << 16
  uint64_t ri = 0;    // the item's record
  if (i < p.n) {
    ri = item_rec(p, i);
    const u32x2 r = reinterpret_cast<const u32x2*>(p.rec)[2u * ri];
    echo = ((r.x >> 16) & 0xffu) == IXG_V_ICMP_ECHO;
    meta = r.y;
  }
  // messages of at most kLaneMax bytes: each lane its own
  if (echo && (meta >> 16) <= kLaneMax) {
    const uint32_t off = meta & 0xffffu, len = meta >> 16;
    uint8_t* f = item_frame<OFFS>(p, i);
    const uintptr_t a = reinterpret_cast<uintptr_t>(f) + off;
    const uint32_t s = (uint32_t)(a & 3u);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a - s);
    const uint32_t nd = (s + len + 3u) >> 2;
    uint32_t acc = 0;
    for (uint32_t j = 0; j < nd; j++) acc = add1c(acc, msg_word(w, j, nd, s, len));
    const uint32_t ck = icmp_ck(acc, s);
    // the old source MAC and IP address first: their bytes are rewritten
    uint8_t src_mac[6], src_ip[4];
#pragma unroll
    for (int k = 0; k < 6; k++) src_mac[k] = f[6 + k];
#pragma unroll
    for (int k = 0; k < 4; k++) src_ip[k] = f[26 + k];
#pragma unroll
    for (int k = 0; k < 6; k++) f[k] = src_mac[k];
#pragma unroll
    for (int k = 0; k < 6; k++) f[6 + k] = p.mac[k];
#pragma unroll
    for (int k = 0; k < 4; k++) f[30 + k] = src_ip[k];
#pragma unroll
    for (int k = 0; k < 4; k++) f[26 + k] = p.host[k];
    f[off] = 0u;
    f[off + 2u] = (uint8_t)(ck & 0xffu);
    f[off + 3u] = (uint8_t)(ck >> 8);
    mark_reply(p, ri);
  }
  const bool big = echo && (meta >> 16) > kLaneMax;
  for (uint64_t m = __builtin_amdgcn_ballot_w64(big); m; m &= m - 1u) {
    const int e = __builtin_ctzll(m);
    const uint64_t fi = c * 64u + (uint64_t)e;
    const uint32_t fm = __builtin_amdgcn_readlane(meta, e);
    const uint32_t off = fm & 0xffffu, len = fm >> 16;  // icmp_input's len >= 8
    uint8_t* f = item_frame<OFFS>(p, fi);
    // the message [a, a + len) as aligned dwords; byte k of dword j is
    // message byte 4j + k - s
    const uintptr_t a = reinterpret_cast<uintptr_t>(f) + off;
    const uint32_t s = (uint32_t)(a & 3u);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a - s);
    const uint32_t nd = (s + len + 3u) >> 2;
    uint32_t acc = 0;
    for (uint32_t j = (uint32_t)lane; j < nd; j += 64u) acc = add1c(acc, msg_word(w, j, nd, s, len));
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc = add1c(acc, (uint32_t)__shfl_xor((int)acc, d, 64));
    const uint32_t ck = icmp_ck(acc, s);  // chksum_internet, stored as is
    // one header byte per lane: all reads, a wave barrier, then the stores
    uint32_t at = 0, val = 0;
    if (lane < 23) val = reply_byte(p, f, off, ck, lane, at);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane < 23) f[at] = (uint8_t)val;
    if (lane == e) mark_reply(p, ri);
  }
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock) ixg_icmp_reflect_s(ixg_iparams p) { reflect<false>(p); }
extern "C" __global__ void __launch_bounds__(kBlock) ixg_icmp_reflect_o(ixg_iparams p) { reflect<true>(p); }

extern "C" int ixgrx_icmp_launch(const void* params, void* stream) {
  const ixg_iparams& p = *static_cast<const ixg_iparams*>(params);
  const uint64_t grid = ((uint64_t)p.n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(p.off ? ixg_icmp_reflect_o : ixg_icmp_reflect_s, dim3((uint32_t)grid), dim3(kBlock), 0,
                     (hipStream_t)stream, p);
  return (int)hipGetLastError();
}
