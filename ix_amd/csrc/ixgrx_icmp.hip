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
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(1))) u32x4 gbl_u32x4;

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
template <class W>
DEV uint32_t msg_word(const W* w, uint32_t j, uint32_t nd, uint32_t s, uint32_t len) {
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

// ---- the flood path: a wave of small echo requests packed in one span ------
// When every item of a wave is an echo request of at most kLaneMax bytes
// (device-resident batches, no item list), the frames lie in increasing
// order without overlapping, and the wave's frames span at most kSpanMax
// bytes, the wave copies the span [lo, hi) (first frame's start, last
// message's end) into its LDS with coalesced 16-B loads, each lane sums its
// message and rewrites its header there, and the wave stores the span back
// coalesced (storing only the pieces that hold a rewritten byte, ~3.5 of a
// 98-B frame's ~7, measured 2 % slower: the lines are dirty either way).
// The other path reads every message dword and writes every
// header byte as a separate access to 64 frames (17 + 10 loads and 23 byte
// stores per lane, each instruction touching ~50 lines).
// The 16-B pieces are read from lo & ~15 and up to hi rounded up, inside
// the pages that hold lo and hi - 1 (so no access can fault); a piece only
// partly inside [lo, hi) is stored byte by byte, only its bytes inside.
constexpr uint32_t kSpanMax = 8192;
constexpr uint32_t kMinEcho = 14u + 20u + 8u;  // the shortest frame icmp_input reflects

template <bool OFFS>
DEV bool flood_wave(const ixg_iparams& p, uint64_t i, int lane, bool valid, bool echo, uint32_t meta,
                    lds_u32* sh) {
  const uint32_t len = meta >> 16, moff = meta & 0xffffu;
  const bool lane_ok = !valid || (echo && len <= kLaneMax);
  if (p.idx || __builtin_amdgcn_ballot_w64(!lane_ok) != 0u) return false;
  const int nv = __builtin_popcountll(__builtin_amdgcn_ballot_w64(valid));  // a prefix of the wave (i < n)
  if (nv == 0) return false;
  const uintptr_t a = valid ? reinterpret_cast<uintptr_t>(item_frame<OFFS>(p, i)) : 0;
  const uint32_t a_lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t a_hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uintptr_t lo = ((uintptr_t)a_hi << 32) | a_lo;
  // frame start and message end relative to the span's start
  const uint64_t ra = valid ? (uint64_t)(a - lo) : 0u, re = valid ? ra + moff + len : 0u;
  if (__builtin_amdgcn_ballot_w64(valid && (a < lo || re > kSpanMax - 16u)) != 0u) return false;
  const uint32_t pe = (uint32_t)__shfl_up((int)(uint32_t)re, 1, 64);
  if (__builtin_amdgcn_ballot_w64(valid && lane > 0 && (uint32_t)ra < pe) != 0u) return false;
  // The span is stored back whole, gaps included. With u64 offsets another
  // wave's frames may lie in this wave's gaps (a permuted offset array), and
  // that wave rewrites them at the same time: take the span path
  // only when no gap can hold an echo request (>= kMinEcho bytes: Ethernet,
  // IPv4 and ICMP headers). Strided frames of other waves lie outside the span.
  if (OFFS && __builtin_amdgcn_ballot_w64(valid && lane > 0 && (uint32_t)ra - pe >= kMinEcho) != 0u) return false;
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)re, nv - 1, 64);  // relative, the largest (ordered)
  const uintptr_t lo16 = lo & ~(uintptr_t)15;
  const uint32_t sh0 = (uint32_t)(lo - lo16);  // span start within the first piece
  const uint32_t np = (sh0 + hi + 15u) >> 4;   // <= kSpanMax / 16
  lds_u32x4* lds = (lds_u32x4*)sh;
  // every round loads (pieces past the span re-read its last one: no
  // branches around the loads) and fills its LDS slots
  u32x4 v[kSpanMax / 16 / 64];
  const gbl_u32x4* g = (const gbl_u32x4*)lo16;
#pragma unroll
  for (int r = 0; r < (int)(kSpanMax / 16 / 64); r++) {
    const uint32_t k = (uint32_t)lane + 64u * (uint32_t)r;
    v[r] = g[k < np ? k : np - 1u];
  }
#pragma unroll
  for (int r = 0; r < (int)(kSpanMax / 16 / 64); r++) lds[(uint32_t)lane + 64u * (uint32_t)r] = v[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (valid) {
    lds_u8* f = (lds_u8*)sh + sh0 + (uint32_t)ra;
    const uint32_t at = sh0 + (uint32_t)ra + moff;  // the message, in the LDS span
    const uint32_t s = at & 3u;
    const lds_u32* w = sh + ((at - s) >> 2);
    const uint32_t nd = (s + len + 3u) >> 2;  // <= 33 (len <= kLaneMax)
    uint32_t acc = 0;
    for (uint32_t j0 = 0; j0 < nd; j0 += 8u) {
#pragma unroll
      for (uint32_t k = 0; k < 8u; k++)
        if (j0 + k < nd) acc = add1c(acc, msg_word(w, j0 + k, nd, s, len));
    }
    const uint32_t ck = icmp_ck(acc, s);
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
    f[moff] = 0u;
    f[moff + 2u] = (uint8_t)(ck & 0xffu);
    f[moff + 3u] = (uint8_t)(ck >> 8);
    mark_reply(p, i);  // (no item list on this path: item i is record i)
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the span back: whole pieces as 16-B stores, the (at most two) pieces
  // that straddle lo or lo + hi byte by byte
  const uint32_t end = sh0 + hi;  // in piece-relative bytes
  gbl_u32x4* gs = (gbl_u32x4*)lo16;
#pragma unroll
  for (int r = 0; r < (int)(kSpanMax / 16 / 64); r++) {
    const uint32_t k = (uint32_t)lane + 64u * (uint32_t)r;
    const uint32_t b0 = 16u * k;
    if (k < np && b0 >= sh0 && b0 + 16u <= end) gs[k] = lds[k];
  }
  // the pieces that straddle the span's ends (lanes of the first and the
  // last piece), byte by byte
  if (lane == 0 || (lane == 1 && np > 1u)) {
    const uint32_t b0 = lane == 0 ? 0u : 16u * (np - 1u);
    if (!(b0 >= sh0 && b0 + 16u <= end)) {
      const lds_u8* src = (const lds_u8*)sh + b0;
      uint8_t* dst = reinterpret_cast<uint8_t*>(lo16 + b0);
      for (uint32_t b = 0; b < 16u; b++)
        if (b0 + b >= sh0 && b0 + b < end) dst[b] = src[b];
    }
  }
  return true;
}

template <bool OFFS>
DEV void reflect(const ixg_iparams& p) {
  const int lane = threadIdx.x & 63;
  const uint64_t c = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t i = c * 64u + (uint64_t)lane;
  __shared__ uint32_t sh_span[kWaves][kSpanMax / 4];
  bool echo = false;
  uint32_t meta = 0;  // l4_off | l4_len << 16
  uint64_t ri = 0;    // the item's record
  if (i < p.n) {
    ri = item_rec(p, i);
    const u32x2 r = reinterpret_cast<const u32x2*>(p.rec)[2u * ri];
    echo = ((r.x >> 16) & 0xffu) == IXG_V_ICMP_ECHO;
    meta = r.y;
  }
  if (flood_wave<OFFS>(p, i, lane, i < p.n, echo, meta, (lds_u32*)sh_span[threadIdx.x >> 6])) return;
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
