// ixgrx_kernels.hip - MI355X (gfx950) RX parse + checksum + flow-hash kernels.
//
// Two kernels per batch, both one wavefront lane per packet:
//
// ixg_rx_fast_{s,o}: the fixed-shape kernel. A persistent grid-stride loop
// over 64-packet chunks, software-pipelined: descriptors two chunks ahead,
// the 52 header bytes a 64 B frame needs (12..63) one chunk ahead. A chunk
// whose 64 frames are all plain IPv4 ihl 5 with the segment inside 64
// bytes (the 64 B TCP config) is parsed with the header geometry
// constant-folded; any other chunk is flagged in the per-chunk defer array.
//
// ixg_rx_general_{s,o}: every header shape the reference handles, for the
// flagged chunks (or all chunks when the fixed-shape kernel is skipped).
// Pass A: each lane loads its 96-byte prefix, parses Ethernet/IPv4 (with
// options)/TCP/UDP/ICMP (and the IPv6 extension) as dp/net/ip.c + dp/lwip
// do, and sums the IP header and the in-prefix part of the L4 segment as
// 32-bit one's complement words. Segments running past the prefix are
// compacted per wave (ballot + mbcnt) into an LDS list; their tails are
// summed by 16-lane groups, 4 packets per round, 8 x 16 B loads per lane
// per round, two rounds in flight, then a 16-lane shuffle reduction.
//
// Both kernels look the 12 tuple bytes up in a per-workgroup LDS copy of
// the combined Toeplitz/CRC-32C byte tables (both hashes are GF(2)-affine
// in the tuple, DESIGN.md "hash tables").
//
// No MFMA: this is integer byte work bound by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/ixgrx.h"
#include "ixgrx_internal.h"
#include "ixgrx_tcpx.h"
#include "ixgrx_walk.h"

#define DEV __device__ __forceinline__

// Wave votes from one v_cmp into an SGPR pair + a scalar compare (the ockl
// __all/__any helpers cost several VALU instructions each). Inactive lanes
// do not vote, as with __all/__any.
DEV bool wave_all(bool pred) { return __builtin_amdgcn_ballot_w64(!pred) == 0; }
DEV bool wave_any(bool pred) { return __builtin_amdgcn_ballot_w64(pred) != 0; }

namespace {

constexpr int kBlock = 256;        // 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kPrefixDw = 24;      // 96-byte header prefix
constexpr int kFastDw = 16;        // the fast shape needs 64 bytes
constexpr int kStreamBase = 96;    // long segments: streamed from here

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));  // frames are 4-byte aligned

using KParams = ixg_kparams;

DEV uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// end-around fold of a 64-bit sum of 32-bit LE words to 16 bits; 0 only
// for an all-zero input (the representation chksum_internet produces)
DEV uint32_t fold16(uint64_t s) {
  s = (s & 0xffffffffull) + (s >> 32);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  return (uint32_t)s;
}

// 32-bit end-around add (never produces 0 from non-zero inputs)
DEV uint32_t add1c(uint32_t a, uint32_t b) {
  uint32_t s = a + b;
  return s + (s < a ? 1u : 0u);
}

DEV uint32_t fold32(uint64_t s) { return add1c((uint32_t)s, (uint32_t)(s >> 32)); }

// acc + a + b (8 dwords) in one's complement (end-around carry) arithmetic:
// one v_add/v_addc per dword and one to fold the last carry. Only additions:
// the result is 0 only if acc and every dword are 0 (the representation
// chksum_internet produces). The final carry-in cannot overflow: after an
// add that carried out, the partial sum is <= 0xfffffffe.
// Two independent adc8 chains interleaved (carries in VCC and in an SGPR
// pair), so consecutive instructions do not depend on each other.
DEV void adc8x2(uint32_t& acc0, const u32x4& a, const u32x4& b, uint32_t& acc1, const u32x4& c, const u32x4& d) {
  uint64_t cc;
  asm volatile(
      "v_add_co_u32 %0, vcc, %0, %3\n\t"
      "v_add_co_u32 %1, %2, %1, %11\n\t"
      "v_addc_co_u32 %0, vcc, %0, %4, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %12, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %5, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %13, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %6, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %14, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %7, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %15, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %8, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %16, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %9, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %17, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, %10, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, %18, %2\n\t"
      "v_addc_co_u32 %0, vcc, %0, 0, vcc\n\t"
      "v_addc_co_u32 %1, %2, %1, 0, %2"
      : "+v"(acc0), "+v"(acc1), "=&s"(cc)
      : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w),
        "v"(c.x), "v"(c.y), "v"(c.z), "v"(c.w), "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w)
      : "vcc");
}

DEV uint32_t adc8(uint32_t acc, const u32x4& a, const u32x4& b) {
  asm volatile(
      "v_add_co_u32 %0, vcc, %0, %1\n\t"
      "v_addc_co_u32 %0, vcc, %0, %2, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %3, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %4, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %5, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %6, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %7, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, %8, vcc\n\t"
      "v_addc_co_u32 %0, vcc, %0, 0, vcc"
      : "+v"(acc)
      : "v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
      : "vcc");
  return acc;
}

// mask of the first k bytes of a dword, k in [0, 4]
DEV uint32_t ones(int k) { return k >= 4 ? 0xffffffffu : ((1u << (8 * k)) - 1u); }

// byte b of the prefix (b compile-time constant in all uses)
template <int N>
DEV uint32_t byte_at(const uint32_t (&d)[N], int b) { return (d[b >> 2] >> (8 * (b & 3))) & 0xffu; }

// d[idx] for a per-lane idx in [lo, hi] (select chain: no dynamic register indexing)
// (hipcc turns a plain ?: chain back into a private-array load through
// scratch; an AND/OR mux with an opaque mask keeps it in VGPRs)
template <int N, int LO, int HI>
DEV uint32_t pick(const uint32_t (&d)[N], int idx) {
  uint32_t r = 0;
#pragma unroll
  for (int j = LO; j <= HI; j++) {
    uint32_t m = 0u - (uint32_t)(idx == j);
    asm volatile("" : "+v"(m));
    r |= d[j] & m;
  }
  return r;
}

// (m & x) | (~m & y): one v_bfi_b32 per dword
DEV uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) { return (m & x) | (~m & y); }
DEV uint64_t bsel(uint32_t m, uint64_t x, uint64_t y) {
  return (uint64_t)bsel(m, (uint32_t)(x >> 32), (uint32_t)(y >> 32)) << 32 | bsel(m, (uint32_t)x, (uint32_t)y);
}

// out[m] = v[s + m] (m < M) for a per-lane s in [0, 2^B): a log-depth mux.
// Stage k (high bit first) picks a[i] or a[i + 2^k] on bit k of s, for the
// entries later stages can still reach; indices past N read 0. Constant
// indices, one all-ones/zero mask per stage (opaque to the compiler, which
// otherwise rebuilds compare chains and spills lane masks) and v_bfi_b32:
// no dynamic register indexing, no scratch.
template <int B, int N, int M, typename T>
DEV void window(const T (&v)[N], uint32_t s, T (&out)[M]) {
  constexpr int W = M + (1 << B) - 1;
  T a[W];
#pragma unroll
  for (int i = 0; i < W; i++) a[i] = i < N ? v[i < N ? i : 0] : T(0);
#pragma unroll
  for (int k = B - 1; k >= 0; k--) {
    uint32_t m = 0u - ((s >> k) & 1u);
    asm volatile("" : "+v"(m));
    const int sh = 1 << k;
#pragma unroll
    for (int i = 0; i < M + sh - 1; i++) a[i] = bsel(m, a[i + sh], a[i]);
  }
#pragma unroll
  for (int m = 0; m < M; m++) out[m] = a[m];
}

template <int B, int N, typename T>
DEV T select(const T (&v)[N], uint32_t s) {
  T o[1];
  window<B, N, 1>(v, s, o);
  return o[0];
}

// Sum of the bytes [a, e) of the prefix as 32-bit LE words, where a = 4*qa+2
// (every region this path sums starts 2 bytes into a dword: the IPv4
// header at 14, L4 headers at 14+4*ihl, IPv6 addresses at 22) and e >= a.
template <int N>
DEV uint64_t region_sum(const uint32_t (&d)[N], int qa, int e) {
  const int qe = e >> 2;
  const uint32_t tail = ones(e & 3);
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < N; j++) {
    uint32_t m = (j < qa) ? 0u : ((j == qa) ? 0xffff0000u : 0xffffffffu);
    m &= (j < qe) ? 0xffffffffu : ((j == qe) ? tail : 0u);
    s += d[j] & m;
  }
  return s;
}

// 16-byte load that is always issued: lanes that must not read their
// frame read `dummy` (an always-valid L1-resident address). Every consumer
// masks by the frame/segment length, so the dummy bytes never count, and
// no select touches the value at issue time (that would force an immediate
// vmcnt wait). Loads inside exec-masked branches make hipcc count them as
// possibly not issued, so its vmcnt waits for the current data would also
// wait for the loads prefetched for the next step.
DEV u32x4 load16(bool ok, const uint8_t* addr, const uint8_t* dummy) {
  return *reinterpret_cast<const u32x4_a4*>(ok ? addr : dummy);
}

// 64-bit wave broadcasts (the builtins return int: each half is taken as
// uint32_t, or a low word >= 2^31 would sign-extend over the high one)
DEV uint64_t rfl64(uint64_t x) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}
DEV uint64_t rl64(uint64_t x, uint32_t lane) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)x, lane) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), lane) << 32);
}

struct Rec {
  uint32_t w0, w1, w2, w3;  // the 16-byte ixg_rx_rec as four dwords
};

// Everything a lane computes for its frame, minus the streamed tail sum.
struct LaneState {
  uint32_t verdict, flags, l4_off, l4_len, rss, bucket, tcp_flags, fg;
  uint32_t ip_res, l4_res;   // residual words for the csum output
  int l4_kind;               // 0 none, 1 TCP/UDP pseudo, 2 ICMP plain
  uint64_t l4_acc;           // in-prefix segment sum + pseudo header
  uint32_t seg_end;          // frame offset where the segment ends
  bool stream;               // segment extends past the prefix
  // fields the deferred verdict needs
  uint32_t l4, l4len, proto, doff, ulen, icmp_type;
  bool v6;
  // the 4-tuple for the fused demux: raw IPs, ports host order (sport | dport << 16)
  uint32_t src, dst, ports;
};

// x & ones(clamp(t, 0, 4)): v_med3 + two shifts (the 64-bit one handles
// the shift by 32) + v_bfi
DEV uint32_t keep_bytes(uint32_t x, int t) {
  const uint32_t u = (uint32_t)(t < 0 ? 0 : (t > 4 ? 4 : t));
  return x & ~(uint32_t)(~0ull << (8u * u));
}

// Bytes at offsets >= L read as zero (DESIGN.md "bytes beyond L"). The
// general parse loads prefixes raw (bytes past L belong to the next frame)
// and masks only what can be consumed past L: every other field is read
// behind a length check that already covers it (the IPv4 fields behind
// ip.c:68's L >= 34, the L4 header and sums behind 14 + ip_len <= L, the
// ports behind l4 + 4 <= L, the IPv6 fields behind L >= 54 / 54 + plen <=
// L). Two are not: the Ethernet type of a frame shorter than 14 bytes, and
// udp_input's length field (l4 + 4, unchecked by udp.c:59's own test).
template <int N>
DEV uint32_t eth_type(const uint32_t (&d)[N], uint32_t L) {
  return ((L > 12u ? byte_at(d, 12) : 0u) << 8) | (L > 13u ? byte_at(d, 13) : 0u);
}

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) uint16_t lds_u16;

// The combined Toeplitz / CRC-32C byte tables (DESIGN.md "hash tables"),
// staged in LDS: look(pos, b) = Toeplitz contribution (low word) and CRC
// contribution (high word; only its low 9 bits reach the PCB bucket) of
// tuple byte pos with value b.
struct Tab64 {  // 12 x 256 u64 (24 KiB)
  const uint64_t* T;
  DEV uint64_t look(int pos, uint32_t b) const { return T[(pos << 8) | b]; }
};
struct TabSplit {  // 12 x 256 u32 Toeplitz + 12 x 256 u16 CRC (18 KiB)
  const lds_u32* t32;
  const lds_u16* t16;
  DEV uint64_t look(int pos, uint32_t b) const {
    return ((uint64_t)t16[(pos << 8) | b] << 32) | t32[(pos << 8) | b];
  }
};

// Header shapes a wave can be specialised for (wave-uniform):
// kShapeFixed: every lane IPv4 with ihl 5, the geometry constant-folded;
// kShapeV4: every lane IPv4 (any ihl) or a non-IP frame, no IPv6 code;
// kShapeV6: every lane IPv6 under IXG_F_IPV6 (L4 at the constant 54);
// kShapeAny: anything.
constexpr int kShapeFixed = 0, kShapeV4 = 1, kShapeV6 = 2, kShapeAny = 3;

// ---- [NIC] flow-director perfect filters (ixg_rx_set_fdir) ----
// The table lives in device memory with its header (ixgrx_internal.h), read
// at run time: a graph captured before the filters changed sees the new set.
// Returns the outbound flow group of a matching frame, or 0xffffffff.
DEV uint32_t fdir_match(const KParams& p, uint32_t src, uint32_t dst, uint32_t ports) {
  // {mask, fg, 0, 0}: a scalar load through the constant address space (the
  // host writes the table only between launches). Read as a plain global
  // load it was a vector load, and its s_waitcnt vmcnt(0) also waited for
  // every frame load the wave had in flight (the next chunk's prefetch)
  typedef const __attribute__((address_space(4))) u32x4 cu32x4;
  const u32x4 hdr = *(cu32x4*)(p.fdir);
  if (hdr.x == 0u) return 0xffffffffu;
  const u32x4* slot = reinterpret_cast<const u32x4*>(p.fdir) + 1;
  uint32_t k = ixg_fdir_hash(src, dst, ports) & hdr.x;
  for (;;) {
    const u32x4 e = slot[k];
    if (e.w == 0u) return 0xffffffffu;
    if (e.x == src && e.y == dst && e.z == ports) return hdr.y;
    k = (k + 1u) & hdr.x;
  }
}

// NDW: prefix dwords available; a segment ending past 4*NDW bytes is left
// to the streaming rounds.
template <int SHAPE, int NDW, class Tab, class T6P = const lds_u32*>
DEV void lane_parse(const KParams& p, const Tab& T, const uint32_t (&d)[kPrefixDw],
                    uint32_t L, LaneState& s, T6P T6 = nullptr) {
  constexpr bool FIXED = SHAPE == kShapeFixed;
  const uint32_t etype = eth_type(d, L);                                   // ip.c:132
  const uint32_t vh = byte_at(d, 14);
  const uint32_t ver = vh >> 4;
  const int ihl = FIXED ? 5 : (int)(vh & 15u);                             // ip.h:84-90
  const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
  const uint32_t ip_off = (byte_at(d, 20) << 8) | byte_at(d, 21);
  const uint32_t proto = byte_at(d, 23);
  const bool frag = (ip_off & 0x3fffu) != 0;                              // ip.c:78
  const uint32_t src = (d[6] >> 16) | (d[7] << 16);                       // bytes 26..29 raw
  const uint32_t dst = (d[7] >> 16) | (d[8] << 16);                       // bytes 30..33 raw
  const int l4 = 14 + 4 * ihl;
  const bool ip4 = SHAPE != kShapeV6 && etype == 0x0800u;
  const bool v6 = SHAPE == kShapeV6 || (SHAPE == kShapeAny && etype == 0x86DDu && (p.flags & IXG_F_IPV6));

  // L4 header dwords: frame byte l4+b sits in dword q + (2+b)/4, where
  // l4 = 4q + 2 (IPv4: q = 3 + max(ihl, 5); the IPv6 extension: L4 at 54,
  // q = 13). The general shapes read them through a 4-stage mux.
  const int q = 3 + (ihl < 5 ? 5 : ihl);
  uint32_t h0, h1, h2, h3;
  // C[k] = one's complement (end-around carry) sum of the 32-bit words of
  // bytes [14, 4k): congruent to the exact sum mod 2^32 - 1, and 0 only when
  // every word is 0, so its 16-bit fold is the exact sum's. Half the registers
  // and mux work of exact 64-bit sums. (General shapes only.)
  uint32_t C[kPrefixDw + 1];
  uint32_t spre = 0, reg32 = 0;
  if (FIXED) {
    h0 = d[8]; h1 = d[9]; h2 = d[10]; h3 = d[11];
  } else {
    C[3] = 0;
    C[4] = d[3] & 0xffff0000u;
#pragma unroll
    for (int k = 4; k < kPrefixDw; k++) C[k + 1] = add1c(C[k], d[k]);
    if (SHAPE == kShapeV6) {
      h0 = d[13]; h1 = d[14]; h2 = d[15]; h3 = d[16];
      spre = add1c(C[13], h0 & 0xffffu);
    } else {
      const uint32_t qs = v6 ? 5u : (uint32_t)(q - 8);  // in [0, 10]
      uint32_t src4[kPrefixDw - 8], h[4];
#pragma unroll
      for (int j = 0; j < kPrefixDw - 8; j++) src4[j] = d[8 + j];
      window<4>(src4, qs, h);
      h0 = h[0]; h1 = h[1]; h2 = h[2]; h3 = h[3];
      // bytes [14, l4) = C[q] + the low half of dword q (= h0): the IPv4
      // header, or the IPv6 header + the Ethernet type's successor bytes
      uint32_t Cq[11];
#pragma unroll
      for (int j = 0; j < 11; j++) Cq[j] = C[8 + j];
      spre = add1c(select<4>(Cq, qs), h0 & 0xffffu);
    }
    // the L4 region's in-prefix sum, computed here while C[] is live (the
    // hash lookups below then run without it)
    {
      static_assert(FIXED || NDW == kPrefixDw, "the general shapes sum the whole prefix");
      const uint32_t se = v6 ? 54u + ((byte_at(d, 18) << 8) | byte_at(d, 19)) : 14u + ip_len;
      const int e = (int)(se < (uint32_t)(4 * NDW) ? se : (uint32_t)(4 * NDW));
      // bytes [l4, e) = [14, e) - [14, l4) (one's complement subtraction:
      // add the complement); e >= l4 + 8 here (segments of at least 8
      // bytes), so e's dword index is in [10, 24]
      const uint32_t qe = (uint32_t)e >> 2;
      const uint32_t qi = (qe < 10u ? 10u : qe) - 10u;
      uint32_t Ce[15], de[15];
#pragma unroll
      for (int j = 0; j < 15; j++) {
        Ce[j] = C[10 + j];
        de[j] = 10 + j < kPrefixDw ? d[10 + j < kPrefixDw ? 10 + j : 0] : 0u;
      }
      const uint32_t s_e = add1c(select<4>(Ce, qi), select<4>(de, qi) & ones(e & 3));
      uint32_t a32 = add1c(s_e, ~spre);
      // x - x gives the negative zero 0xffffffff; it stands for an exact 0
      // only when every byte of the region is 0 (the ICMP residual, which
      // has no pseudo header, depends on the difference): rare, checked
      // exactly, one mask per dword
      if (wave_any(a32 == 0xffffffffu)) {
        const int a = v6 ? 54 : l4;
        uint32_t nz = 0;
#pragma unroll
        for (int j = 3; j < kPrefixDw; j++) {
          const int lo = a - 4 * j, hi = e - 4 * j;
          nz |= d[j] & keep_bytes(~0u, hi) & ~keep_bytes(~0u, lo);
        }
        if (a32 == 0xffffffffu && nz == 0) a32 = 0;
      }
      reg32 = a32;
    }
  }
  const uint32_t b0 = (h0 >> 16) & 0xffu, b1 = h0 >> 24;                  // sport (wire)
  const uint32_t b2 = h1 & 0xffu, b3 = (h1 >> 8) & 0xffu;                 // dport (wire)
  const uint32_t w45 = h1 >> 16;                                          // L4 bytes 4,5 (LE)
  const uint32_t doff_byte = (h3 >> 16) & 0xffu;                          // TCP byte 12
  const uint32_t tflags = h3 >> 24;                                       // TCP byte 13

  s.v6 = v6;
  s.proto = v6 ? byte_at(d, 20) : proto;
  s.src = src;
  s.dst = dst;
  s.ports = ((b0 << 8) | b1) | (((b2 << 8) | b3) << 16);
  const uint32_t v6_plen = (byte_at(d, 18) << 8) | byte_at(d, 19);
  const bool v6_ok = v6 && L >= 54 && (vh >> 4) == 6 && 54 + v6_plen <= L;

  // ---- [NIC] IPv4 header checksum (DESIGN.md NIC rules) ----
  const bool hdr_ok = ip4 && ver == 4 && ihl >= 5 && (uint32_t)l4 <= L;
  s.flags = 0;
  s.ip_res = 0xffffu;
  if (hdr_ok) {
    uint64_t hs;
    if (FIXED) {
      hs = (uint64_t)(d[3] >> 16) + d[4] + d[5] + d[6] + d[7] + (d[8] & 0xffffu);
    } else {
      hs = spre;  // bytes [14, 14 + 4 ihl)
    }
    s.ip_res = (~fold16(hs)) & 0xffffu;                                    // chksum_internet
    s.flags |= IXG_RF_IP_CSUM_CHECKED | (s.ip_res == 0 ? IXG_RF_IP_CSUM_OK : 0u);
  }

  // ---- [NIC] RSS Toeplitz + tcp_to_idx via the byte tables ----
  const bool rss4 = hdr_ok && !frag && (proto == 6 || proto == 17) && (uint32_t)(l4 + 4) <= L;
  // The 12 lookups serve both families: an IPv4 lane looks up its tuple
  // (src, dst, ports), an IPv6 lane the first 12 bytes of its 36-byte tuple
  // (frame bytes 22..33: the same key offsets, so the same tables' Toeplitz
  // words; its bucket is never used). A mixed wave then runs 12 + 24
  // lookups instead of 12 + 36.
  uint64_t hx = 0;
  {
    const uint32_t t4 = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    const uint32_t a6 = (d[5] >> 16) | (d[6] << 16);  // bytes 22..25
    uint32_t sb = src, db = dst, pb = t4;
    if (SHAPE == kShapeV6) {
      sb = a6; db = src; pb = dst;
    } else if (SHAPE == kShapeAny) {
      uint32_t m6 = 0u - (uint32_t)v6;
      asm volatile("" : "+v"(m6));
      sb = bsel(m6, a6, src);
      db = bsel(m6, src, dst);
      pb = bsel(m6, dst, t4);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      hx ^= T.look(k, (sb >> (8 * k)) & 0xffu);
      hx ^= T.look(4 + k, (db >> (8 * k)) & 0xffu);
      hx ^= T.look(8 + k, (pb >> (8 * k)) & 0xffu);
    }
  }
  s.rss = 0;
  if (rss4) {
    s.rss = (uint32_t)hx;
    s.flags |= IXG_RF_RSS;
  }
  // IPv6 extension: Toeplitz over src(16) dst(16) sport dport, one byte
  // table lookup per tuple byte: positions 0..11 share the IPv4 tables' key
  // offsets (their low words), positions 12..35 come from the IPv6 tables
  // staged in LDS by the general kernels (IXG_TAB6_WORDS)
  if (SHAPE != kShapeFixed && SHAPE != kShapeV4 && v6 && L >= 58 && ver == 6 && (s.proto == 6 || s.proto == 17)) {
    uint32_t h = (uint32_t)hx;  // tuple bytes 0..11, above
#pragma unroll
    for (int k = 12; k < 36; k++) {
      const uint32_t b = byte_at(d, k < 32 ? 22 + k : 54 + (k - 32));
      h ^= T6[((k - 12) << 8) | b];
    }
    s.rss = h;
    s.flags |= IXG_RF_RSS;
  }
  s.fg = p.fg_base + (s.rss & p.fg_mask);
  s.bucket = ((uint32_t)(hx >> 32) ^ p.crc_const) & (IXG_PCB_BUCKETS - 1);  // (9 bits of the CRC)

  // ---- L4 segment: [l4, 14 + ip_len) ----
  uint32_t l4len = ip_len - 4u * (uint32_t)ihl;
  uint32_t seg_end = 14 + ip_len;
  bool seg_ok = ip4 && ver == 4 && ihl >= 5 && !frag && ip_len >= 4u * (uint32_t)ihl && seg_end <= L;
  if (v6) {
    l4len = v6_plen;
    seg_end = 54 + v6_plen;
    seg_ok = v6_ok;
  }
  s.l4 = v6 ? 54 : l4;
  s.l4len = l4len;
  s.seg_end = seg_end;
  s.doff = doff_byte >> 4;
  s.tcp_flags = tflags & 0x3fu;
  s.ulen = bswap16(keep_bytes(w45, (int)L - (int)s.l4 - 4));  // (udp_input reads it unchecked)
  s.icmp_type = b0;

  const uint32_t sp = s.proto;
  // UDP checksum field: L4 bytes 6,7 = low half of dword q+2
  const uint32_t ucs = v6 ? 1u : (h2 & 0xffffu);
  int kind = 0;
  if (seg_ok && ((sp == 6 && l4len >= 20) || (sp == 17 && l4len >= 8 && ucs != 0))) kind = 1;
  if (!v6 && seg_ok && sp == 1 && l4len >= 8) kind = 2;
  s.l4_kind = kind;
  uint64_t acc = 0;
  if (kind) {
    const int e = (int)(seg_end < (uint32_t)(4 * NDW) ? seg_end : (uint32_t)(4 * NDW));
    if constexpr (FIXED) {
      uint32_t dd[NDW];
#pragma unroll
      for (int j = 0; j < NDW; j++) dd[j] = d[j];
      acc = region_sum(dd, 8, e);
    } else {
      acc = reg32;
    }
    if (kind == 1) {
      uint64_t ps;
      if (v6) {
        // src + dst: bytes [22, 54) = [14, 54) - [14, 22)
        ps = add1c(add1c(C[13], d[13] & 0xffffu), ~add1c(C[5], d[5] & 0xffffu));
      } else {
        ps = (uint64_t)(src & 0xffffu) + (src >> 16) + (dst & 0xffffu) + (dst >> 16);
      }
      acc += ps + (sp << 8) + bswap16(l4len & 0xffffu);  // htons(proto) + htons(proto_len)
    }
  }
  s.l4_acc = acc;
  s.stream = kind != 0 && seg_end > (uint32_t)(4 * NDW);
  // ---- [NIC] flow-director perfect filters (ixg_rx_set_fdir): a matching
  // IPv4 TCP frame has FLM set, so the driver gives it MBUF_INVALID_FG_ID
  // (ixgbe.c:329-330) and eth_recv_handle_fg_transition the CPU's outbound
  // group (ethfg.c:504-505)
  if (SHAPE != kShapeV6 && rss4 && proto == 6u) {
    const uint32_t g = fdir_match(p, src, dst, s.ports);
    if (g != 0xffffffffu) {
      s.fg = g;
      s.flags |= IXG_RF_FDIR;
    }
  }
}

// The record for a lane given its L4 residual: the residual computed, or a
// hypothesis (0 / non-zero) for a long segment whose tail is summed later.
// Mirrors the verdict order of the oracle's rx_one (driver checksum drops,
// then eth_input / ip_input / tcp_input head / udp_input / icmp_input).
// FIXED: the lane is known to be IPv4 with version 4, ihl 5 (the
// fixed-shape check), so the ethertype/version/ihl tests fold away.
template <bool FIXED = false>
DEV Rec make_record(const KParams& p, const uint32_t (&d)[kPrefixDw], uint32_t L, const LaneState& s,
                    uint32_t l4_res) {
  const uint32_t etype = FIXED ? 0x0800u : eth_type(d, L);
  const uint32_t vh = FIXED ? 0x45u : byte_at(d, 14);
  const uint32_t ver = vh >> 4, ihl = vh & 15u;
  const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
  const uint32_t ip_off = (byte_at(d, 20) << 8) | byte_at(d, 21);
  const bool frag = (ip_off & 0x3fffu) != 0;

  uint32_t flags = s.flags;
  if (s.l4_kind == 1) flags |= IXG_RF_L4_CSUM_CHECKED | (l4_res == 0 ? IXG_RF_L4_CSUM_OK : 0u);

  uint32_t v = 0, off = 0, len = 0, bucket = IXG_NO_BUCKET, tfl = 0;
  const bool csum_drop = !(p.flags & IXG_F_NO_CSUM_DROP);
  const uint32_t proto = s.proto, l4 = s.l4, l4len = s.l4len;
  if (csum_drop && (flags & IXG_RF_IP_CSUM_CHECKED) && !(flags & IXG_RF_IP_CSUM_OK)) {
    v = IXG_V_DROP_CSUM_IP;                                         // ixgbe.c:313-317
  } else if (csum_drop && (flags & IXG_RF_L4_CSUM_CHECKED) && !(flags & IXG_RF_L4_CSUM_OK)) {
    v = IXG_V_DROP_CSUM_L4;                                         // ixgbe.c:320-324
  } else if (etype == 0x0806u) {                                    // ip.c:134-135
    v = IXG_V_ARP; off = 14; len = L >= 14 ? L - 14 : 0;
  } else if (!s.v6 && etype != 0x0800u) {
    v = IXG_V_DROP_ETHERTYPE;                                       // ip.c:136-137
  } else {
    bool go = true;
    if (s.v6) {
      const uint32_t plen = (byte_at(d, 18) << 8) | byte_at(d, 19);
      if (!(L >= 54 && ver == 6 && 54 + plen <= L) || (proto != 6 && proto != 17)) {
        v = IXG_V_DROP_IP6; go = false;
      }
    } else {
      if (L < 34) v = IXG_V_DROP_IP_SHORT;                          // ip.c:68
      else if (ver != 4) v = IXG_V_DROP_IP_VERSION;                 // ip.c:71
      else if (ihl < 5) v = IXG_V_DROP_IP_IHL;                      // ip.c:74
      else if (frag) v = IXG_V_DROP_IP_FRAG;                        // ip.c:78
      else if (ip_len < 4 * ihl) v = IXG_V_DROP_IP_LEN;             // ip.c:85
      else if (14 + ip_len > L) v = IXG_V_DROP_IP_TRUNC;            // ip.c:87
      go = v == 0;
    }
    if (go) {
      if (proto == 6) {
        const uint32_t plen16 = l4len & 0xffffu;                    // misc.c:61 (u16)
        if (plen16 < 20) {
          v = IXG_V_DROP_TCP_SHORT;                                 // tcp_in.c:189
        } else if (s.doff != 0 && s.doff * 4 > plen16) {
          v = IXG_V_DROP_TCP_HDRLEN;                                // tcp_in.c:222, pbuf.c:461-465
        } else {
          v = s.v6 ? IXG_V_TCP6 : IXG_V_TCP;
          off = l4 + s.doff * 4;
          len = plen16 - s.doff * 4;
          tfl = s.tcp_flags;                                        // tcp_in.c:240
          if (!s.v6) bucket = s.bucket;                             // tcp_in.c:233
        }
      } else if (proto == 17) {
        if (l4 + s.ulen > L) {
          v = IXG_V_DROP_UDP_LEN;                                   // udp.c:59
        } else {
          v = s.v6 ? IXG_V_UDP6 : IXG_V_UDP;
          off = l4 + 8;                                             // udp.c:55
          len = s.ulen;                                             // udp.c:88
        }
      } else if (proto == 1 && !s.v6) {
        if (l4len < 8) v = IXG_V_DROP_ICMP_SHORT;                   // icmp.c:80
        else if (l4_res != 0) v = IXG_V_DROP_ICMP_CSUM;             // icmp.c:82
        else if (s.icmp_type != 8) v = IXG_V_DROP_ICMP_TYPE;        // icmp.c:88-108
        else { v = IXG_V_ICMP_ECHO; off = l4; len = l4len; }
      } else {
        v = s.v6 ? IXG_V_DROP_IP6 : IXG_V_DROP_IP_PROTO;            // ip.c:106-107
      }
    }
  }
  Rec r;
  r.w0 = (s.fg & 0xffffu) | (v << 16) | (flags << 24);
  r.w1 = (off & 0xffffu) | ((len & 0xffffu) << 16);
  r.w2 = s.rss;
  r.w3 = bucket | (tfl << 16);
  return r;
}

DEV uint32_t l4_residual(const LaneState& s) { return s.l4_kind ? ((~fold16(s.l4_acc)) & 0xffffu) : 0xffffu; }

// NT (the fixed-shape kernels): records are written once and not read back
// by this launch, so streaming (non-temporal) stores -- 4% faster on C2 than
// default-policy ones; the general kernels measured no gain
template <bool NT = false>
DEV void store_record(const KParams& p, uint32_t i, const Rec& r, uint32_t ip_res, uint32_t l4_res) {
  u32x4 w = {r.w0, r.w1, r.w2, r.w3};
  if (NT)
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p.out + i));
  else
    *reinterpret_cast<u32x4*>(p.out + i) = w;
  if (p.csum) p.csum[i] = ip_res | (l4_res << 16);
}

// Fused PCB demux (ixg_rx_demux_batch_dev): the tcp_input lookup of an
// IXG_V_TCP record straight from the parse state, no second pass over the
// frames or the records (ixgrx_walk.h; dp/net/tcp_in.c:233-323, 500-510).
// DMX false: a build without the fused demux (no lookup code in the kernel)
template <bool DMX = true>
DEV void store_demux(const KParams& p, uint32_t i, const Rec& r, uint32_t src, uint32_t dst, uint32_t ports) {
  if (!DMX || !p.dmx) return;
  uint32_t id = 0, kind = IXG_D_NONE;
  if (((r.w0 >> 16) & 0xffu) == IXG_V_TCP) {
    const ixgwalk::Tables t{p.active_start, p.bline, p.active, p.tw, p.listen, p.nfg + p.n_out, p.n_listen};
    ixgwalk::walk(t, ixg_demux_group(r.w0 & 0xffffu, p.fg_base, p.nfg, p.n_out), r.w3 & 0xffffu, (r.w3 >> 16) & 0xffu,
                  src, dst, ports, id, kind);
  }
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  reinterpret_cast<u32x2v*>(p.dmx)[i] = u32x2v{id, kind};
}

// Frame i's byte offset. The layout (u64 offsets vs fixed stride) is a
// template parameter, not a runtime branch: a branch on p.off makes hipcc
// join the two paths with a conservative s_waitcnt vmcnt(0) that drains
// every load in flight (and with it any software pipelining).
template <bool OFFS>
DEV uint64_t frame_off(const KParams& p, uint32_t i) {
  return OFFS ? p.off[i] : (uint64_t)i * p.stride;
}

// load 16-byte chunks [K0, K1) of the prefix; chunk k only if 16k < L.
// Raw: bytes at offsets >= L are never consumed unmasked (eth_type and the
// UDP length mask themselves; every other field sits behind a length check)
template <int K0, int K1>
DEV void load_prefix(const uint8_t* f, uint32_t L, const uint8_t* dummy, uint32_t (&d)[kPrefixDw]) {
  static_assert(K0 == 0, "prefix loads start at the frame start");
  // bytes 0..11 (MAC addresses) are never read: one dword for 12..15
  d[0] = d[1] = d[2] = 0;
  d[3] = *reinterpret_cast<const uint32_t*>((12u < L ? f : dummy) + 12);
#pragma unroll
  for (int k = K0 + 1; k < K1; k++) {
    const u32x4 v = load16((uint32_t)(16 * k) < L, f + 16 * k, dummy);
    d[4 * k + 0] = v.x;
    d[4 * k + 1] = v.y;
    d[4 * k + 2] = v.z;
    d[4 * k + 3] = v.w;
  }
}


// Bytes at offsets >= L read as zero, every dword at or past the wave's
// shortest frame masked (one compare + a wave-uniform branch per dword).
// The parse masks the two fields that can be consumed past L (eth_type,
// the UDP length), so the span kernel skips this (C5 -9 % in a
// same-process A/B); the long kernel keeps it (C3 2-3 % faster with it).
DEV void mask_prefix(uint32_t (&d)[kPrefixDw], uint32_t L) {
#pragma unroll
  for (int j = 3; j < kPrefixDw; j++)
    if (!wave_all(L >= 4u * (uint32_t)j + 4u)) d[j] = keep_bytes(d[j], (int)L - 4 * j);
}


// the fixed-shape path: everything in the 64-byte prefix
DEV void process_fast(const KParams& p, const uint64_t* __restrict__ T, uint32_t i, bool valid, uint32_t L,
                      const uint32_t (&d)[kPrefixDw]) {
  LaneState s;
  lane_parse<kShapeFixed, kFastDw>(p, Tab64{T}, d, L, s);
  if (valid) {
    const uint32_t r4 = l4_residual(s);
    const Rec r = make_record<true>(p, d, L, s, r4);
    store_record<true>(p, i, r, s.ip_res, r4);
    store_demux(p, i, r, s.src, s.dst, s.ports);
  }
}

// Buffer descriptors (gfx950 raw buffers, stride 0): the chunk's base and
// extent are scalars, each lane's offset a constant, and a piece past the
// extent reads 0 with no memory access (a store past it is dropped). So a
// chunk's loads and stores cost no per-lane address arithmetic.
constexpr int kRsrcWord3 = 0x00020000;  // 32-bit data format, raw addressing
constexpr int kAuxNT = 2;               // cache policy: nt (streaming)
DEV __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kRsrcWord3);
}

// ---- the lean fixed-shape path (C2's chunks) --------------------------------
// A one's complement (end-around carry) 32-bit sum, one v_add/v_addc per
// term: the carry travels between statements in an SGPR pair. Only
// additions, so the sum is 0 only when every term is 0, and congruent to the
// exact sum mod 2^32 - 1 (hence mod 0xffff: its 16-bit fold is the exact
// sum's for any non-zero sum).
struct Adc {
  uint32_t acc;
  uint64_t cc;
  DEV Adc(uint32_t a, uint32_t b) { asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(acc), "=s"(cc) : "v"(a), "v"(b)); }
  DEV void add(uint32_t x) { asm volatile("v_addc_co_u32 %0, %1, %0, %2, %1" : "+v"(acc), "+s"(cc) : "v"(x)); }
  DEV uint32_t end() {
    asm volatile("v_addc_co_u32 %0, %1, %0, 0, %1" : "+v"(acc), "+s"(cc));
    return acc;
  }
};

// 16-bit fold of a 32-bit one's complement sum (two adds of the halves)
DEV uint32_t fold32to16(uint32_t x) {
  x = (x & 0xffffu) + (x >> 16);
  return (x & 0xffffu) + (x >> 16);
}

// a ^ b ^ c in one v_bitop3_b32
DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// A fixed-shape chunk (every frame IPv4 ihl 5 inside 64 bytes, the check of
// fastc_loop) where, in addition, every frame is a TCP segment tcp_input
// accepts and all share one IP total length `ipl` (wave-uniform, so the
// segment end and every byte mask are scalars): C2's chunks, and a stream of
// 64-byte ACKs in general. Per lane what lane_parse + make_record<true>
// compute for such a frame, with no per-lane geometry: the IP header sum
// (bytes 14..33), the L4 sum (bytes 34..e) + pseudo header, the 12 hash
// lookups, and a verdict that can only be TCP or a checksum drop
// (ixgbe.c:312-324 then tcp_in.c:189-241). The caller guarantees per lane:
// proto 6, no fragment bits, 14 + ipl <= L, doff*4 <= ipl - 20 (TCPOK).
DEV Rec lean_tcp(const KParams& p, const uint64_t* __restrict__ T, uint32_t i, int lane,
                 const uint32_t (&d)[kPrefixDw], uint32_t ipl, __amdgpu_buffer_rsrc_t out) {
  // ---- IP header checksum: hi16(d3) + d4..d7 + lo16(d8) (chksum_internet) ----
  Adc ip(d[3] >> 16, d[4]);
  ip.add(d[5]);
  ip.add(d[6]);
  ip.add(d[7]);
  ip.add(d[8] & 0xffffu);
  const uint32_t ipf = fold32to16(ip.end());
  const bool ip_ok = ipf == 0xffffu;
  // ---- L4 sum over [34, e), e = 14 + ipl in [54, 64], plus the pseudo header
  // (inet_chksum_pseudo_partial): src + dst as 16-bit halves = hi16(d6) +
  // lo16(d7) + hi16(d7) + lo16(d8), which is congruent mod 0xffff to hi16(d6)
  // + d7 + lo16(d8); with the segment's hi16(d8) that is d7 + d8 (a 32-bit
  // word counts as its two halves mod 0xffff). The sum is non-zero (proto
  // term), so the congruent sum folds to the same 16 bits.
  const uint32_t e = 14u + ipl;  // scalar
  const uint32_t l4len = ipl - 20u;
  auto keep = [](uint32_t x, int t) -> uint32_t {  // scalar mask of the first t bytes
    return t >= 4 ? x : (t <= 0 ? 0u : x & ((1u << (8 * t)) - 1u));
  };
  const uint32_t m13 = keep(~0u, (int)e - 52), m14 = keep(~0u, (int)e - 56), m15 = keep(~0u, (int)e - 60);
  const uint32_t kps = (6u << 8) + bswap16(l4len);  // htons(proto) + htons(proto_len)
  Adc l4(d[6] >> 16, d[7]);
  l4.add(d[8]);
  l4.add(d[9]);
  l4.add(d[10]);
  l4.add(d[11]);
  l4.add(d[12]);
  l4.add(d[13] & m13);
  l4.add(d[14] & m14);
  l4.add(d[15] & m15);
  l4.add(kps);
  const uint32_t l4f = fold32to16(l4.end());
  const bool l4_ok = l4f == 0xffffu;
  // ---- Toeplitz + tcp_to_idx: tuple bytes 26..37 (src, dst, sport, dport) ----
  uint64_t h[12];
#pragma unroll
  for (int k = 0; k < 12; k++) h[k] = T[(k << 8) | byte_at(d, 26 + k)];
  const uint32_t rlo = xor3(xor3((uint32_t)h[0], (uint32_t)h[1], (uint32_t)h[2]),
                            xor3((uint32_t)h[3], (uint32_t)h[4], (uint32_t)h[5]),
                            xor3(xor3((uint32_t)h[6], (uint32_t)h[7], (uint32_t)h[8]),
                                 xor3((uint32_t)h[9], (uint32_t)h[10], (uint32_t)h[11]), 0u));
  const uint32_t rhi = xor3(xor3((uint32_t)(h[0] >> 32), (uint32_t)(h[1] >> 32), (uint32_t)(h[2] >> 32)),
                            xor3((uint32_t)(h[3] >> 32), (uint32_t)(h[4] >> 32), (uint32_t)(h[5] >> 32)),
                            xor3(xor3((uint32_t)(h[6] >> 32), (uint32_t)(h[7] >> 32), (uint32_t)(h[8] >> 32)),
                                 xor3((uint32_t)(h[9] >> 32), (uint32_t)(h[10] >> 32), (uint32_t)(h[11] >> 32)),
                                 p.crc_const));
  uint32_t fg = p.fg_base | (rlo & p.fg_mask);
  uint32_t flags = IXG_RF_IP_CSUM_CHECKED | IXG_RF_L4_CSUM_CHECKED | IXG_RF_RSS | (ip_ok ? IXG_RF_IP_CSUM_OK : 0u) |
                   (l4_ok ? IXG_RF_L4_CSUM_OK : 0u);
  {  // flow-director filters (one scalar header load when none are installed)
    const uint32_t src = (d[6] >> 16) | (d[7] << 16), dst = (d[7] >> 16) | (d[8] << 16);
    const uint32_t ports = bswap16(d[8] >> 16) | (bswap16(d[9] & 0xffffu) << 16);
    const uint32_t g = fdir_match(p, src, dst, ports);
    if (g != 0xffffffffu) {
      fg = g;
      flags |= IXG_RF_FDIR;
    }
  }
  // ---- verdict: the driver's checksum drops, else tcp_input's delivery ----
  const uint32_t doff4 = (d[11] >> 18) & 0x3cu;  // TCPH_HDRLEN * 4 (tcp_in.c:222)
  const bool drop = !(p.flags & IXG_F_NO_CSUM_DROP) && !(ip_ok && l4_ok);
  const uint32_t v = drop ? (ip_ok ? IXG_V_DROP_CSUM_L4 : IXG_V_DROP_CSUM_IP) : IXG_V_TCP;
  Rec r;
  r.w0 = (fg & 0xffffu) | (v << 16) | (flags << 24);
  r.w1 = drop ? 0u : ((34u + doff4) | ((l4len - doff4) << 16));
  r.w2 = rlo;
  r.w3 = drop ? IXG_NO_BUCKET : ((rhi & (IXG_PCB_BUCKETS - 1)) | (((d[11] >> 24) & 0x3fu) << 16));
  // (out covers the chunk's valid frames only: the stores of other lanes drop)
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{r.w0, r.w1, r.w2, r.w3}, out, 16 * lane, 0, kAuxNT);
  if (p.csum && i < p.n) p.csum[i] = ((~ipf) & 0xffffu) | (((~l4f) & 0xffffu) << 16);
  return r;
}

// the 4-tuple of a lean chunk's frame (bytes 26..37) as the fused demux takes
// it: raw IPs, ports host order (sport | dport << 16)
DEV void lean_tuple(const uint32_t (&d)[kPrefixDw], uint32_t& src, uint32_t& dst, uint32_t& ports) {
  src = (d[6] >> 16) | (d[7] << 16);
  dst = (d[7] >> 16) | (d[8] << 16);
  ports = bswap16(d[8] >> 16) | (bswap16(d[9] & 0xffffu) << 16);
}

// LDS (address space 3) pointers: through generic pointers these would be
// flat_* accesses, which count on vmcnt as well and force vmcnt(0) waits
// that serialise the streaming loads.
#define LDS(T, x) ((T*)(x))

// masked sum of a 16-byte piece whose first byte is `rem` bytes before the
// segment end (rem <= 0: nothing of it is inside)
DEV uint64_t piece_sum(const u32x4& v, int rem) {
  return (uint64_t)(v.x & ones(rem < 0 ? 0 : rem)) + (v.y & ones(rem - 4 < 0 ? 0 : rem - 4)) +
         (v.z & ones(rem - 8 < 0 ? 0 : rem - 8)) + (v.w & ones(rem - 12 < 0 ? 0 : rem - 12));
}

// ---- general path -------------------------------------------------------
// Pass A: lane per packet, 96-byte prefix, full parse. Lanes whose L4
// segment runs past the prefix ("long") are compacted per wave (ballot +
// mbcnt) into an LDS list and their tails [96, end) are streamed by groups
// of kG lanes, kRoundPk packets per round, kT 16-byte loads per lane per
// round (2 KiB per packet). Rounds use two register buffers A/B whose loads
// are always issued (dummy when a group has no packet), so hipcc's vmcnt
// waits for one buffer never cover the other.
constexpr int kG = 16;
constexpr int kRoundPk = 64 / kG;
constexpr int kT = 8;

struct WaveLds {  // per-wave scratch, LDS address space
  lds_u32* list;  // compacted long lanes
  lds_u32* end;   // per lane: end of the whole 16-byte pieces to stream
  lds_u32* offlo; // per lane: frame offset (low/high words)
  lds_u32* offhi;
  lds_u32* sum;   // per lane: streamed tail sum
  const lds_u32* t6;  // IPv6 Toeplitz table (IXG_F_IPV6), block-shared
  lds_u32* pre;   // big chunks: the 64 frames' prefixes (kPrefixDw dwords each)
};

struct Round {
  u32x4 v[kT];
  uint32_t end;   // owner's end of whole pieces (0: this group has no packet)
  uint32_t owner;
  uint32_t gsh;   // general rounds: log2 of the group size
  u32x4 ve;       // big rounds: the piece holding the frame end (group lane 0)
};

// Which list entry a round's group streams (SM, the stream mapping):
// 0: every long segment by a 16-lane group, 4 per round, 2 KiB each.
// 1: rounds [0, rm) take the medium segments (whole pieces ending at or
//    below kStreamBase + kMedSpan) by 4-lane groups, 16 per round, 512 B
//    each; the rounds after take the rest as in 0.
// 2: packed: the list (medium entries first) laid out over consecutive
//    lanes, 4 per medium entry and 16 per other entry (the first of those
//    16-aligned), 64 lanes per round; tail rounds of the two kinds share.
// (16-lane groups alone: a 590-B frame's 31 pieces used 31 of a group's 128
// load slots.)
constexpr uint32_t kMedG = 4;
constexpr uint32_t kMedSpan = 16u * kMedG * kT;  // 512
struct RoundPlan {
  uint32_t nmed;   // list entries [0, nmed): medium segments
  uint32_t nlong;  // list entries [0, nlong): every long segment
  uint32_t rm;     // SM 1: rounds of medium segments
};

template <int SM>
DEV void round_issue(const KParams& p, const WaveLds& w, uint32_t r, const RoundPlan& plan, int lane, Round& b) {
  uint32_t gsh, k;
  bool act;
  if (SM == 2) {
    const uint32_t G = 64u * r + (uint32_t)lane, bigb = 4u * ((plan.nmed + 3u) & ~3u);
    const bool big = G >= bigb;
    gsh = big ? 4u : 2u;
    k = big ? plan.nmed + ((G - bigb) >> 4) : G >> 2;
    act = big ? k < plan.nlong : k < plan.nmed;
  } else {
    const bool med = SM == 1 && r < plan.rm;  // wave-uniform
    gsh = med ? 2u : 4u;
    const uint32_t g = (uint32_t)lane >> gsh;
    k = med ? r * (64u >> gsh) + g : plan.nmed + (r - plan.rm) * (uint32_t)kRoundPk + g;
    act = k < (med ? plan.nmed : plan.nlong);
  }
  const uint32_t gl = (uint32_t)lane & ((1u << gsh) - 1u);
  const uint32_t owner = w.list[act ? k : 0u];
  b.owner = owner;
  b.gsh = gsh;
  b.end = act ? w.end[owner] : 0u;
  const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
  const uint8_t* f = p.base + off;
  // pieces at or past the segment end read the zero page: they add nothing
  const uint8_t* zero = p.zero + 16 * lane;
#pragma unroll
  for (int t = 0; t < kT; t++) {
    const uint32_t pos = kStreamBase + 16u * gl + (16u << gsh) * (uint32_t)t;
    b.v[t] = load16(pos < b.end, f + pos, zero);
  }
}

template <int SM>
DEV void round_finish(const KParams& p, const WaveLds& w, int lane, const Round& b) {
  const uint32_t gsh = SM ? b.gsh : 4u;
  const uint32_t gsz = 1u << gsh;
  const uint32_t gl = (uint32_t)lane & (gsz - 1u);
  // every piece is inside the segment or reads the zero page (pass A summed
  // the piece holding the segment end, masked): plain one's complement sums
  static_assert(kT % 4 == 0, "two interleaved chains of piece pairs");
  uint32_t a = 0, a1 = 0;
#pragma unroll
  for (int t = 0; t < kT; t += 4) adc8x2(a, b.v[t], b.v[t + 1], a1, b.v[t + 2], b.v[t + 3]);
  a = add1c(a, a1);
  // frames longer than 96 + 2 KiB (not IX mbufs): the rest, synchronously
  const uint32_t more = kStreamBase + (16u << gsh) * kT;
  if (wave_any(b.end > more)) {
    const uint64_t off = ((uint64_t)w.offhi[b.owner] << 32) | w.offlo[b.owner];
    const uint8_t* zero = p.zero + 16 * lane;
    for (uint32_t pos0 = more; wave_any(pos0 < b.end); pos0 += 32u * gsz) {
      const uint32_t pos = pos0 + 16u * gl;
      const u32x4 v0 = load16(pos < b.end, p.base + off + pos, zero);
      const u32x4 v1 = load16(pos + 16u * gsz < b.end, p.base + off + pos + 16u * gsz, zero);
      a = adc8(a, v0, v1);
    }
  }
  // group reduction: every lane shuffles (SM 2 mixes group sizes in a
  // wave); xor partners below a lane's group size stay in its group
#pragma unroll
  for (uint32_t m = 1; m < (uint32_t)kG; m <<= 1) {
    const uint32_t x = (uint32_t)__shfl_xor((int)a, (int)m);
    if (m < gsz) a = add1c(a, x);
  }
  if (gl == 0 && b.end != 0u) w.sum[b.owner] = a;
}

// A chunk's descriptors and frame bytes, loaded ahead by general_body's
// pipeline (descriptors two chunks ahead, bytes one chunk ahead).
struct GDesc {
  uint32_t L;
  uint64_t off;
};
struct GPre {
  uint32_t d[kPrefixDw];  // bytes 0..95 (0..11 never loaded), zero past L
  u32x4 v96;              // bytes 96..111 of frames shorter than 128 B, else zero page
};

constexpr uint32_t kNoChunk = 0xffffffffu;
// the long kernel's chunk order: runs of kRun consecutive chunks per wave,
// kRunBig when the sample is mostly big chunks (general_body)
constexpr uint64_t kRun = 64, kRunBig = 1;
constexpr bool kPreT = true;  // the long walk's transposed prefix load (gen_pre_t)
// the coalesced fixed-shape kernel's (fastc_loop)
constexpr uint32_t kRunC = 2;
// the span-staged short kernel's (short_span_body)
constexpr uint32_t kRunS = 1;
static_assert(64 % kRunC == 0, "whole runs within a wave's 64 drained chunks");
// big chunks: every frame at least this long (or past the batch end)
constexpr uint32_t kBigMin = 256;

template <bool OFFS>
DEV void gen_desc(const KParams& p, uint32_t chunk, int lane, GDesc& g) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = chunk != kNoChunk && i < p.n;
  const uint32_t ic = valid ? i : 0u;  // clamped: descriptor loads without a branch
  g.L = valid ? (uint32_t)p.len[ic] : 0u;
  g.off = frame_off<OFFS>(p, ic);
}

// every load is issued (zero page / dummy when there is nothing to read), so
// hipcc's vmcnt accounting stays exact across the pipeline
// GATE: load nothing for a chunk with a frame of IXG_SHORT_MAX bytes or more
// (the short-first pass leaves such chunks to the long kernel)
// (a big chunk, see big_chunk, loads its prefixes in its rounds instead)
template <bool GATE = false, bool BIG = false>
DEV void gen_pre(const KParams& p, const GDesc& g, int lane, GPre& x) {
  const bool skip = GATE ? !wave_all(g.L < IXG_SHORT_MAX) : (BIG && wave_all(g.L >= kBigMin || g.L == 0u));
  const uint32_t Lg = skip ? 0u : g.L;
  load_prefix<0, 6>(p.base + g.off, Lg, reinterpret_cast<const uint8_t*>(p.tab), x.d);
  const bool short_tail = g.L > (uint32_t)kStreamBase && g.L < (uint32_t)kStreamBase + 32u;
  x.v96 = load16(short_tail, p.base + g.off + kStreamBase, p.zero + 16 * lane);
}

// The long kernel's prefix load, transposed through LDS: the 64 frames' 6
// prefix pieces (bytes 0..95) are numbered frame-major, and wave instruction
// t loads pieces 64t .. 64t+63, i.e. ~11 frames' consecutive pieces, instead
// of one piece of each of the 64 frames (64 cache lines per instruction,
// which stalled the L1 on their misses: C3's prefix phase alone ran at ~2.8
// TB/s). The pieces go to the wave's LDS stash (w.pre, 64 x 96 B) and each
// lane reads its own frame's row back. Synchronous: the caller uses it where
// the prefix is waited for at once (the walk without the one-ahead prefetch).
template <bool BIG>
DEV void gen_pre_t(const KParams& p, const GDesc& g, int lane, const WaveLds& w, GPre& x) {
  const bool skip = BIG && wave_all(g.L >= kBigMin || g.L == 0u);
  const bool short_tail = g.L > (uint32_t)kStreamBase && g.L < (uint32_t)kStreamBase + 32u;
  x.v96 = load16(short_tail, p.base + g.off + kStreamBase, p.zero + 16 * lane);
  x.d[0] = x.d[1] = x.d[2] = 0;
  if (skip) {  // a big chunk loads its prefixes in its rounds (big_chunk)
#pragma unroll
    for (int k = 3; k < kPrefixDw; k++) x.d[k] = 0u;
    return;
  }
  w.offlo[lane] = (uint32_t)g.off;
  w.offhi[lane] = (uint32_t)(g.off >> 32);
  w.end[lane] = g.L;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  u32x4 v[6];
#pragma unroll
  for (int t = 0; t < 6; t++) {
    const uint32_t q = 64u * (uint32_t)t + (uint32_t)lane, f = q / 6u, j = q - 6u * f;
    const uint64_t o = ((uint64_t)w.offhi[f] << 32) | w.offlo[f];
    v[t] = load16(16u * j < w.end[f], p.base + o + 16u * j, p.zero + 16 * lane);
  }
#pragma unroll
  for (int t = 0; t < 6; t++) {
    lds_u32* st = w.pre + 4u * (64u * (uint32_t)t + (uint32_t)lane);  // row f, piece j = dword 24 f + 4 j
    st[0] = v[t].x; st[1] = v[t].y; st[2] = v[t].z; st[3] = v[t].w;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const lds_u32* row = w.pre + (uint32_t)lane * kPrefixDw;
#pragma unroll
  for (int k = 3; k < kPrefixDw; k++) x.d[k] = row[k];
  // (the stash is read before anything else writes it: the big-chunk path
  // fills it only inside big_chunk, after this wave's reads)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- big chunks ---------------------------------------------------------
// A chunk whose frames are all >= kBigMin bytes (the 1500 B configs) skips
// the lane-per-frame prefix pass: 16-lane groups stream every frame from
// byte 0, 4 frames per round, and the pieces of bytes [0, 96) go to the
// wave's LDS stash instead of the sum, so each frame's bytes are fetched
// once, by one group, in one round (a separate prefix pass fetches the lines
// holding byte 12 and byte 96 a second time, by then evicted from L2: C4's
// traffic was 1.18x the frame bytes). The streamed sum covers [96, L); the
// lane then parses its prefix from LDS. A segment ending before L (IPv4
// ip_len short of the frame) re-sums [96, seg_end) on its own (rare).

// FPW: the frames a wave takes (64: a chunk; fewer: the host-memory kernel)
template <uint32_t FPW = 64>
DEV void big_issue(const KParams& p, const WaveLds& w, uint32_t r, int lane, Round& b) {
  const int g = lane / kG, gl = lane % kG;
  const uint32_t k = r * kRoundPk + (uint32_t)g;
  const bool act = k < FPW;
  const uint32_t owner = act ? k : 0u;
  b.owner = k;
  b.end = act ? w.end[owner] : 0u;
  const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
  const uint8_t* f = p.base + off;
  const uint8_t* zero = p.zero + 16 * lane;
  // whole pieces only; the piece holding L (if L is not a multiple of 16)
  // is group lane 0's extra load, masked in big_finish
  const uint32_t whole = b.end & ~15u;
#pragma unroll
  for (int t = 0; t < kT; t++) {
    const uint32_t pos = 16u * gl + 16u * kG * t;
    b.v[t] = load16(pos < whole, f + pos, zero);
  }
  b.ve = load16(gl == 0 && whole < b.end && whole < 16u * kG * kT, f + whole, zero);
}

DEV u32x4 mask_piece(const u32x4& v, int rem) {
  return u32x4{v.x & ones(rem < 0 ? 0 : rem), v.y & ones(rem - 4 < 0 ? 0 : rem - 4),
               v.z & ones(rem - 8 < 0 ? 0 : rem - 8), v.w & ones(rem - 12 < 0 ? 0 : rem - 12)};
}

template <uint32_t FPW = 64>
DEV void big_finish(const KParams& p, const WaveLds& w, int lane, Round& b) {
  const int gl = lane % kG;
  static_assert(kStreamBase == 16 * 6 && kPrefixDw == 24, "the prefix is pieces 0..5 of round slot t = 0");
  if (gl < 6 && b.owner < FPW) {
    lds_u32* q = w.pre + b.owner * kPrefixDw + 4 * gl;
    q[0] = b.v[0].x; q[1] = b.v[0].y; q[2] = b.v[0].z; q[3] = b.v[0].w;
  }
  if (gl < 6) b.v[0] = u32x4{0u, 0u, 0u, 0u};
  uint32_t a = 0, a1 = 0;
#pragma unroll
  for (int t = 0; t < kT; t += 4) adc8x2(a, b.v[t], b.v[t + 1], a1, b.v[t + 2], b.v[t + 3]);
  a = add1c(a, a1);
  // the end piece (zero page in every other lane): masked to L
  const u32x4 ve = mask_piece(b.ve, (int)(b.end & 15u));
  a = add1c(a, fold32((uint64_t)ve.x + ve.y + ve.z + ve.w));
  // frames longer than 2 KiB (not IX mbufs): the rest, synchronously
  const uint32_t more = 16u * kG * kT;
  if (wave_any(b.end > more)) {
    const uint32_t owner = b.owner < FPW ? b.owner : 0u;
    const uint64_t off = ((uint64_t)w.offhi[owner] << 32) | w.offlo[owner];
    const uint8_t* zero = p.zero + 16 * lane;
    for (uint32_t pos0 = more; wave_any(pos0 < b.end); pos0 += 16u * kG) {
      const uint32_t pos = pos0 + 16u * gl;
      // (b.ve did not load the end piece of such a frame)
      const u32x4 v = mask_piece(load16(pos < b.end, p.base + off + pos, zero), (int)b.end - (int)pos);
      a = add1c(a, fold32((uint64_t)v.x + v.y + v.z + v.w));
    }
  }
#pragma unroll
  for (int m = 1; m < kG; m <<= 1) a = add1c(a, (uint32_t)__shfl_xor((int)a, m, kG));
  if (gl == 0 && b.owner < FPW) w.sum[b.owner] = a;
}

// one's complement sum of the frame bytes [a, e) (a 16-aligned), lane-serial
DEV uint32_t span_sum(const KParams& p, uint64_t off, uint32_t a, uint32_t e) {
  uint64_t s = 0;
  for (uint32_t pos = a; pos < e; pos += 16u) {
    const u32x4 v = mask_piece(load16(true, p.base + off + pos, p.zero), (int)(e - pos));
    s += (uint64_t)v.x + v.y + v.z + v.w;
  }
  return fold32(s);
}

template <bool OFFS, bool DMX = true, uint32_t FPW = 64>
DEV void big_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane, const WaveLds& w,
                   const GDesc& g) {
  static_assert(FPW % (2 * kRoundPk) == 0 && FPW <= 64, "whole round pairs");
  const uint32_t i = chunk * FPW + (uint32_t)lane;
  const bool valid = (uint32_t)lane < FPW && i < p.n;
  const uint32_t L = g.L;  // 0 past the end
  w.end[lane] = L;
  w.offlo[lane] = (uint32_t)g.off;
  w.offhi[lane] = (uint32_t)(g.off >> 32);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  constexpr uint32_t R = FPW / kRoundPk;
  Round A, B;
  big_issue<FPW>(p, w, 0, lane, A);
#pragma clang loop unroll(disable)
  for (uint32_t r = 0; r < R; r += 2) {
    big_issue<FPW>(p, w, r + 1, lane, B);
    big_finish<FPW>(p, w, lane, A);
    big_issue<FPW>(p, w, r + 2, lane, A);
    big_finish<FPW>(p, w, lane, B);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint32_t d[kPrefixDw];
  d[0] = d[1] = d[2] = 0;  // MAC addresses: never read
  const lds_u32* q = w.pre + lane * kPrefixDw;
#pragma unroll
  for (int j = 3; j < kPrefixDw; j++) d[j] = q[j];  // L >= 96: no masking
  LaneState s;
  const bool fixed = !valid || (eth_type(d, L) == 0x0800u && byte_at(d, 14) == 0x45u);
  if (wave_all(fixed))
    lane_parse<kShapeFixed, kPrefixDw>(p, Tab64{T}, d, L, s);
  else
    lane_parse<kShapeAny, kPrefixDw>(p, Tab64{T}, d, L, s, w.t6);
  if (!valid) return;
  uint32_t res = l4_residual(s);
  if (s.stream) {
    const uint32_t tail = s.seg_end == L ? w.sum[lane] : span_sum(p, g.off, (uint32_t)kStreamBase, s.seg_end);
    res = (~fold16(add1c(fold32(s.l4_acc), tail))) & 0xffffu;
  }
  const Rec r = make_record(p, d, L, s, res);
  store_record(p, i, r, s.ip_res, res);
  store_demux<DMX>(p, i, r, s.src, s.dst, s.ports);
}

// MODE: kModeLong: any chunk; kModeFirst (the short kernel): the chunk's
// class is checked here, a chunk with a frame of IXG_SHORT_MAX bytes or more
// is flagged for the long kernel, and for the others no segment needs the
// streaming rounds (compiled out). Returns true when the chunk was deferred.
constexpr int kModeLong = 0, kModeFirst = 2;

// BIG: big chunks take big_chunk (the walks without the one-ahead prefix
// prefetch, so its registers are not live across the rounds)
// LATE (long mode without the one-ahead prefetch): the next chunk's prefix
// (Dn -> Pn) is loaded here, after this chunk's last streaming round is
// issued (its registers free by then), instead of after this chunk, where
// the next chunk waited out its whole latency
template <bool OFFS, int MODE, bool BIG, int SM = 0, bool LATE = false, bool DMX = true>
DEV bool general_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane,
                       const WaveLds& w, const GDesc& g, const GPre& x, const GDesc* Dn = nullptr,
                       GPre* Pn = nullptr) {
  constexpr bool SHORT = MODE != kModeLong;
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;
  if (MODE == kModeFirst) {
    const bool defer = !wave_all(L < IXG_SHORT_MAX);  // L = 0 past the end
    if (lane == 0) p.defer[chunk] = defer ? (uint8_t)IXG_CLS_LONG : (uint8_t)0;
    if (defer) return true;
  }
  if (BIG && wave_all(g.L >= kBigMin || g.L == 0u)) {
    big_chunk<OFFS, DMX>(p, T, chunk, lane, w, g);
    if (LATE) gen_pre<false, BIG>(p, *Dn, lane, *Pn);
    return false;
  }
  const uint64_t off = g.off;
  uint32_t d[kPrefixDw];
#pragma unroll
  for (int j = 0; j < kPrefixDw; j++) d[j] = x.d[j];
  // (not needed for the results, eth_type and the UDP length mask
  // themselves; but C3 measured 2-3 % faster with it in a same-process A/B)
  mask_prefix(d, L);
  const u32x4& v96 = x.v96;
  const bool short_tail = L > (uint32_t)kStreamBase && L < (uint32_t)kStreamBase + 32u;
  LaneState s;
  const bool fixed = !valid || (eth_type(d, L) == 0x0800u && byte_at(d, 14) == 0x45u);
  if (wave_all(fixed))
    lane_parse<kShapeFixed, kPrefixDw>(p, Tab64{T}, d, L, s);
  else
    lane_parse<kShapeAny, kPrefixDw>(p, Tab64{T}, d, L, s, w.t6);
  // The 16-byte piece (counted from byte 96) holding the segment end is
  // summed by this lane, masked to the segment; streaming rounds read only
  // the whole pieces before it. A segment ending within 16 bytes past the
  // prefix is finished with v96; a longer one loads its end piece now and
  // adds it after the rounds, so the load's latency hides behind them.
  const bool strm = valid && s.stream;
  const uint32_t tail = s.seg_end - (uint32_t)kStreamBase;
  const uint32_t rr = tail & 15u, pend = (uint32_t)kStreamBase + (tail & ~15u);
  const bool lng = !SHORT && strm && (pend > (uint32_t)kStreamBase || !short_tail);
  if (strm && !lng) s.l4_acc += piece_sum(v96, (int)rr);
  const uint64_t m = SHORT ? 0ull : __ballot(lng);
  if (SHORT || !m) {  // no long segment in this chunk (wave-uniform)
    if (LATE) gen_pre<false, BIG>(p, *Dn, lane, *Pn);
    if (valid) {
      const uint32_t r4 = l4_residual(s);
      const Rec r = make_record(p, d, L, s, r4);
      store_record(p, i, r, s.ip_res, r4);
      store_demux<DMX>(p, i, r, s.src, s.dst, s.ports);
    }
    return false;
  }
  // records for both outcomes of the pending L4 check; then only these
  // few registers stay live across the streaming rounds
  const uint32_t r4 = lng ? 0u : l4_residual(s);
  Rec rok = make_record(p, d, L, s, r4);
  Rec rbad = make_record(p, d, L, s, 1u);
  uint32_t acc32 = fold32(s.l4_acc), ip_res = s.ip_res;
  uint32_t tsrc = s.src, tdst = s.dst, tports = s.ports;
  const u32x4 ve = load16(lng && rr != 0u, p.base + off + pend, p.zero + 16 * lane);
  // materialise these now, so the parse state (d[], s) is dead during the
  // streaming rounds instead of being kept live for sunk computations
  asm volatile("" : "+v"(rok.w0), "+v"(rok.w1), "+v"(rok.w2), "+v"(rok.w3));
  asm volatile("" : "+v"(rbad.w0), "+v"(rbad.w1), "+v"(rbad.w2), "+v"(rbad.w3));
  asm volatile("" : "+v"(acc32), "+v"(ip_res));
  asm volatile("" : "+v"(tsrc), "+v"(tdst), "+v"(tports));
  // SM > 0: the medium segments first in the list, then the rest
  constexpr bool MED = SM != 0;
  const bool lmed = MED && lng && pend <= (uint32_t)kStreamBase + kMedSpan;
  const uint64_t mm = MED ? __ballot(lmed) : 0ull, mb = MED ? m & ~mm : m;
  const uint32_t nmed = (uint32_t)__popcll(mm);
  if (lng) {
    const uint64_t mine = lmed ? mm : mb;
    const uint32_t at = (lmed ? 0u : nmed) +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
    w.list[at] = (uint32_t)lane;
    w.end[lane] = pend;
    w.offlo[lane] = (uint32_t)off;
    w.offhi[lane] = (uint32_t)(off >> 32);
  }
  __builtin_amdgcn_wave_barrier();
  const uint32_t nlong = (uint32_t)__popcll(m);
  const RoundPlan plan{nmed, nlong, SM == 1 ? (nmed + 64u / kMedG - 1u) / (64u / kMedG) : 0u};
  const uint32_t R = SM == 2 ? (4u * ((nmed + 3u) & ~3u) + 16u * (nlong - nmed) + 63u) / 64u
                             : plan.rm + (nlong - nmed + kRoundPk - 1) / kRoundPk;
  Round A, B;
  round_issue<SM>(p, w, 0, plan, lane, A);
  if (LATE) {
    // pairs while more than two rounds remain, then the last one or two
    // (a dummy B when one) with the next prefix issued behind them
    uint32_t r = 0;
#pragma clang loop unroll(disable)
    for (; r + 2 < R; r += 2) {
      round_issue<SM>(p, w, r + 1, plan, lane, B);
      round_finish<SM>(p, w, lane, A);
      round_issue<SM>(p, w, r + 2, plan, lane, A);
      round_finish<SM>(p, w, lane, B);
    }
    round_issue<SM>(p, w, r + 1, plan, lane, B);
    gen_pre<false, BIG>(p, *Dn, lane, *Pn);
    round_finish<SM>(p, w, lane, A);
    round_finish<SM>(p, w, lane, B);
  } else {
#pragma clang loop unroll(disable)
    for (uint32_t r = 0; r < R; r += 2) {
      round_issue<SM>(p, w, r + 1, plan, lane, B);
      round_finish<SM>(p, w, lane, A);
      round_issue<SM>(p, w, r + 2, plan, lane, A);
      round_finish<SM>(p, w, lane, B);
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (valid) {
    if (lng) {
      const uint32_t end_piece = fold32(piece_sum(ve, (int)rr));
      const uint32_t res = (~fold16(add1c(add1c(acc32, w.sum[lane]), end_piece))) & 0xffffu;
      store_record(p, i, res == 0 ? rok : rbad, ip_res, res);
      store_demux<DMX>(p, i, res == 0 ? rok : rbad, tsrc, tdst, tports);
    } else {
      store_record(p, i, rok, ip_res, r4);
      store_demux<DMX>(p, i, rok, tsrc, tdst, tports);
    }
  }
  return false;
}

// stage the hash tables (24 KiB) once per persistent workgroup
DEV void stage_tables(const KParams& p, uint64_t* T) {
  for (int k = threadIdx.x; k < 12 * 256 / 2; k += blockDim.x) {
    const u32x4 v = reinterpret_cast<const u32x4*>(p.tab)[k];
    reinterpret_cast<u32x4*>(T)[k] = v;
  }
  __syncthreads();
}

// ---- frames in host memory, all long ---------------------------------------
// A batch in host memory (the asynchronous path's DIRECT mode) whose frames
// are all at least kBigMin bytes (KParams.long_only): every load crosses the
// host link, so a wave's time is its round trips, not its bytes. A 64-frame
// chunk per wave is 16 rounds of 4 frames (8 round trips with two rounds in
// flight): a 1514-B batch took 28-34 us per launch whether it held 342 or
// 683 frames. Here a wave takes kHostFpw frames (kHostFpw / 4 rounds), so a
// batch spreads over 64 / kHostFpw times the waves and has that many more
// bytes in flight; the per-frame work (big_chunk) is the same.
#ifndef IXG_HOST_FPW
#define IXG_HOST_FPW 8
#endif
constexpr uint32_t kHostFpw = IXG_HOST_FPW;

template <bool OFFS>
DEV void host_big_body(const KParams& p) {
  __shared__ uint64_t T[12 * 256];
  __shared__ uint32_t sh_end[kWaves][64], sh_offlo[kWaves][64], sh_offhi[kWaves][64], sh_sum[kWaves][64];
  __shared__ uint32_t sh_pre[kWaves][64 * kPrefixDw];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  extern __shared__ u32x4 dyn6[];
  if (p.tab6) {
    for (int k = threadIdx.x; k < (int)IXG_TAB6_WORDS / 4; k += 64 * kWaves) dyn6[k] = reinterpret_cast<const u32x4*>(p.tab6)[k];
  }
  stage_tables(p, T);
  const WaveLds w{nullptr, LDS(lds_u32, sh_end[wave]), LDS(lds_u32, sh_offlo[wave]), LDS(lds_u32, sh_offhi[wave]),
                  LDS(lds_u32, sh_sum[wave]), LDS(const lds_u32, dyn6), LDS(lds_u32, sh_pre[wave])};
  const uint32_t nsub = (p.n + kHostFpw - 1u) / kHostFpw;
  for (uint32_t c = blockIdx.x * kWaves + (uint32_t)wave; c < nsub; c += gridDim.x * kWaves) {
    const uint32_t i = c * kHostFpw + (uint32_t)lane;
    const bool valid = (uint32_t)lane < kHostFpw && i < p.n;
    const uint32_t ic = valid ? i : 0u;
    GDesc g;
    g.L = valid ? (uint32_t)p.len[ic] : 0u;
    g.off = frame_off<OFFS>(p, ic);
    big_chunk<OFFS, false, kHostFpw>(p, T, c, lane, w, g);
  }
}

extern "C" __global__ void __launch_bounds__(kBlock) ixg_rx_host_big_s(KParams p) { host_big_body<false>(p); }
extern "C" __global__ void __launch_bounds__(kBlock) ixg_rx_host_big_o(KParams p) { host_big_body<true>(p); }

// ---- fixed-shape kernel --------------------------------------------------
// Software-pipelined over the wave's chunks (64 packets each, grid-stride):
// descriptors (len, offset) are fetched two chunks ahead, the 64-byte
// prefixes one chunk ahead, so a wave always has its next chunk's frame
// bytes in flight while it computes the current one. Chunks that are not
// all "fast shape" are flagged for the general kernel.

template <bool OFFS>
DEV void fetch_desc(const KParams& p, uint32_t chunk, int lane, uint32_t& L, uint64_t& o) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const uint32_t ic = i < p.n ? i : p.n - 1;  // clamped, branch-free
  L = p.len[ic];
  o = frame_off<OFFS>(p, ic);
}

// The fast path never reads bytes 0..11 (MAC addresses): load exactly
// bytes 12..63 (one dword + three 16-byte loads). Loading 0..15 as one
// dwordx4 leaves dead lanes in the destination that the register allocator
// reuses at once, and that write-after-write forces a vmcnt(0) right after
// the prefetch is issued.
struct Prefix {
  uint32_t w3;   // bytes 12..15
  u32x4 v[3];    // bytes 16..63
};

DEV void fetch_prefix(const KParams& p, uint32_t chunk, int lane, uint32_t L, uint64_t o, Prefix& x) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  // only frames that can be fast are worth loading; the bytes may run past
  // L into the next frame or the tail pad (include/ixgrx.h IXG_TAIL_PAD)
  // decided per wave: a chunk with any longer frame is deferred anyway
  const bool ok = i < p.n && wave_all(L <= 64u || i >= p.n);
  const uint8_t* f = ok ? p.base + o : reinterpret_cast<const uint8_t*>(p.tab);
  x.w3 = *reinterpret_cast<const uint32_t*>(f + 12);
#pragma unroll
  for (int k = 0; k < 3; k++) x.v[k] = *reinterpret_cast<const u32x4_a4*>(f + 16 + 16 * k);
}

// a deferred chunk's class (ixgrx_internal.h): SHORT when no frame can need
// the streaming rounds
DEV uint32_t defer_class(bool valid, uint32_t L) {
  return wave_all(!valid || L < IXG_SHORT_MAX) ? IXG_CLS_SHORT : IXG_CLS_LONG;
}

// Publish the classes a wave deferred (bit k = class k): one store per wave
// and class, so the general kernels of an empty class exit at once.
DEV void publish_classes(const KParams& p, uint32_t seen, int lane) {
  if (lane == 0) {
    if (seen & (1u << IXG_CLS_SHORT)) p.present[IXG_CLS_SHORT] = p.epoch;
    if (seen & (1u << IXG_CLS_LONG)) p.present[IXG_CLS_LONG] = p.epoch;
  }
}

// the launch's IXG_MODE_* (FAST when the sampler did not run)
DEV uint32_t launch_mode(const KParams& p) {
  return (p.defer && p.present[0] == p.epoch) ? p.present[3] : IXG_MODE_FAST;
}

// The launch's IXG_MODE_* from the lengths of up to 64 evenly spread chunks,
// for a block of W waves (block-uniform; every thread returns it). Every
// length load is issued before the first vote: one round trip, not one per
// sample (the sampling is on every launch's critical path).
template <int W>
DEV uint32_t sample_mode(const KParams& p, uint32_t (*cnt)[3], uint32_t& big) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  const uint32_t ns = nchunks < 64u ? nchunks : 64u;
  constexpr int kPer = 64 / W;
  uint32_t L[kPer];
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const uint32_t k = (uint32_t)wave + (uint32_t)(W * j);
    const uint32_t c = ns ? k * nchunks / ns : 0u;  // k * nchunks < 64 * 2^26
    const uint32_t i = c * 64u + (uint32_t)lane;
    const bool ok = k < ns && i < p.n;
    const uint32_t v = p.len[ok ? i : 0u];
    L[j] = ok ? v : 0u;
  }
  uint32_t nf = 0, nsh = 0, nb = 0;
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    if ((uint32_t)wave + (uint32_t)(W * j) >= ns) break;
    nf += wave_all(L[j] <= 64u) ? 1u : 0u;
    nsh += wave_all(L[j] < IXG_SHORT_MAX) ? 1u : 0u;
    nb += wave_all(L[j] >= 256u || L[j] == 0u) ? 1u : 0u;  // (kBigMin)
  }
  if (lane == 0) {
    cnt[wave][0] = nf;
    cnt[wave][1] = nsh;
    cnt[wave][2] = nb;
  }
  __syncthreads();
  uint32_t f = 0, sh = 0, b = 0;
#pragma unroll
  for (int w = 0; w < W; w++) {
    f += cnt[w][0];
    sh += cnt[w][1];
    b += cnt[w][2];
  }
  uint32_t mode = 2 * f >= ns ? IXG_MODE_FAST : (2 * sh >= ns ? IXG_MODE_SHORT : IXG_MODE_LONG);
  if (p.force_mode != IXG_MODE_AUTO) mode = p.force_mode;
  big = 2 * b >= ns ? 1u : 0u;
  return mode;
}

// publish a launch's mode for the kernels after this one (launch_mode), and
// whether most sampled chunks are big (every frame >= 256 B: the long
// kernel then walks its chunks strided, launch_big)
DEV void publish_mode(const KParams& p, uint32_t mode, uint32_t big) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    p.present[3] = mode;
    p.present[6] = big;
    p.present[0] = p.epoch;
  }
}

DEV bool launch_big(const KParams& p) { return p.defer && p.present[0] == p.epoch && p.present[6] != 0u; }


// returns 1 << class for a deferred chunk, 0 when done here
DEV uint32_t fast_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane, uint32_t L,
                        const Prefix& x) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  uint32_t d[kPrefixDw];
  d[0] = d[1] = d[2] = 0;  // MAC addresses: never read on this path
  d[3] = x.w3 & ones((int)L - 12 < 0 ? 0 : (int)L - 12);
#pragma unroll
  for (int k = 1; k < 4; k++) {
    const u32x4& v = x.v[k - 1];
    d[4 * k + 0] = v.x & ones((int)L - (16 * k + 0) < 0 ? 0 : (int)L - (16 * k + 0));
    d[4 * k + 1] = v.y & ones((int)L - (16 * k + 4) < 0 ? 0 : (int)L - (16 * k + 4));
    d[4 * k + 2] = v.z & ones((int)L - (16 * k + 8) < 0 ? 0 : (int)L - (16 * k + 8));
    d[4 * k + 3] = v.w & ones((int)L - (16 * k + 12) < 0 ? 0 : (int)L - (16 * k + 12));
  }
#pragma unroll
  for (int j = 16; j < kPrefixDw; j++) d[j] = 0;
  const uint32_t etype = (byte_at(d, 12) << 8) | byte_at(d, 13);
  const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
  const bool fast = !valid || (L <= 64u && etype == 0x0800u && byte_at(d, 14) == 0x45u && ip_len >= 20 &&
                               14 + ip_len <= 64);
  const bool all_fast = wave_all(fast);
  const uint32_t cls = all_fast ? 0u : defer_class(valid, L);
  if (lane == 0) p.defer[chunk] = (uint8_t)cls;
  if (!all_fast) return 1u << cls;
  process_fast(p, T, i, valid, L, d);
  return 0;
}

}  // namespace

// AHEAD = how many chunks' prefixes a wave keeps in flight while it
// computes one (register double/triple buffering); descriptors run one
// stage further ahead because the prefix address depends on them.
template <bool OFFS, int AHEAD>
DEV void fast_loop(const KParams& p, const uint64_t* __restrict__ T) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  uint32_t c = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (c >= nchunks || launch_mode(p) != IXG_MODE_FAST) return;
  uint32_t Ld[AHEAD + 1];
  uint64_t od[AHEAD + 1];
  Prefix v[AHEAD];
  uint32_t seen = 0;
#pragma unroll
  for (int a = 0; a <= AHEAD; a++) fetch_desc<OFFS>(p, c + a * nw, lane, Ld[a], od[a]);
#pragma unroll
  for (int a = 0; a < AHEAD; a++) fetch_prefix(p, c + a * nw, lane, Ld[a], od[a], v[a]);
  for (;;) {
    // chunks past the end read clamped descriptors and no frame bytes
    uint32_t Ln;
    uint64_t on;
    fetch_desc<OFFS>(p, c + (AHEAD + 1) * nw, lane, Ln, on);
    Prefix vn;
    fetch_prefix(p, c + AHEAD * nw, lane, Ld[AHEAD], od[AHEAD], vn);
    seen |= fast_chunk(p, T, c, lane, Ld[0], v[0]);
    c += nw;
    if (c >= nchunks) break;
#pragma unroll
    for (int a = 0; a < AHEAD; a++) {
      Ld[a] = Ld[a + 1];
      od[a] = od[a + 1];
    }
    Ld[AHEAD] = Ln;
    od[AHEAD] = on;
#pragma unroll
    for (int a = 0; a + 1 < AHEAD; a++) v[a] = v[a + 1];
    v[AHEAD - 1] = vn;
  }
  publish_classes(p, seen, lane);
}

#define IXG_FAST_KERNEL(NAME, OFFS, AHEAD, WAVES)                                    \
  extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) \
  NAME(KParams p) {                                                                 \
    __shared__ uint64_t T[12 * 256];                                                \
    /* outside IXG_MODE_FAST the kernel has nothing to do: exit before staging  */ \
    /* the tables (24 KiB per block; the empty dispatch took 5.2 us with them)  */ \
    if (launch_mode(p) != IXG_MODE_FAST) return;                                    \
    stage_tables(p, T);                                                             \
    fast_loop<OFFS, AHEAD>(p, T);                                                   \
  }

// _s: fixed-stride layout, _o: u64 offsets
IXG_FAST_KERNEL(ixg_rx_fast_s, false, 1, 5)
IXG_FAST_KERNEL(ixg_rx_fast_o, true, 1, 5)

// ---- fixed-shape kernel, coalesced (fixed stride <= 64 B) ---------------
// A wave's 64 frames are one contiguous 64*stride-byte run. The wave loads
// the run's first 4 KiB (64*stride + the 64 bytes the last frame may need
// are within it) as aligned 16-byte lane loads, 4 per lane, writes them to
// its own 4 KiB of LDS and each lane reads its frame's bytes 12..63 back
// (stride/4 dwords apart: conflict-free for stride/4 odd, at most 2-way
// otherwise). The next chunk's loads are issued before the current chunk
// is transposed and parsed.
// The chunk base is wave-uniform (scalar); each lane adds its 32-bit
// offset, clamped to the last 16-byte piece that is readable. A clamped
// piece only ever replaces bytes no lane consumes: every byte a lane needs
// lies below (n-1)*stride + min(L_last, 64) <= lim - 64. A chunk past the
// end reads the zero page (IXG_ZERO_PAGE = 4096 covers the 4 KiB image).
// cc, nchunks and lim are wave-uniform (SGPRs)
// s_waitcnt immediates (gfx9 encoding: vmcnt [3:0] + [15:14], expcnt [6:4],
// lgkmcnt [11:8]; a field at its maximum does not wait)
constexpr uint32_t kGldsWait = 0x0F70;  // vmcnt(0)
constexpr uint32_t kLdsWait = 0xC07F;   // lgkmcnt(0)

DEV void fastc_issue(const KParams& p, uint32_t cc, uint32_t nchunks, uint64_t lim, int lane, u32x4 (&v)[4],
                     uint32_t& L) {
  const bool live = cc < nchunks;
  const uint64_t cbase = (uint64_t)cc * 64u * p.stride;
  // the chunk's own 64 * stride bytes only, and nothing past the batch's
  // readable end (pieces past either read 0: no traffic); a frame reaching
  // past its chunk (L > stride in lane 63) is not fixed-shape. A chunk past
  // the end reads nothing.
  // (p.overlap: frames run up to 64 bytes past their slot, lane 63's into
  // the next chunk; the 4 KiB image covers them, stride <= 64)
  const uint32_t cap = p.overlap ? (p.stride < 63u ? 64u * p.stride + 64u : 4096u) : 64u * p.stride;
  const uint64_t room = live ? lim - cbase : 0u;
  const __amdgpu_buffer_rsrc_t rs = rsrc(live ? p.base + cbase : p.zero, room < cap ? (uint32_t)room : cap);
#pragma unroll
  for (int k = 0; k < 4; k++)
    // frames are read once: non-temporal loads (with the nt record stores,
    // 7-8% on C2 over default-policy loads and stores)
    v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (lane + 64 * k), 0, kAuxNT);
  // lengths of the chunk's frames (0 past the batch's last)
  const uint32_t rem = live ? (p.n - cc * 64u < 64u ? p.n - cc * 64u : 64u) : 0u;
  const __amdgpu_buffer_rsrc_t rl = rsrc(live ? p.len + (uint64_t)cc * 64u : p.len, 2u * rem);
  L = __builtin_amdgcn_raw_buffer_load_b16(rl, 2 * lane, 0, 0);
}

// The fused demux of the coalesced kernel, one chunk behind: the chunk's
// bucket lines are loaded right after its records are stored and matched in
// the next iteration, after that chunk's frame loads are issued. (Matched at
// once, the wait for the line -- vmcnt is in order -- also waited for the
// next chunk's frames, loaded just before: the prefetch became synchronous.)
// The lines come 4 lanes per line (ixgwalk::lines_issue) and reach their
// lanes through the wave's LDS buffer when the lookups are matched.
struct PendDmx {
  u32x4 piece[4];  // ixgwalk::lines_issue's pieces
  uint32_t c;      // the chunk (wave-uniform); kNoDmx: nothing pending
  uint32_t key;    // ixgwalk::lookup_key
  uint32_t src, dst, ports;
};
constexpr uint32_t kNoDmx = 0xffffffffu;

DEV ixgwalk::Tables dmx_tables(const KParams& p) {
  return ixgwalk::Tables{p.active_start, p.bline, p.active, p.tw, p.listen, p.nfg + p.n_out, p.n_listen};
}

// record r of frame i of chunk c (valid lanes) -> pending lookup, the
// chunk's bucket lines loaded
DEV void dmx_issue(const KParams& p, bool valid, uint32_t c, const Rec& r, uint32_t src, uint32_t dst, uint32_t ports,
                   int lane, PendDmx& q) {
  const bool tcp = valid && ((r.w0 >> 16) & 0xffu) == IXG_V_TCP;
  const uint32_t ng = p.nfg + p.n_out;
  const uint32_t fg = ixg_demux_group(r.w0 & 0xffffu, p.fg_base, p.nfg, p.n_out);
  const bool look = tcp && fg < ng;
  const uint32_t bucket = r.w3 & (IXG_PCB_BUCKETS - 1u);
  q.c = c;
  q.key = ixgwalk::lookup_key(valid ? (tcp ? (look ? fg : ixgwalk::kGrpNone) : ixgwalk::kGrpNotTcp) : ixgwalk::kGrpNoFrame,
                              bucket, (r.w3 >> 16) & 0xffu);
  q.src = src;
  q.dst = dst;
  q.ports = ports;
  const uint32_t nlines = ng * IXG_PCB_BUCKETS;
  ixgwalk::lines_issue(p.bline, nlines, look ? fg * IXG_PCB_BUCKETS + bucket : nlines, lane, q.piece);
}

// the queue reads the tuples back from the frames (fixed stride, ihl 5)
DEV ixgwalk::Frames dmx_frames(const KParams& p) { return ixgwalk::Frames{p.base, p.stride}; }

// match the pending lookups (buf: the wave's 4 KiB of LDS, free); the
// ones the line cannot decide join the wave's queue sq
DEV void dmx_finish(const KParams& p, const PendDmx& q, int lane, lds_u32* buf, ixgwalk::SlowQ& sq) {
  if (q.c == kNoDmx) return;
  u32x4 ln[4];
  ixgwalk::lines_exchange(q.piece, lane, buf, ln);
  const uint32_t i = q.c * 64u + (uint32_t)lane;
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  if ((q.key & 0x3fffu) == ixgwalk::kGrpNotTcp) reinterpret_cast<u32x2v*>(p.dmx)[i] = u32x2v{0u, (uint32_t)IXG_D_NONE};
  ixgwalk::walk_line(dmx_tables(p), sq, i, q.key, q.src, q.dst, q.ports, ln[0], ln[1], ln[2], ln[3], lane, buf,
                     reinterpret_cast<uint32_t*>(p.dmx), dmx_frames(p));
}

// A chunk the coalesced kernel could not take as fixed-shape, finished by
// the same wave after its fixed-shape chunks (no second dispatch): per-lane
// prefix loads, the general parse, and a lane-serial sum of any segment
// tail past byte 96 (coalesced batches have strides <= 64 B, so such tails
// only come from frames reaching into the following slots: rare). The IPv6
// tables, when in use, are read from global memory (rare path: no LDS).
// The fused tcp_input head (ixg_rx_tcpx_batch_dev; dp/net/tcp_in.c:230-241):
// frame i's ixg_tcp_ext from its record and the five header dwords from 2
// bytes before the TCP header, stored non-temporal (zero for a record that is
// not IXG_V_TCP / IXG_V_TCP6), and with IXG_TCPX_INPLACE the in-place
// conversion. ext_fixed: a fixed-shape frame (IPv4 ihl 5: the dwords are the
// prefix's d[8..12], already in registers), stored through the chunk's
// buffer resource (lanes past the batch drop). ext_reload: any frame, the
// header loaded again (the coalesced kernel's rare non-fixed-shape chunks).
DEV void ext_fixed(const KParams& p, uint32_t c, uint32_t rem, int lane, bool valid, const Rec& r,
                   const uint32_t (&d)[kPrefixDw]) {
  const bool tcp = ((r.w0 >> 16) & 0xffu) == IXG_V_TCP;
  ixgx_ext e{0u, 0u, 0u, 0u};
  if (tcp) e = ixgx_make(d[8], d[9], d[10], d[11], d[12], r.w1, r.w3);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{e.x, e.y, e.z, e.w}, rsrc(p.ext + (uint64_t)c * 64u, 16u * rem),
                                         16 * lane, 0, kAuxNT);
  if (tcp && valid && (p.xflags & IXG_TCPX_INPLACE))
    ixgx_inplace(reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(p.base) + (uint64_t)(c * 64u + (uint32_t)lane) * p.stride + 32u),
                 d[8], d[11], d[12], e);
}
DEV void ext_reload(const KParams& p, uint32_t i, uint64_t off, const Rec& r, const uint32_t (&d)[kPrefixDw]) {
  const uint32_t v = (r.w0 >> 16) & 0xffu;
  ixgx_ext e{0u, 0u, 0u, 0u};
  if (v == IXG_V_TCP || v == IXG_V_TCP6) {
    const uint32_t l4 = v == IXG_V_TCP6 ? 54u : 14u + 4u * (byte_at(d, 14) & 15u);
    uint32_t* t = reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(p.base) + off + l4 - 2u);
    const uint32_t D0 = t[0], D1 = t[1], D2 = t[2], D3 = t[3], D4 = t[4];
    e = ixgx_make(D0, D1, D2, D3, D4, r.w1, r.w3);
    if (p.xflags & IXG_TCPX_INPLACE) ixgx_inplace(t, D0, D3, D4, e);
  }
  __builtin_nontemporal_store(u32x4{e.x, e.y, e.z, e.w}, reinterpret_cast<u32x4*>(p.ext + i));
}

template <bool DMX, bool TCPX = false>
DEV void slow_chunk(const KParams& p, const uint64_t* __restrict__ T, uint32_t chunk, int lane) {
  GDesc g;
  gen_desc<false>(p, chunk, lane, g);
  GPre x;
  gen_pre<false, false>(p, g, lane, x);
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;
  uint32_t d[kPrefixDw];
#pragma unroll
  for (int k = 0; k < kPrefixDw; k++) d[k] = x.d[k];
  LaneState s;
  lane_parse<kShapeAny, kPrefixDw>(p, Tab64{T}, d, L, s, p.tab6);
  if (!valid) return;
  uint32_t res = l4_residual(s);
  if (s.stream) res = (~fold16(add1c(fold32(s.l4_acc), span_sum(p, g.off, (uint32_t)kStreamBase, s.seg_end)))) & 0xffffu;
  const Rec r = make_record(p, d, L, s, res);
  store_record(p, i, r, s.ip_res, res);
  store_demux<DMX>(p, i, r, s.src, s.dst, s.ports);
  if (TCPX) ext_reload(p, i, g.off, r, d);
}

// TCPX: the fused tcp_input head (p.ext; not with DMX)
template <bool DMX, bool DRAIN = true, bool TCPX = false>
DEV void fastc_loop(const KParams& p, uint64_t* __restrict__ T, lds_u32* buf) {
  static_assert(!(DMX && TCPX), "one fused pass at a time");
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  // the wave's k-th chunk: runs of kRunC consecutive chunks dealt out
  // round-robin (kRunC = 1: grid-stride, the grid reads one window)
  const uint32_t w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  auto chunk_of = [&](uint32_t k) -> uint32_t {
    const uint64_t c64 = ((uint64_t)(k / kRunC) * nw + w0) * kRunC + k % kRunC;
    return c64 < nchunks ? (uint32_t)c64 : nchunks;
  };
  uint32_t c = chunk_of(0);
  constexpr int kTabV = 12 * 256 / 2 / kBlock;
  static_assert(kTabV * kBlock == 12 * 256 / 2, "table pieces per thread");
  uint64_t dmask = 0;  // bit k: the wave's k-th chunk was not fixed-shape
  uint32_t kth = 0;
  // readable bytes: up to IXG_TAIL_PAD past the last frame's end
  const uint64_t lim = (uint64_t)(p.n - 1) * p.stride + p.len[p.n - 1] + IXG_TAIL_PAD;
  const uint32_t fw = (uint32_t)lane * (p.stride >> 2);  // this lane's frame, in dwords
  u32x4 cur[4];
  uint32_t Lc, seen = 0;
  PendDmx pend;
  ixgwalk::SlowQ sq;
  if (DMX) {
    pend.c = kNoDmx;
    sq.n = 0;
  }
  // the block's hash tables (24 KiB) are staged into LDS with the first
  // chunk's frame loads already in flight: table loads, frame loads, then
  // the LDS writes and the barrier (each of the 8 blocks a CU slot runs per
  // launch paid the staging latency before its first frame load: 0.4 % on
  // C2, profiles/r04/fstage/). A wave with no chunk still joins the barrier.
  u32x4 tv[kTabV];
#pragma unroll
  for (int k = 0; k < kTabV; k++) tv[k] = reinterpret_cast<const u32x4*>(p.tab)[threadIdx.x + k * kBlock];
  fastc_issue(p, c, nchunks, lim, lane, cur, Lc);
#pragma unroll
  for (int k = 0; k < kTabV; k++) reinterpret_cast<u32x4*>(T)[threadIdx.x + k * kBlock] = tv[k];
  __syncthreads();
  if (c >= nchunks) return;
  for (;;) {
    const uint32_t cn = chunk_of(kth + 1);
    u32x4 nxt[4];
    uint32_t Ln;
    fastc_issue(p, cn, nchunks, lim, lane, nxt, Ln);
    if (DMX) dmx_finish(p, pend, lane, buf, sq);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      lds_u32* w = buf + 4 * (lane + 64 * k);
      w[0] = cur[k].x; w[1] = cur[k].y; w[2] = cur[k].z; w[3] = cur[k].w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t i = c * 64u + (uint32_t)lane;
    const bool valid = i < p.n;
    uint32_t d[kPrefixDw];
    d[0] = d[1] = d[2] = 0;  // MAC addresses: never read on this path
#pragma unroll
    for (int j = 3; j < 16; j++) d[j] = buf[fw + j];
#pragma unroll
    for (int j = 16; j < kPrefixDw; j++) d[j] = 0;
    // Bytes at offsets >= L read as zero. On this path nothing consumes a
    // byte >= L beyond offset 47 (the checksum regions end at or below L),
    // so frames with L >= 48 need no masking.
    if (!wave_all(!valid || Lc >= 48u)) {
#pragma unroll
      for (int j = 3; j < 16; j++) d[j] &= ones((int)Lc - 4 * j < 0 ? 0 : (int)Lc - 4 * j);
    }
    // fixed-shape: ethertype 0x0800 and version/ihl 0x45 (bytes 12..14 as
    // one masked dword), 20 <= ip_len <= 50 (14 + ip_len <= 64), L <= 64.
    // Non-short-circuit `&` / `|`: evaluated straight through, with no
    // exec-mask branches (a `&&` chain here compiled to nested branches)
    const uint32_t ip_len = bswap16(d[4] & 0xffffu);  // bytes 16..17
    const bool fast = !valid | ((Lc <= 64u) & ((d[3] & 0x00ffffffu) == 0x00450008u) & (ip_len - 20u <= 30u) &
                                ((lane != 63) | (Lc <= p.stride) | (p.overlap != 0u)));
    const bool all_fast = wave_all(fast);
    // chunks that are not fixed-shape are finished after the loop (DRAIN)
    // or flagged for the general kernels
    const uint32_t cls = all_fast ? 0u : defer_class(valid, Lc);
    if (!DRAIN || kth >= 64u) {
      if (lane == 0) p.defer[c] = (uint8_t)cls;
      seen |= (1u << cls) & ~1u;
    }
    if (DRAIN && kth < 64u && !all_fast) dmask |= 1ull << kth;
    kth++;
    // the lean path (lean_tcp) when every frame is a TCP segment tcp_input
    // accepts and all share one IP total length
    const uint32_t ipl = __builtin_amdgcn_readfirstlane(ip_len);
    const bool tcpok = ((d[5] & 0xff00ff3fu) == 0x06000000u) & (14u + ipl <= Lc) & (((d[11] >> 18) & 0x3cu) <= ipl - 20u);
    const bool lean = all_fast & (ipl >= 40u) & wave_all(!valid | ((ip_len == ipl) & tcpok));
    const uint32_t rem = p.n - c * 64u < 64u ? p.n - c * 64u : 64u;
    if (DMX) {
      // (a deferred chunk's records and demux records are the general kernel's)
      Rec r{0u, 0u, 0u, 0u};
      uint32_t src = 0, dst = 0, ports = 0;
      if (lean) {
        r = lean_tcp(p, T, i, lane, d, ipl, rsrc(p.out + (uint64_t)c * 64u, 16u * rem));
        lean_tuple(d, src, dst, ports);
      } else if (all_fast) {
        LaneState s;
        lane_parse<kShapeFixed, kFastDw>(p, Tab64{T}, d, Lc, s);
        const uint32_t r4 = l4_residual(s);
        r = make_record<true>(p, d, Lc, s, r4);
        if (valid) store_record<true>(p, i, r, s.ip_res, r4);
        src = s.src;
        dst = s.dst;
        ports = s.ports;
      }
      dmx_issue(p, all_fast && valid, c, r, src, dst, ports, lane, pend);
    } else if (TCPX) {
      if (lean) {
        const Rec r = lean_tcp(p, T, i, lane, d, ipl, rsrc(p.out + (uint64_t)c * 64u, 16u * rem));
        ext_fixed(p, c, rem, lane, valid, r, d);
      } else if (all_fast) {
        LaneState s;
        lane_parse<kShapeFixed, kFastDw>(p, Tab64{T}, d, Lc, s);
        const uint32_t r4 = l4_residual(s);
        const Rec r = make_record<true>(p, d, Lc, s, r4);
        if (valid) store_record<true>(p, i, r, s.ip_res, r4);
        ext_fixed(p, c, rem, lane, valid, r, d);
      }
    } else if (lean) {
      lean_tcp(p, T, i, lane, d, ipl, rsrc(p.out + (uint64_t)c * 64u, 16u * rem));
    } else if (all_fast) {
      process_fast(p, T, i, valid, Lc, d);
    }
    // the next iteration's LDS writes must not pass this one's reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    c = cn;
    if (c >= nchunks) break;
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    Lc = Ln;
  }
  if (DMX) {
    dmx_finish(p, pend, lane, buf, sq);
    ixgwalk::slowq_flush(dmx_tables(p), sq, lane, reinterpret_cast<uint32_t*>(p.dmx), dmx_frames(p));
  }
  publish_classes(p, seen, lane);
  if (DRAIN) {
    // the wave's own deferred chunks (its first 64: a wave has ~8; the rest,
    // if any, were flagged for the general kernels above)
    for (uint64_t m = dmask; m; m &= m - 1) slow_chunk<DMX, TCPX>(p, T, chunk_of((uint32_t)__builtin_ctzll(m)), lane);
  }
}

extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
ixg_rx_fastc_s(KParams p) {
  __shared__ uint64_t T[12 * 256];
  __shared__ uint32_t buf[kWaves][1024];
  fastc_loop<false>(p, T, LDS(lds_u32, buf[threadIdx.x >> 6]));
}

// with the fused PCB demux (p.dmx set: ixg_rx_demux_batch_dev); 3 waves per
// SIMD (168 VGPRs) rather than 4: the lookup's state one chunk behind gets
// registers, fused demux 0.2948 -> 0.2909 ms (profiles/r06/demux/ab_waves.json)
extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
ixg_rx_fastc_dmx_s(KParams p) {
  __shared__ uint64_t T[12 * 256];
  __shared__ uint32_t buf[kWaves][1024];
  fastc_loop<true>(p, T, LDS(lds_u32, buf[threadIdx.x >> 6]));
}

// with the fused tcp_input head (p.ext set: ixg_rx_tcpx_batch_dev)
extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
ixg_rx_fastc_tcpx_s(KParams p) {
  __shared__ uint64_t T[12 * 256];
  __shared__ uint32_t buf[kWaves][1024];
  fastc_loop<false, true, true>(p, T, LDS(lds_u32, buf[threadIdx.x >> 6]));
}


// ---- the flat long walk (C3: packed frames of every length) -----------------
// The long kernel's walk over chunks whose 64 frames lie in one span of at
// most kFlatRows KiB, in ascending order (packed batches: IMIX). Instead of a
// prefix pass per frame and tail rounds per segment (a chain of 3-4 round
// trips per chunk, with the wave's loads in flight only during the rounds),
// the wave streams the chunk's whole span [A, A + nb) as rows of 1 KiB (one
// fully coalesced 16-byte load per lane per row, all rows issued at once,
// raw buffer loads bounded to the span: rows past it read nothing). Every
// 16-byte piece's one's complement
// sum goes to LDS; a lane-blocked scan turns them into prefix sums P over
// the span (lane t's 32 pieces hold their sums from the lane's first piece,
// E[t] the sum of everything before that), and a frame's tail [96, seg_end)
// is P(E) - P(S) (one's complement subtraction: add the complement), each P
// completed inside its piece: S's from the prefix dwords in registers (frame
// starts are 4-aligned, so S = F + 96 is too), E's from the frame's end
// piece. The prefixes (bytes 0..95, transposed: wave instruction t fetches
// pieces 64t..64t+63 of the frame-major list) and the end pieces are copied
// into LDS with global_load_lds right behind the span's rows, so they hit
// the lines the rows bring into L2 and hold no registers: every frame byte is
// fetched from HBM once. tools/probe_c3.hip read C3's spans at 5.3-5.6 TB/s
// this way (one chunk per step, the next in flight) against 4.5 TB/s for the
// per-segment rounds.
// The rows (120 VGPRs) are live only while no parse state is: 256 VGPRs, two
// waves per SIMD, 8-wave blocks whose span buffers fill the CU's LDS.
// A chunk that is not flat (span over kFlatRows KiB, frames out of order)
// takes flat_fallback (per-lane prefixes and tails, 16 pieces in flight).
constexpr uint32_t kFlatRows = 30;                 // the largest span taken: 30 KiB (rows + parse in 256 VGPRs)
constexpr uint32_t kFlatPieces = 64u * kFlatRows;  // its 16-byte pieces
// S[] holds piece q at q + q / 32: the lane-blocked scan (lane t: pieces
// 32t .. 32t + 31) then reads and writes conflict-free; it covers 64 blocks
// of 32 pieces whatever the span (lanes past the span scan garbage, in bounds)
constexpr uint32_t kFlatS = 64u * 33u;
static_assert(kFlatPieces <= 64u * 32u, "the scan's 64 lane blocks cover the span");
DEV uint32_t sidx(uint32_t q) { return q + (q >> 5); }

struct FlatLds {
  lds_u32* S;      // [kFlatS] piece sums, then each lane block's inclusive sums
  lds_u32* E;      // [64] the sum before each lane block
  lds_u32* xch;    // [64 * 4] the chunk's frames {offset lo, hi, L, -} for the copies
  lds_u32* pre[2]; // [64 * kPrefixDw] prefixes, frame-major (DMA), per row set
  lds_u32* ve[2];  // [64 * 4] end pieces (DMA), per row set
};

struct FlatPlan {
  uint64_t A;   // span base (16-aligned, relative to p.base)
  uint32_t nb;  // span bytes, a multiple of 16; 0: not flat (or no chunk)
};

// Is chunk c flat (wave-uniform)? Frames ascending: lane 0's start is the
// span's base and the last frame's end its end, every frame inside.
DEV FlatPlan flat_plan(const KParams& p, uint32_t c, const GDesc& g, int lane) {
  FlatPlan f{0, 0};
  if (c == kNoChunk) return f;
  const uint32_t i = c * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t rest = p.n - c * 64u - 1u;
  const uint32_t last = rest < 63u ? rest : 63u;  // the chunk's last frame's lane (wave-uniform)
  const uint64_t A = rfl64(g.off) & ~15ull;
  const uint64_t end = g.off + g.L;
  const uint64_t e = rl64(end, last);
  const bool ok = !valid || g.L == 0u || (g.off >= A && end <= e);
  if (!wave_all(ok) || e < A || e - A > 16ull * kFlatPieces) return f;
  f.A = A;
  f.nb = (uint32_t)((e - A + 15u) & ~15ull);  // (the last piece: inside the batch's tail pad)
  return f;
}

// the span's rows, all issued (a chunk that is not flat reads nothing)
DEV void flat_rows(const KParams& p, const FlatPlan& f, int lane, u32x4 (&v)[kFlatRows]) {
  const __amdgpu_buffer_rsrc_t rs = rsrc(f.nb ? p.base + f.A : p.zero, f.nb);
#pragma unroll
  for (int r = 0; r < (int)kFlatRows; r++)
    // (one lane offset for all rows: the row's 4 KiB group in the scalar
    // offset, its 1 KiB within the group in the instruction's immediate)
    v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane + 1024 * (r & 3), 4096 * (r >> 2), 0);
}

// The prefixes (6 pieces per frame, pieces at or past L from the zero page)
// and the end pieces, HBM/L2 -> LDS (pre, ve); always 7 copies per lane
// (static vmcnt): a chunk that is not flat copies the zero page. The frames'
// offsets and lengths reach the lanes that copy their pieces through xch.
DEV void flat_dma(const KParams& p, const FlatPlan& f, const GDesc& g, int lane0, lds_u32* xch, lds_u32* pre,
                  lds_u32* ve) {
  // (the lane's per-copy frame and piece are recomputed per chunk, not held
  // across the walk in registers)
  uint32_t lane = (uint32_t)lane0;
  asm volatile("" : "+v"(lane));
  xch[4 * lane] = (uint32_t)g.off;
  xch[4 * lane + 1] = (uint32_t)(g.off >> 32);
  xch[4 * lane + 2] = g.L;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int t = 0; t < 6; t++) {
    const uint32_t q = 64u * (uint32_t)t + (uint32_t)lane, fr = q / 6u, j = q - 6u * fr;
    const u32x4 x = *(const lds_u32x4*)(xch + 4u * fr);
    const uint64_t fo = ((uint64_t)x.y << 32) | x.x;
    const uint8_t* src = f.nb && 16u * j < x.z ? p.base + fo + 16u * j : p.zero + 16 * lane;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(pre + 256u * t), 16,
                                     0, 0);
  }
  // (xch may be the end pieces' buffer: every lane has read it)
  __builtin_amdgcn_s_waitcnt(kLdsWait);
  __builtin_amdgcn_wave_barrier();
  // the piece holding the frame end F + L (span-relative), when the frame
  // can have a tail (L > 96) and its end is not piece-aligned
  const uint64_t e = g.off + g.L - f.A;
  const uint8_t* se = f.nb && g.L > (uint32_t)kStreamBase && (e & 15u) ? p.base + f.A + (e & ~15ull)
                                                                      : p.zero + 16 * lane;
  __builtin_amdgcn_global_load_lds((const void*)se, (__attribute__((address_space(3))) void*)ve, 16, 0, 0);
}

// one's complement (end-around carry) sum of a piece's four dwords
DEV uint32_t sum4(const u32x4& v) {
  Adc a(v.x, v.y);
  a.add(v.z);
  a.add(v.w);
  return a.end();
}

// inclusive one's complement scan across the wave (DPP: row shifts, then the
// row broadcasts; lanes with no source add 0)
template <int CTRL, int ROWS>
DEV uint32_t dpp_add1c(uint32_t t) {
  return add1c(t, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)t, CTRL, ROWS, 0xf, false));
}
DEV uint32_t wave_scan1c(uint32_t t) {
  t = dpp_add1c<0x111, 0xf>(t);  // row_shr:1
  t = dpp_add1c<0x112, 0xf>(t);  // row_shr:2
  t = dpp_add1c<0x114, 0xf>(t);  // row_shr:4
  t = dpp_add1c<0x118, 0xf>(t);  // row_shr:8
  t = dpp_add1c<0x142, 0xa>(t);  // row_bcast:15 (rows 1, 3)
  t = dpp_add1c<0x143, 0xc>(t);  // row_bcast:31 (rows 2, 3)
  return t;
}

// rows -> piece sums (S): the rows' registers are free after this
DEV void flat_sums(const FlatPlan& f, const u32x4 (&v)[kFlatRows], int lane, const FlatLds& fl) {
  // piece 64r + lane sits at 66r + lane + lane / 32 (sidx): one lane base,
  // the row in the instructions' immediate offsets
  lds_u32* s0 = fl.S + (uint32_t)lane + ((uint32_t)lane >> 5);
#pragma unroll
  for (int r = 0; r < (int)kFlatRows; r++)
    if (1024u * (uint32_t)r < f.nb) s0[66 * r] = sum4(v[r]);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// piece sums -> per lane block inclusive sums (S) and block bases (E)
DEV void flat_blocks(int lane, const FlatLds& fl) {
  // lane t: pieces 32t .. 32t + 31 (past the span: garbage, never read back)
  lds_u32* b = fl.S + 33u * (uint32_t)lane;
  uint32_t x[32];
#pragma unroll
  for (int k = 0; k < 32; k++) x[k] = b[k];
#pragma unroll
  for (int k = 1; k < 32; k++) x[k] = add1c(x[k - 1], x[k]);
#pragma unroll
  for (int k = 0; k < 32; k++) b[k] = x[k];
  // the sum before each block: exclusive scan of the blocks' totals
  const uint32_t incl = wave_scan1c(x[31]);
  fl.E[lane] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xf, 0xf, false);  // wave_shr:1
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// P at span position x (bytes [0, x) of the span): P of the pieces before
// x's piece plus `part`, the bytes of x's piece before x
DEV uint32_t flat_p(const FlatLds& fl, uint32_t x, uint32_t part) {
  const uint32_t q = x >> 4;
  const uint32_t pq = q ? add1c(fl.S[sidx(q - 1u)], fl.E[(q - 1u) >> 5]) : 0u;
  return add1c(pq, part);
}

// chunk c's records from its staged (masked) prefixes and the span's P;
// SHAPE: kShapeFixed for a wave of IPv4 ihl 5 frames, else kShapeAny
template <int SHAPE, bool DMX>
DEV void flat_finish(const KParams& p, const uint64_t* __restrict__ T, uint32_t c, int lane, const WaveLds& w,
                     const FlatLds& fl, const FlatPlan& f, const GDesc& g, const uint32_t (&d)[kPrefixDw],
                     const u32x4& ve) {
  const uint32_t i = c * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;
  LaneState s;
  lane_parse<SHAPE, kPrefixDw>(p, Tab64{T}, d, L, s, w.t6);
  uint32_t res = l4_residual(s);
  const bool strm = valid && s.stream;
  if (wave_any(strm)) {
    const uint32_t rf = (uint32_t)(g.off - f.A);  // the frame's start in the span (4-aligned)
    // S = F + 96: its piece's bytes before S are prefix dwords 24 - k .. 23
    const uint32_t ks = (rf & 15u) >> 2;
    const uint32_t ps = add1c(ks >= 3u ? d[21] : 0u, add1c(ks >= 2u ? d[22] : 0u, ks >= 1u ? d[23] : 0u));
    const uint32_t pS = flat_p(fl, rf + (uint32_t)kStreamBase, ps);
    // E = F + seg_end: its piece, masked (the end piece staged for E = F + L;
    // a segment ending short of the frame in another piece loads its own)
    const uint32_t re = rf + s.seg_end;
    u32x4 v = ve;
    const bool other = strm && (re & ~15u) != ((rf + L) & ~15u);
    if (wave_any(other) && other) v = load16(true, p.base + f.A + (re & ~15u), p.zero);
    const uint32_t pE = flat_p(fl, re, sum4(mask_piece(v, (int)(re & 15u))));
    uint32_t tail = add1c(pE, ~pS);
    // x - x is the negative zero 0xffffffff: exact for a non-zero tail sum,
    // but a tail of zero bytes sums to 0 (ICMP, with no pseudo header, can
    // tell the two apart): such lanes sum their tail exactly (rare)
    const bool amb = strm && tail == 0xffffffffu;
    if (wave_any(amb) && amb) tail = span_sum(p, g.off, (uint32_t)kStreamBase, s.seg_end);
    if (strm) res = (~fold16(add1c(fold32(s.l4_acc), tail))) & 0xffffu;
  }
  if (!valid) return;
  const Rec r = make_record(p, d, L, s, res);
  store_record(p, i, r, s.ip_res, res);
  store_demux<DMX>(p, i, r, s.src, s.dst, s.ports);
}

// A chunk the flat walk does not take (its span over kFlatRows KiB, or its
// frames out of order; rare in packed batches of IX frames): per-lane
// prefix loads, the general parse, and each tail [96, seg_end) summed by its
// own lane, 16 pieces in flight (slow_chunk's path with the loads batched;
// 16 against 8: C3 -1.1 %, profiles/r06/flat/ab_c3_tail16.json).
// Registers stay within the flat path's own (no streaming rounds).
DEV uint32_t tail_sum16(const KParams& p, uint64_t off, uint32_t a, uint32_t e) {
  uint32_t s = 0;
  for (uint32_t pos = a; wave_any(pos < e); pos += 256u) {
    u32x4 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = load16(pos + 16u * k < e, p.base + off + pos + 16u * k, p.zero);
#pragma unroll
    for (int k = 0; k < 16; k++) s = add1c(s, sum4(mask_piece(v[k], (int)e - (int)(pos + 16u * k))));
  }
  return s;
}
template <bool DMX>
DEV void flat_fallback(const KParams& p, const uint64_t* __restrict__ T, const WaveLds& w, uint32_t c, int lane,
                       const GDesc& g) {
  GPre x;
  gen_pre<false, false>(p, g, lane, x);
  const uint32_t i = c * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t L = g.L;
  uint32_t d[kPrefixDw];
#pragma unroll
  for (int k = 0; k < kPrefixDw; k++) d[k] = x.d[k];
  mask_prefix(d, L);
  LaneState s;
  lane_parse<kShapeAny, kPrefixDw>(p, Tab64{T}, d, L, s, w.t6);
  uint32_t res = l4_residual(s);
  const bool strm = valid && s.stream;
  if (wave_any(strm)) {
    const uint32_t t = tail_sum16(p, g.off, (uint32_t)kStreamBase, strm ? s.seg_end : 0u);
    if (strm) res = (~fold16(add1c(fold32(s.l4_acc), t))) & 0xffffu;
  }
  if (!valid) return;
  const Rec r = make_record(p, d, L, s, res);
  store_record(p, i, r, s.ip_res, res);
  store_demux<DMX>(p, i, r, s.src, s.dst, s.ports);
}

// The walk. Per chunk: its rows and staging copies, then its descriptors'
// successor, then (rows landed) the scan, the staged prefixes and the parse.
// The rows are in flight while no parse state is live, so a wave fits in
// 256 VGPRs and two waves share a SIMD: one parses while the other waits on
// its rows. (Pipelined one chunk deep instead -- chunk j+1's rows in flight
// during chunk j's parse -- the rows and the parse do not fit 256 VGPRs
// together: 30 rows spill two of them, C3 1.482 ms; 28 rows, spill-free,
// 1.403 ms; this walk 1.335 ms, same process, profiles/r06/flat/.)
template <bool OFFS, int SM, bool DMX>
DEV void flat_walk(const KParams& p, const uint64_t* __restrict__ T, const WaveLds& w, const FlatLds& fl,
                   const lds_u32* q, uint32_t nq, int lane0, GDesc D0) {
  for (uint32_t j = 0; j < nq; j++) {
    // the lane index laundered per chunk: everything derived from it
    // (addresses, masks) is recomputed here instead of being held in
    // registers across the walk, which the rows need
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const uint32_t c = q[j];
    const FlatPlan F = flat_plan(p, c, D0, lane);
    u32x4 R[kFlatRows];
    if (F.nb) {
      flat_rows(p, F, lane, R);
      flat_dma(p, F, D0, lane, fl.xch, fl.pre[0], fl.ve[0]);
    }
    GDesc D1;
    gen_desc<OFFS>(p, j + 1 < nq ? q[j + 1] : kNoChunk, lane, D1);
    if (F.nb) {
      flat_sums(F, R, lane, fl);
      flat_blocks(lane, fl);
      __builtin_amdgcn_s_waitcnt(kGldsWait);
      __builtin_amdgcn_wave_barrier();
      uint32_t d[kPrefixDw];
      const lds_u32* row = fl.pre[0] + (uint32_t)lane * kPrefixDw;
      d[0] = d[1] = d[2] = 0;  // MAC addresses: never read
      d[3] = row[3];
#pragma unroll
      for (int k = 1; k < 6; k++) {
        const u32x4 v = *(const lds_u32x4*)(row + 4 * k);
        d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
      }
      const u32x4 ve = *(const lds_u32x4*)(fl.ve[0] + 4u * (uint32_t)lane);
      // (no mask_prefix: the copies zero-fill the pieces at or past L and the
      // parse masks the two fields it can read past L; C3 -0.8 %, VALU per
      // chunk 1038 -> 873, profiles/r06/flat/ab_c3_nomask*.json)
      if (wave_all(c * 64u + (uint32_t)lane >= p.n || (eth_type(d, D0.L) == 0x0800u && byte_at(d, 14) == 0x45u)))
        flat_finish<kShapeFixed, DMX>(p, T, c, lane, w, fl, F, D0, d, ve);
      else
        flat_finish<kShapeAny, DMX>(p, T, c, lane, w, fl, F, D0, d, ve);
    } else {
      // not flat: each lane its own tail
      flat_fallback<DMX>(p, T, w, c, lane, D0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    D0 = D1;
  }
}

// ---- general kernel --------------------------------------------------------
// Every header shape the reference handles. Waves scan the defer flags 64
// chunks at a time and process the flagged chunks (all chunks when
// p.defer is null) one at a time.
// Walk a wave's chunk list with descriptors two chunks ahead; EARLY: the
// frame bytes one chunk ahead too, else loaded right before each chunk.
template <bool OFFS, bool EARLY, int MODE, int SM = 0, bool LATE_OK = false, bool BIG_OK = true, bool DMX = true>
DEV bool gen_walk(const KParams& p, const uint64_t* __restrict__ T, const WaveLds& w, const lds_u32* q,
                  uint32_t nq, int lane, GDesc D0) {
  constexpr bool GATE = MODE == kModeFirst;
  constexpr bool BIG = BIG_OK && MODE == kModeLong && !EARLY;
  bool deferred = false;
  uint32_t c0 = q[0], c1 = nq > 1 ? q[1] : kNoChunk;
  GDesc D1;
  gen_desc<OFFS>(p, c1, lane, D1);
  GPre P0;
  // the walk that waits for each prefix at once takes the transposed load
  constexpr bool TP = kPreT && MODE == kModeLong && !EARLY && !(LATE_OK && MODE == kModeLong);
  if (TP)
    gen_pre_t<BIG>(p, D0, lane, w, P0);
  else
    gen_pre<GATE, BIG>(p, D0, lane, P0);
  for (uint32_t j = 0; j < nq; j++) {
    const uint32_t c2 = j + 2 < nq ? q[j + 2] : kNoChunk;
    GDesc D2;
    gen_desc<OFFS>(p, c2, lane, D2);
    GPre P1;
    if (EARLY) gen_pre<GATE, BIG>(p, D1, lane, P1);
    constexpr bool LATE = LATE_OK && !EARLY && MODE == kModeLong;
    deferred |= general_chunk<OFFS, MODE, BIG, SM, LATE, DMX>(p, T, c0, lane, w, D0, P0, &D1, &P1);
    if (!EARLY && !LATE) {
      if (TP)
        gen_pre_t<BIG>(p, D1, lane, w, P1);
      else
        gen_pre<GATE, BIG>(p, D1, lane, P1);
    }
    c0 = c1;
    c1 = c2;
    D0 = D1;
    D1 = D2;
    P0 = P1;
  }
  return deferred;
}

// CLS: the class this kernel takes. IXG_CLS_SHORT: no streaming code at
// all, so fewer registers and more waves; it takes the chunks the
// fixed-shape kernel deferred as short or, in IXG_MODE_SHORT, walks every
// chunk and defers the long ones itself. IXG_CLS_LONG: everything; the
// deferred long chunks, or every chunk (p.defer null, or IXG_MODE_LONG).
// FLAT: chunk lists in long mode take flat_walk (8-wave blocks, no IPv6
// tables: its span buffers use the LDS they would need)
template <bool OFFS, uint32_t CLS, bool SEARLY = true, int SM = 0, bool LATE = false, bool BIGOK = true,
          int kWaves = 4, int kQGroups = 4, bool DMX = true, bool FLAT = false>
DEV void general_body(const KParams& p) {
  __shared__ uint64_t T[12 * 256];
  // (FLAT: the span sums; the per-segment path's lists live in them, and
  // the frames' exchange for the staging copies in the end pieces' buffer)
  constexpr int kFw = FLAT ? kWaves : 1;
  __shared__ uint32_t sh_S[kFw][FLAT ? kFlatS : 1], sh_E[kFw][FLAT ? 64 : 1], sh_ve[kFw][FLAT ? 256 : 1];
  constexpr int kLw = FLAT ? 1 : kWaves;
  __shared__ uint32_t sh_list[kLw][64], sh_end[kLw][64], sh_offlo[kLw][64], sh_offhi[kLw][64], sh_sum[kLw][64],
      sh_q[kWaves][64 * kQGroups];
  // the big-chunk prefix stash (not in the short kernel: no big chunks there)
  constexpr int kPre = CLS == IXG_CLS_SHORT ? 1 : 64 * kPrefixDw;
  __shared__ uint32_t sh_pre[kWaves][kPre];
  // (the wave index is wave-uniform: kept in an SGPR)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  const uint32_t ngroups = (nchunks + 63u) >> 6;
  // a block with no deferred chunk exits before staging the tables (the
  // common case behind the fixed-shape kernel: 64 B frames)
  const uint32_t mode = launch_mode(p);
  const bool all = CLS == IXG_CLS_SHORT ? mode == IXG_MODE_SHORT : (p.defer == nullptr || mode == IXG_MODE_LONG);
  // (p.present is only read when the flags are in use: it is null with
  // p.defer when the general kernel runs alone)
  if (!all) {
    const bool stamped = CLS == IXG_CLS_ANY
                             ? (p.present[IXG_CLS_SHORT] == p.epoch || p.present[IXG_CLS_LONG] == p.epoch)
                             : p.present[CLS] == p.epoch;
    if (!stamped) return;  // nothing of this class deferred
  }
  auto mine = [&](uint32_t ci) { return CLS == IXG_CLS_ANY ? p.defer[ci] != 0 : p.defer[ci] == CLS; };
  bool any = all;
  for (uint32_t g = blockIdx.x * kWaves + wave; !any && g < ngroups; g += nw) {
    const uint32_t ci = g * 64u + (uint32_t)lane;
    any = __ballot(ci < nchunks && mine(ci)) != 0;
  }
  if (!__syncthreads_or(any)) return;
  // IPv6 Toeplitz tables (24 KiB, dynamic LDS: present only with IXG_F_IPV6)
  extern __shared__ u32x4 dyn6[];
  if (p.tab6) {
    for (int k = threadIdx.x; k < (int)IXG_TAB6_WORDS / 4; k += 64 * kWaves) dyn6[k] = reinterpret_cast<const u32x4*>(p.tab6)[k];
  }
  stage_tables(p, T);
  lds_u32* lists = FLAT ? LDS(lds_u32, sh_S[FLAT ? wave : 0]) : nullptr;
  const WaveLds w = FLAT ? WaveLds{lists, lists + 64, lists + 128, lists + 192, lists + 256, LDS(const lds_u32, dyn6),
                                   LDS(lds_u32, sh_pre[wave])}
                         : WaveLds{LDS(lds_u32, sh_list[wave]), LDS(lds_u32, sh_end[wave]), LDS(lds_u32, sh_offlo[wave]),
                                   LDS(lds_u32, sh_offhi[wave]), LDS(lds_u32, sh_sum[wave]), LDS(const lds_u32, dyn6),
                                   LDS(lds_u32, sh_pre[wave])};
  lds_u32* q = LDS(lds_u32, sh_q[wave]);
  bool seen = false;
  // groups g0, g0+nw, ... of this wave, kQGroups at a time: their deferred
  // chunk ids go to an LDS list, which the pipeline then walks
  // Chunk order: wave w takes groups of 64 consecutive chunks (w, w + nw,
  // ...), or, when most sampled chunks are big (1500-B frames), chunks w,
  // w + nw, w + 2 nw, ... so the grid reads one window of the batch at a
  // time: C4 -3.8 %, C3 +7.8 % in same-process A/Bs of the two orders
  // (in general: the wave's j-th chunk is ((j / G) nw + w) G + j % G, runs
  // of G consecutive chunks dealt out round-robin; G = 64 or 1)
  const uint32_t wv0 = blockIdx.x * kWaves + wave;
  // (frames in host memory: one chunk per wave, latency-bound; the grid has
  // one wave per chunk, ixgrx_launch)
  const uint64_t G = p.host_mem || (CLS == IXG_CLS_LONG && launch_big(p)) ? kRunBig : kRun;
  for (uint32_t it = 0; ((uint64_t)64u * kQGroups * it / G * nw + wv0) * G < nchunks; it++) {
    uint32_t nq = 0;
#pragma unroll
    for (int k = 0; k < kQGroups; k++) {
      const uint64_t j = (uint32_t)lane + 64ull * (it * kQGroups + (uint32_t)k);
      const uint64_t c64 = (j / G * nw + wv0) * G + j % G;
      const uint32_t ci = c64 < nchunks ? (uint32_t)c64 : 0u;
      const bool want = c64 < nchunks && (all || mine(ci));
      const uint64_t m = __ballot(want);
      if (want) q[nq + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = ci;
      nq += (uint32_t)__popcll(m);
    }
    __builtin_amdgcn_wave_barrier();
    if (nq == 0) continue;
    // Prefix prefetch one chunk ahead pays when chunks are parse-bound
    // (short frames); when they stream, loading the next prefix during the
    // rounds costs more than it hides. Decided once per list from its first
    // chunk, as two separate loops, so no load in either is conditional.
    GDesc D0;
    gen_desc<OFFS>(p, q[0], lane, D0);
    if (CLS == IXG_CLS_SHORT)
      seen |= gen_walk<OFFS, SEARLY, kModeFirst, 0, false, true, DMX>(p, T, w, q, nq, lane, D0);
    else if (FLAT && !launch_big(p))
      flat_walk<OFFS, SM, DMX>(p, T, w,
                               FlatLds{LDS(lds_u32, sh_S[FLAT ? wave : 0]), LDS(lds_u32, sh_E[FLAT ? wave : 0]),
                                       LDS(lds_u32, sh_ve[FLAT ? wave : 0]),
                                       {LDS(lds_u32, sh_pre[wave]), LDS(lds_u32, sh_pre[wave])},
                                       {LDS(lds_u32, sh_ve[FLAT ? wave : 0]), LDS(lds_u32, sh_ve[FLAT ? wave : 0])}},
                               q, nq, lane, D0);
    else if (!SEARLY || wave_any(D0.L > (uint32_t)kStreamBase + 32u))
      gen_walk<OFFS, false, kModeLong, SM, LATE, BIGOK, DMX>(p, T, w, q, nq, lane, D0);
    else
      gen_walk<OFFS, true, kModeLong, SM, false, true, DMX>(p, T, w, q, nq, lane, D0);
    __builtin_amdgcn_wave_barrier();
  }
  if (CLS == IXG_CLS_SHORT) publish_classes(p, seen ? 1u << IXG_CLS_LONG : 0u, lane);
}

#define IXG_GEN_KERNEL(NAME, OFFS, CLS, WAVES, ...)                                                 \
  extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) \
  NAME(KParams p) { general_body<OFFS, CLS, ##__VA_ARGS__>(p); }
// Blocks of BW waves sharing one LDS copy of the hash tables (24 KiB, + the
// IPv6 tables' 24 KiB under IXG_F_IPV6): two 10-wave blocks per CU give 5
// waves per SIMD within LDS (2 x 58 KiB), 8-wave blocks 4.
#define IXG_GENW_KERNEL(NAME, BW, OFFS, CLS, WAVES, ...)                                              \
  extern "C" __global__ void __launch_bounds__(64 * BW) __attribute__((amdgpu_waves_per_eu(WAVES)))  \
  NAME(KParams p) { general_body<OFFS, CLS, ##__VA_ARGS__>(p); }
// (the default streams medium segments with 4-lane groups: C3 -5.5% in
// A/B, and C3's FETCH_SIZE 6.64 -> 6.53 GB)
IXG_GEN_KERNEL(ixg_rx_general_s, false, IXG_CLS_LONG, 2, true, 1)
IXG_GEN_KERNEL(ixg_rx_general_o, true, IXG_CLS_LONG, 2, true, 1)
// the long kernel with the flat walk (8-wave blocks sharing one table copy:
// the 8 waves' span buffers fill the CU's LDS); not under IXG_F_IPV6
IXG_GENW_KERNEL(ixg_rx_glong_s, 8, false, IXG_CLS_LONG, 2, false, 1, false, true, 8, 1, true, true)
IXG_GENW_KERNEL(ixg_rx_glong_o, 8, true, IXG_CLS_LONG, 2, false, 1, false, true, 8, 1, true, true)
// the short-class general kernel (no streaming rounds): 4 waves/SIMD
// without the one-ahead prefix prefetch (128 VGPRs; C5 -3% against the
// 3-wave prefetching build)
// without the fused demux code and with it (4 waves/SIMD, 8-wave blocks;
// the build without it at 5 waves/SIMD and 96 VGPRs, A/B variant w10, ran
// C5 20% slower)
IXG_GENW_KERNEL(ixg_rx_short_w8_s, 8, false, IXG_CLS_SHORT, 4, false, 0, false, true, 8, 4, false)
IXG_GENW_KERNEL(ixg_rx_short_w8_o, 8, true, IXG_CLS_SHORT, 4, false, 0, false, true, 8, 4, false)
IXG_GENW_KERNEL(ixg_rx_short_w8d_s, 8, false, IXG_CLS_SHORT, 4, false, 0, false, true, 8)
IXG_GENW_KERNEL(ixg_rx_short_w8d_o, 8, true, IXG_CLS_SHORT, 4, false, 0, false, true, 8)

// ---- the span-staged short kernel ------------------------------------------
// Short chunks (every frame < IXG_SHORT_MAX bytes) whose frames lie in one
// contiguous span of at most kSpanMax bytes (packed batches: the frames of a
// chunk back to back; fixed strides <= 96 B) are staged through LDS: the
// wave copies the span HBM -> LDS with global_load_lds_dwordx4 (1 KiB per
// wave instruction, fully coalesced, no VGPRs), then each lane reads its own
// frame's bytes 12..111 from LDS. Per-lane 16-byte loads of the prefixes
// (the other kernels) touch 64 cache lines per instruction; measured on C5
// the L1 spent most cycles stalled on their pending misses (TD busy 85 %,
// TA stalled by TC). The copy of the wave's next chunk is issued as soon as
// the current one has been read out of LDS, so it overlaps the parse.
// Chunks that are not span-contiguous take per-lane loads.
constexpr uint32_t kSpanMax = 6144;             // bytes per wave's span buffer
constexpr int kSpanWaves = 16;                  // 1024-thread blocks, 1 per CU


// A chunk's span: LDS image of [base, base + 1024 * npc) (npc = 0: not
// span-contiguous, load per lane)
struct Span {
  uint64_t base;
  uint32_t npc;
};

// Decide and issue the span copy of a chunk (descriptors g, wave-uniform
// result). Every lane needs bytes [off, off + min(L, 112)).
template <bool OFFS, int AUX = 0>
DEV Span span_issue(const KParams& p, const GDesc& g, int lane, bool live, lds_u32* buf) {
  Span sp{0, 0};
  if (!live) return sp;
  const uint32_t need = g.L < IXG_SHORT_MAX ? g.L : IXG_SHORT_MAX;
  const uint64_t base = rfl64(g.off);
  const uint64_t b16 = base & ~15ull;
  const uint64_t end = g.off + need;
  // the last lane's end bounds the span when the offsets ascend (packed)
  const uint64_t e63 = rl64(end, 63);
  const bool ok = g.L == 0u || (g.off >= base && end <= e63 && e63 - b16 <= kSpanMax);
  if (!wave_all(ok)) return sp;
  sp.base = b16;
  sp.npc = (uint32_t)((e63 - b16 + 1023u) >> 10);
  const uint64_t top = e63 - b16;  // bytes of the span that exist (the rest: zero page)
  for (uint32_t k = 0; k < sp.npc; k++) {
    const uint32_t o = 1024u * k + 16u * (uint32_t)lane;
    const uint8_t* src = o < top ? p.base + b16 + o : p.zero + 16 * lane;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + 256u * k),
                                     16, 0, AUX);
  }
  return sp;
}

// The lane parse specialised for the wave's header family (wave-uniform):
// all IPv4 ihl 5 -> the constant geometry; no IPv6 lane -> no IPv6 code;
// every lane IPv6 (IXG_F_IPV6) -> L4 at the constant 54, no IPv4 mux.
template <class Tab>
DEV void parse_dispatch(const KParams& p, const Tab& tab, const uint32_t (&d)[kPrefixDw], uint32_t L, bool valid,
                        LaneState& st, const lds_u32* t6) {
  const uint32_t et = eth_type(d, L);
  const bool six = (p.flags & IXG_F_IPV6) && et == 0x86DDu;
  if (wave_all(!valid || (et == 0x0800u && byte_at(d, 14) == 0x45u)))
    lane_parse<kShapeFixed, kPrefixDw>(p, tab, d, L, st);
  else if (wave_all(!valid || !six))
    lane_parse<kShapeV4, kPrefixDw>(p, tab, d, L, st, t6);
  else if (wave_all(!valid || six))
    lane_parse<kShapeV6, kPrefixDw>(p, tab, d, L, st, t6);
  else
    lane_parse<kShapeAny, kPrefixDw>(p, tab, d, L, st, t6);
}

// AUX: the copies' cache policy (2 = nt)
template <bool OFFS, bool DMX, int AUX = 0, bool STRIDED = true>
DEV void short_span_body(const KParams& p) {
  constexpr int W = kSpanWaves;
  __shared__ uint64_t T[12 * 256];
  // (+32 dwords: a lane reads up to 112 bytes from its frame start; the
  // bytes past its frame are masked, but stay inside the buffer)
  __shared__ uint32_t sh_span[W][kSpanMax / 4 + 32];
  __shared__ uint32_t sh_q[W][64];
  extern __shared__ u32x4 dyn6[];  // IPv6 Toeplitz tables (IXG_F_IPV6)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * W;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  const uint32_t ngroups = (nchunks + 63u) >> 6;
  // p.self_sample (the default plan for offset and wide-stride batches):
  // no sampler or fixed-shape kernel ran before this one; every block
  // samples the launch's mode itself (the same lengths: L2 hits after the
  // first blocks), block 0 publishes it for the long kernel, and FAST counts
  // as SHORT (this kernel takes fixed-shape chunks at the fixed-shape
  // kernel's speed: C2's frames in the offset layout within 1.2 %). Two
  // dispatches fewer per launch: ~10 us (C5 -2 %).
  __shared__ uint32_t cnt[W][3];
  uint32_t mode;
  if (p.self_sample) {
    uint32_t big;
    mode = sample_mode<W>(p, cnt, big);
    if (mode == IXG_MODE_FAST) mode = IXG_MODE_SHORT;
    publish_mode(p, mode, big);
  } else {
    mode = launch_mode(p);
  }
  const bool all = mode == IXG_MODE_SHORT;
  if (!all && (mode == IXG_MODE_LONG || p.present[IXG_CLS_SHORT] != p.epoch)) return;  // nothing deferred short
  auto mine = [&](uint32_t ci) { return p.defer[ci] == IXG_CLS_SHORT; };
  // STRIDED: the wave's j-th chunk is ((j / kRunS) nw + wv) kRunS + j % kRunS
  // (runs of kRunS consecutive chunks dealt out round-robin)
  const uint32_t wv = blockIdx.x * W + wave;
  auto sch = [&](uint32_t j) -> uint64_t { return ((uint64_t)(j / kRunS) * nw + wv) * kRunS + j % kRunS; };
  bool any = all;
  for (uint32_t g = STRIDED ? 0u : wv; !any && (STRIDED ? sch(64u * g) < nchunks : g < ngroups);
       g += STRIDED ? 1u : nw) {
    const uint64_t c64 = STRIDED ? sch(64u * g + (uint32_t)lane) : (uint64_t)g * 64u + (uint32_t)lane;
    const uint32_t ci = c64 < nchunks ? (uint32_t)c64 : 0u;
    any = wave_any(c64 < nchunks && mine(ci));
  }
  if (!__syncthreads_or(any)) return;
  if (p.tab6) {
    for (int k = threadIdx.x; k < (int)IXG_TAB6_WORDS / 4; k += 64 * W)
      dyn6[k] = reinterpret_cast<const u32x4*>(p.tab6)[k];
  }
  stage_tables(p, T);
  const Tab64 tab{T};
  const lds_u32* t6 = LDS(const lds_u32, dyn6);
  lds_u32* buf = LDS(lds_u32, sh_span[wave]);
  lds_u32* q = LDS(lds_u32, sh_q[wave]);
  bool seen = false;
  // chunk assignment (STRIDED): wave wv takes chunks wv, wv + nw, wv + 2 nw, ...,
  // so at any moment the grid reads one contiguous window of the batch (a
  // wave per chunk) rather than one region per wave; else wave g takes the
  // 64 consecutive chunks of group g
  for (uint32_t g0 = STRIDED ? 0u : wv; STRIDED ? sch(64u * g0) < nchunks : g0 < ngroups;
       g0 += STRIDED ? 1u : nw) {
    const uint64_t c64 = STRIDED ? sch(64u * g0 + (uint32_t)lane) : (uint64_t)g0 * 64u + (uint32_t)lane;
    const uint32_t ci = c64 < nchunks ? (uint32_t)c64 : 0u;
    const bool want = c64 < nchunks && (all || mine(ci));
    const uint64_t m = __ballot(want);
    if (want) q[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = ci;
    const uint32_t nq = (uint32_t)__popcll(m);
    __builtin_amdgcn_wave_barrier();
    if (nq == 0) continue;
    // a chunk is live unless it holds a frame of IXG_SHORT_MAX bytes or more
    // (then it is flagged for the long kernel here)
    auto classify = [&](uint32_t chunk, GDesc& g) {
      const bool defer = !wave_all(g.L < IXG_SHORT_MAX);  // (L = 0 past the batch end)
      if (lane == 0) p.defer[chunk] = defer ? (uint8_t)IXG_CLS_LONG : (uint8_t)0;
      seen |= defer;
      if (defer) g.L = 0;
      return !defer;
    };
    uint32_t c0 = q[0];
    GDesc D0, D1;
    gen_desc<OFFS>(p, c0, lane, D0);
    bool live0 = classify(c0, D0);
    Span S0 = span_issue<OFFS, AUX>(p, D0, lane, live0, buf);
    uint32_t c1 = nq > 1 ? q[1] : kNoChunk;
    gen_desc<OFFS>(p, c1, lane, D1);
    for (uint32_t j = 0; j < nq; j++) {
      const uint32_t i = c0 * 64u + (uint32_t)lane;
      const bool valid = live0 && i < p.n;
      const uint32_t L = D0.L;
      uint32_t d[kPrefixDw];
      u32x4 v96 = {0u, 0u, 0u, 0u};
      if (S0.npc) {
        __builtin_amdgcn_s_waitcnt(kGldsWait);
        __builtin_amdgcn_wave_barrier();
        const uint32_t w0 = (uint32_t)(D0.off - S0.base) >> 2;
        const lds_u32* f = buf + (L ? w0 : 0u);
        d[0] = d[1] = d[2] = 0;
#pragma unroll
        for (int k = 3; k < kPrefixDw; k++) d[k] = f[k];
        if (wave_any(L > (uint32_t)kStreamBase)) v96 = u32x4{f[24], f[25], f[26], f[27]};
      } else {
        GPre x;
        gen_pre<false, false>(p, D0, lane, x);
#pragma unroll
        for (int k = 0; k < kPrefixDw; k++) d[k] = x.d[k];
        v96 = x.v96;
      }
      // (every lane has its bytes: the next chunk's copy may overwrite the buffer)
      __builtin_amdgcn_s_waitcnt(kLdsWait);
      __builtin_amdgcn_wave_barrier();
      const uint32_t c2 = j + 2 < nq ? q[j + 2] : kNoChunk;
      bool live1 = false;
      Span S1{0, 0};
      if (j + 1 < nq) {
        live1 = classify(c1, D1);
        S1 = span_issue<OFFS, AUX>(p, D1, lane, live1, buf);
      }
      GDesc D2;
      gen_desc<OFFS>(p, c2, lane, D2);
      // ---- parse chunk c0 ----
      if (live0) {
        LaneState st;
        parse_dispatch(p, tab, d, L, valid, st, t6);
        // the 16-byte piece holding a segment end past byte 96 (frames < 112 B)
        if (valid && st.stream) st.l4_acc += piece_sum(v96, (int)(st.seg_end - (uint32_t)kStreamBase));
        if (valid) {
          const uint32_t r4 = l4_residual(st);
          const Rec r = make_record(p, d, L, st, r4);
          // non-temporal record stores: C5 0.4307 -> 0.4007 ms, c5r 0.3972
          // -> 0.3634 ms in one process (profiles/r05/rec_nt/; the same in
          // the long kernels: C3 1.474 -> 1.526 ms, C4 unchanged, not taken)
          store_record<true>(p, i, r, st.ip_res, r4);
          store_demux<DMX>(p, i, r, st.src, st.dst, st.ports);
        }
      }
      c0 = c1;
      c1 = c2;
      D0 = D1;
      D1 = D2;
      live0 = live1;
      S0 = S1;
    }
    __builtin_amdgcn_wave_barrier();
  }
  publish_classes(p, seen ? 1u << IXG_CLS_LONG : 0u, lane);
}

#define IXG_SPAN_KERNEL(NAME, OFFS, DMX, ...)                                                                  \
  extern "C" __global__ void __launch_bounds__(64 * kSpanWaves) __attribute__((amdgpu_waves_per_eu(4))) \
  NAME(KParams p) { short_span_body<OFFS, DMX, ##__VA_ARGS__>(p); }
// span copies non-temporal (AUX 2: each span is read once, out of LDS):
// C5 0.4343 -> 0.4275 ms, c5r 0.4138 -> 0.3960, C3 unchanged in a
// same-process A/B (profiles/r04/span_nt/)
IXG_SPAN_KERNEL(ixg_rx_short_sp_s, false, false, 2)
IXG_SPAN_KERNEL(ixg_rx_short_sp_o, true, false, 2)


// The sampler: one block picks the launch's IXG_MODE_*: FAST when at least
// half of the sampled chunks could be fixed-shape by length (every frame <=
// 64 B), else SHORT when at least half are short, else LONG.
extern "C" __global__ void __launch_bounds__(kBlock) ixg_rx_sample(KParams p) {
  __shared__ uint32_t cnt[kWaves][3];
  uint32_t big;
  const uint32_t mode = sample_mode<kWaves>(p, cnt, big);
  publish_mode(p, mode, big);
}

typedef void (*kern_fn)(KParams);
// [layout: 0 = stride, 1 = offsets]
static const kern_fn k_fast[2] = {ixg_rx_fast_s, ixg_rx_fast_o};
static const kern_fn k_gen[2] = {ixg_rx_general_s, ixg_rx_general_o};
// the short kernel and its block size: the span-staged kernel, or with the
// fused demux (p.dmx) the general short kernel in 512-thread blocks
struct ShortK {
  kern_fn k[2];
  int block;
};
static const ShortK k_short_dmx = {{ixg_rx_short_w8d_s, ixg_rx_short_w8d_o}, 512};
static const ShortK k_short = {{ixg_rx_short_sp_s, ixg_rx_short_sp_o}, 64 * kSpanWaves};

// blocks per CU, cached per (kernel, dynamic LDS): a handful of entries,
// filled under a lock (contexts on several host threads launch concurrently)
static int occupancy(kern_fn k, size_t shmem, int block) {
  struct Entry { kern_fn k; size_t shmem; int nb; };
  static std::mutex mu;
  static Entry cache[32];
  static int used = 0;
  std::lock_guard<std::mutex> lock(mu);
  for (int i = 0; i < used; i++)
    if (cache[i].k == k && cache[i].shmem == shmem) return cache[i].nb;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, block, shmem) != hipSuccess || nb < 1) nb = 1;
  if (used < 32) cache[used++] = Entry{k, shmem, nb};
  return nb;
}

static uint32_t grid_for(kern_fn k, uint64_t want, uint32_t ncu, size_t shmem = 0, int block = kBlock) {
  const uint64_t cap = (uint64_t)ncu * (uint64_t)occupancy(k, shmem, block);
  const uint64_t g = want < cap ? want : cap;
  return g ? (uint32_t)g : 1u;
}

// The asynchronous host path's completion stamp (ixgrx_async.c): after
// everything enqueued before it on the stream, one lane stores v to a word of
// coherent pinned host memory with a system-scope release, so the host sees
// a finished batch by reading that word (no runtime call, no runtime lock).
// Ordering assumption: the batch's kernels (the RX kernels
// writing records to pinned memory in DIRECT mode, the echo reflect writing
// records and mbufs) and its D2H copy run before the stamp on the same
// stream, and what they wrote is host-visible by the time the stamp is,
// through the release fences the runtime puts on their dispatch packets and
// copies plus this store's own system-scope release (which writes back only
// the L2 of the XCD it runs on). HIP does not document those fence scopes;
// what pins the assumption is the tests that read every record and every
// reflected mbuf byte of multi-batch runs after polling the word, in DIRECT
// and copy modes (tests/test_async.py, tests/test_icmp.py async tests,
// tests/test_integration_example.py).
// The word is the first of four: f[2..3] get the device's wall clock
// (wall_clock64, constant rate) when the stamp runs, stored before the
// release, so the host can tell how late it saw a finished batch
// (ixg_rx_async_stats' worst-batch split).
extern "C" __global__ void __launch_bounds__(64) ixg_done_stamp(uint32_t* f, uint32_t v) {
  if (threadIdx.x == 0) {
    const uint64_t t = wall_clock64();
    f[2] = (uint32_t)t;
    f[3] = (uint32_t)(t >> 32);
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

extern "C" int ixgrx_stamp(uint32_t* flag, uint32_t v, void* stream) {
  hipLaunchKernelGGL(ixg_done_stamp, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, v);
  return (int)hipGetLastError();
}

// The launch plan: coalesced fixed strides <= 64 B
// (16-B aligned base) take the coalesced fixed-shape kernel alone; other
// layouts the span-staged short kernel, which samples the mode itself, then
// the general kernel for what it deferred. Forced splits (ixg_rx_set_split,
// tests) and the fused demux run the sampler and the lane-load fixed-shape
// kernel first.
extern "C" int ixgrx_launch(const void* params, uint32_t ncu, void* stream) {
  const KParams& p = *static_cast<const KParams*>(params);
  const int lay = p.off ? 1 : 0;
  const uint64_t nchunks = ((uint64_t)p.n + 63u) / 64u;
  if (p.long_only && p.host_mem) {
    // host-memory batch of long frames: kHostFpw frames per wave
    static const kern_fn k_hb[2] = {ixg_rx_host_big_s, ixg_rx_host_big_o};
    const uint64_t nsub = ((uint64_t)p.n + kHostFpw - 1u) / kHostFpw;
    const size_t sh6 = p.tab6 ? IXG_TAB6_WORDS * sizeof(uint32_t) : 0u;
    hipLaunchKernelGGL(k_hb[lay], dim3(grid_for(k_hb[lay], (nsub + kWaves - 1) / kWaves, ncu, sh6)), dim3(kBlock), sh6,
                       (hipStream_t)stream, p);
    return (int)hipGetLastError();
  }
  const uint64_t wave_blocks = (nchunks + kWaves - 1) / kWaves;              // one wave per chunk
  const uint64_t group_blocks = ((nchunks + 63u) / 64u + kWaves - 1) / kWaves; // one wave per 64 chunks
  const bool coal = !p.off && p.stride <= 64u && (p.stride & 3u) == 0u &&
                      (reinterpret_cast<uintptr_t>(p.base) & 15u) == 0u;
  const size_t sh6 = p.tab6 ? IXG_TAB6_WORDS * sizeof(uint32_t) : 0u;
  if (p.ext && !ixgrx_tcpx_fusable(params)) return (int)hipErrorInvalidValue;  // (the host checks first)
  // offset and wide-stride batches in the default split: the span-staged
  // short kernel runs first and samples the mode itself (no sampler, no
  // fixed-shape kernel dispatch); forced splits and the fused demux keep the
  // sampler + fixed-shape kernel plan
  const bool self = p.defer && !coal && !p.dmx && p.force_mode == IXG_MODE_AUTO;
  if (p.defer && !self) {
    kern_fn kf = nullptr;
    const bool forced = p.force_mode != IXG_MODE_AUTO;
    if (coal) {
      // coalesced fixed stride: always fixed-shape first (no sampler),
      // unless a test forces another split
      if (forced) hipLaunchKernelGGL(ixg_rx_sample, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, p);
      if (!forced || p.force_mode == IXG_MODE_FAST) kf = p.dmx ? ixg_rx_fastc_dmx_s : p.ext ? ixg_rx_fastc_tcpx_s : ixg_rx_fastc_s;
    } else {
      hipLaunchKernelGGL(ixg_rx_sample, dim3(1), dim3(kBlock), 0, (hipStream_t)stream, p);
      kf = k_fast[lay];
    }
    // the coalesced kernel runs 16 resident-grids' worth of blocks (each
    // wave ~4 chunks, two runs of kRunC): with the table staging overlapped
    // with the first chunk's loads, C2 0.2135 -> 0.2005 ms against 8 grids
    // (round 4 same-process A/B of 6x .. 64x: 6x 0.2176, 12x 0.2076, 24x
    // 0.2018, 32x 0.2051, 48x 0.2213, 64x 0.240 ms; the fused demux 0.3057
    // -> 0.3011 ms; profiles/r04/grid/); at least one block per 64 chunks
    // per wave, so every wave can finish its own deferred chunks
    // (fastc_loop's DRAIN)
    const bool fc = kf == ixg_rx_fastc_s || kf == ixg_rx_fastc_dmx_s || kf == ixg_rx_fastc_tcpx_s;
    const uint32_t gcu = fc ? 16u * ncu : ncu;
    if (kf) {
      uint64_t gb = grid_for(kf, wave_blocks, gcu);
      // (a wave takes runs of kRunC chunks: at most 64 / kRunC runs each)
      const uint64_t runs = (nchunks + kRunC - 1) / kRunC, per = 64u / kRunC;
      const uint64_t gmin = ((runs + per - 1) / per + kWaves - 1) / kWaves;
      if (fc && gb < gmin) gb = gmin;
      hipLaunchKernelGGL(kf, dim3((uint32_t)gb), dim3(kBlock), 0, (hipStream_t)stream, p);
    }
  }
  // coalesced batches in the default split: the coalesced kernel finished
  // every chunk itself
  if (p.defer && coal && p.force_mode == IXG_MODE_AUTO) return (int)hipGetLastError();
  if (p.defer) {
    const ShortK& ks = p.dmx ? k_short_dmx : k_short;
    // one wave per 64 chunks (frames in host memory: one per chunk)
    const uint64_t ngroups = (nchunks + 63u) / 64u, bw = (uint64_t)ks.block / 64u;
    const uint64_t want = ((p.host_mem ? nchunks : ngroups) + bw - 1) / bw;
    KParams ps = p;
    ps.self_sample = self ? 1u : 0u;
    hipLaunchKernelGGL(ks.k[lay], dim3(grid_for(ks.k[lay], want, ncu, sh6, ks.block)), dim3(ks.block), sh6,
                       (hipStream_t)stream, ps);
  }
  // the flat walk's build (8-wave blocks) unless the IPv6 tables need the LDS,
  // or a fixed stride puts every chunk's span over kFlatRows KiB (C4: the
  // general kernel's big-chunk walk, glong's build of it is ~1 % slower)
  static const kern_fn k_glong[2] = {ixg_rx_glong_s, ixg_rx_glong_o};
  if (!p.tab6 && !p.host_mem && (p.off || 63ull * p.stride < 16ull * kFlatPieces)) {
    const kern_fn kg = k_glong[lay];
    const uint64_t gb8 = ((nchunks + 63u) / 64u + 7u) / 8u;
    hipLaunchKernelGGL(kg, dim3(grid_for(kg, gb8, ncu, 0, 512)), dim3(512), 0, (hipStream_t)stream, p);
    return (int)hipGetLastError();
  }
  const kern_fn kg = k_gen[lay];
  hipLaunchKernelGGL(kg, dim3(grid_for(kg, p.host_mem ? wave_blocks : group_blocks, ncu, sh6)), dim3(kBlock), sh6,
                     (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

// the fused tcp_input head runs in the coalesced fixed-shape kernel alone
// (ixg_rx_fastc_tcpx_s, which finishes every chunk of its batch itself): a
// coalesced fixed-stride layout in the default split, no fused demux
extern "C" int ixgrx_tcpx_fusable(const void* params) {
  const KParams& p = *static_cast<const KParams*>(params);
  const bool coal = !p.off && p.stride <= 64u && (p.stride & 3u) == 0u &&
                    (reinterpret_cast<uintptr_t>(p.base) & 15u) == 0u;
  return coal && p.defer && p.force_mode == IXG_MODE_AUTO && !p.dmx && !p.host_mem ? 1 : 0;
}

extern "C" uint32_t ixgrx_kparams_size(void) { return (uint32_t)sizeof(KParams); }
extern "C" uint32_t ixgrx_block(void) { return (uint32_t)kBlock; }
