// ixgrx_kernels.hip - MI355X (gfx950) RX parse + checksum + flow-hash kernels.
//
// One wavefront lane per packet. Each lane loads the first 96 bytes of its
// frame as 16-byte vector loads (header prefix; the IPv4 header with options
// and every L4 header field the path reads sit inside it), parses
// Ethernet/IPv4/TCP/UDP/ICMP exactly as dp/net/ip.c + dp/lwip do, sums the
// IP header and the in-prefix part of the L4 segment as 32-bit one's
// complement words, and looks the 12 tuple bytes up in a per-workgroup LDS
// copy of the combined Toeplitz/CRC-32C byte tables (both hashes are
// GF(2)-affine in the tuple, DESIGN.md "hash tables"). Segments that extend
// past the prefix (IMIX, 1500 B frames) are compacted per wave with
// ballot/mbcnt into an LDS list and summed cooperatively: 16 lanes (one DPP
// row) per packet, 256 contiguous bytes per wave-instruction per packet,
// up to 8 loads in flight per lane, then a row reduction.
//
// A wave whose 64 packets are all plain IPv4 (ihl 5, segment ending inside
// the first 64 bytes: the 64 B TCP config) takes an instantiation where the
// header geometry is constant-folded. Both instantiations produce identical
// records (same code, template on a constant).
//
// No MFMA: this is integer byte work bound by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_internal.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;        // 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kPrefixDw = 24;      // 96-byte header prefix
constexpr int kFastDw = 16;        // the fast shape needs 64 bytes
constexpr int kStreamBase = 96;    // long segments: streamed from here
constexpr int kGroup = 16;         // lanes per packet in the streaming sum
constexpr int kStreamUnroll = 8;   // 16-byte loads per lane per pass

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
};

template <bool FAST>
DEV void lane_parse(const KParams& p, const uint64_t* __restrict__ T, const uint32_t (&d)[kPrefixDw],
                    uint32_t L, LaneState& s) {
  const uint32_t etype = (byte_at(d, 12) << 8) | byte_at(d, 13);       // ip.c:132
  const uint32_t vh = byte_at(d, 14);
  const uint32_t ver = vh >> 4;
  const int ihl = FAST ? 5 : (int)(vh & 15u);                             // ip.h:84-90
  const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
  const uint32_t ip_off = (byte_at(d, 20) << 8) | byte_at(d, 21);
  const uint32_t proto = byte_at(d, 23);
  const bool frag = (ip_off & 0x3fffu) != 0;                              // ip.c:78
  const uint32_t src = (d[6] >> 16) | (d[7] << 16);                       // bytes 26..29 raw
  const uint32_t dst = (d[7] >> 16) | (d[8] << 16);                       // bytes 30..33 raw
  const int l4 = 14 + 4 * ihl;
  const bool ip4 = etype == 0x0800u;
  const bool v6 = !FAST && etype == 0x86DDu && (p.flags & IXG_F_IPV6);

  // L4 header dwords: frame byte l4+b sits in dword q + (2+b)/4
  const int q = 3 + (ihl < 5 ? 5 : ihl);
  uint32_t h0, h1, h3;
  if (FAST) {
    h0 = d[8]; h1 = d[9]; h3 = d[11];
  } else {
    h0 = pick<kPrefixDw, 8, 18>(d, q);
    h1 = pick<kPrefixDw, 9, 19>(d, q + 1);
    h3 = pick<kPrefixDw, 11, 21>(d, q + 3);
  }
  // IPv6 extension: fixed offsets (L4 at 54 = dword 13 + 2)
  if (v6) { h0 = d[13]; h1 = d[14]; h3 = d[16]; }
  const uint32_t b0 = (h0 >> 16) & 0xffu, b1 = h0 >> 24;                  // sport (wire)
  const uint32_t b2 = h1 & 0xffu, b3 = (h1 >> 8) & 0xffu;                 // dport (wire)
  const uint32_t w45 = h1 >> 16;                                          // L4 bytes 4,5 (LE)
  const uint32_t doff_byte = (h3 >> 16) & 0xffu;                          // TCP byte 12
  const uint32_t tflags = h3 >> 24;                                       // TCP byte 13

  s.v6 = v6;
  s.proto = v6 ? byte_at(d, 20) : proto;
  const uint32_t v6_plen = (byte_at(d, 18) << 8) | byte_at(d, 19);
  const bool v6_ok = v6 && L >= 54 && (vh >> 4) == 6 && 54 + v6_plen <= L;

  // ---- [NIC] IPv4 header checksum (DESIGN.md NIC rules) ----
  const bool hdr_ok = ip4 && ver == 4 && ihl >= 5 && (uint32_t)l4 <= L;
  s.flags = 0;
  s.ip_res = 0xffffu;
  if (hdr_ok) {
    uint64_t hs;
    if (FAST) {
      hs = (uint64_t)(d[3] >> 16) + d[4] + d[5] + d[6] + d[7] + (d[8] & 0xffffu);
    } else {
      hs = region_sum(d, 3, l4);
    }
    s.ip_res = (~fold16(hs)) & 0xffffu;                                    // chksum_internet
    s.flags |= IXG_RF_IP_CSUM_CHECKED | (s.ip_res == 0 ? IXG_RF_IP_CSUM_OK : 0u);
  }

  // ---- [NIC] RSS Toeplitz + tcp_to_idx via the byte tables ----
  const bool rss4 = hdr_ok && !frag && (proto == 6 || proto == 17) && (uint32_t)(l4 + 4) <= L;
  uint64_t hx = 0;
  {
    const uint32_t t4 = b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
    uint32_t sb = src, db = dst, pb = t4;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      hx ^= T[(k << 8) | ((sb >> (8 * k)) & 0xffu)];
      hx ^= T[((4 + k) << 8) | ((db >> (8 * k)) & 0xffu)];
      hx ^= T[((8 + k) << 8) | ((pb >> (8 * k)) & 0xffu)];
    }
  }
  s.rss = 0;
  if (rss4) {
    s.rss = (uint32_t)hx;
    s.flags |= IXG_RF_RSS;
  }
  // IPv6 extension: Toeplitz over src(16) dst(16) sport dport from a global
  // 36 x 256 table (L2-resident; only v6 lanes touch it)
  if (v6 && L >= 58 && ver == 6 && (s.proto == 6 || s.proto == 17)) {
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 32; k++) h ^= p.tab6[(k << 8) | byte_at(d, 22 + k)];
#pragma unroll
    for (int k = 0; k < 4; k++) h ^= p.tab6[((32 + k) << 8) | byte_at(d, 54 + k)];
    s.rss = h;
    s.flags |= IXG_RF_RSS;
  }
  s.fg = p.fg_base + (s.rss & p.fg_mask);
  s.bucket = ((uint32_t)(hx >> 32) ^ p.crc_const) & (IXG_PCB_BUCKETS - 1);

  // ---- L4 segment: [l4, 14 + ip_len) ----
  uint32_t l4len = ip_len - 4u * (uint32_t)ihl;
  uint32_t seg_end = 14 + ip_len;
  bool seg_ok = ip4 && ver == 4 && ihl >= 5 && !frag && ip_len >= 4u * (uint32_t)ihl && seg_end <= L;
  int qa = q;
  if (v6) {
    l4len = v6_plen;
    seg_end = 54 + v6_plen;
    seg_ok = v6_ok;
    qa = 13;
  }
  s.l4 = v6 ? 54 : l4;
  s.l4len = l4len;
  s.seg_end = seg_end;
  s.doff = doff_byte >> 4;
  s.tcp_flags = tflags & 0x3fu;
  s.ulen = bswap16(w45);
  s.icmp_type = b0;

  const uint32_t sp = s.proto;
  // UDP checksum field: L4 bytes 6,7 = low half of dword q+2
  const uint32_t ucs = v6 ? 1u : (pick<kPrefixDw, 10, 20>(d, q + 2) & 0xffffu);
  int kind = 0;
  if (seg_ok && ((sp == 6 && l4len >= 20) || (sp == 17 && l4len >= 8 && ucs != 0))) kind = 1;
  if (!v6 && seg_ok && sp == 1 && l4len >= 8) kind = 2;
  s.l4_kind = kind;
  uint64_t acc = 0;
  if (kind) {
    const int e = (int)(seg_end < (uint32_t)(FAST ? 4 * kFastDw : kStreamBase) ? seg_end
                                                                             : (FAST ? 4 * kFastDw : kStreamBase));
    if (FAST) {
      uint32_t dd[kFastDw];
#pragma unroll
      for (int j = 0; j < kFastDw; j++) dd[j] = d[j];
      acc = region_sum(dd, 8, e);
    } else {
      acc = region_sum(d, qa, e);
    }
    if (kind == 1) {
      uint64_t ps;
      if (v6) {
        ps = region_sum(d, 5, 54);                      // src + dst (bytes 22..53)
      } else {
        ps = (uint64_t)(src & 0xffffu) + (src >> 16) + (dst & 0xffffu) + (dst >> 16);
      }
      acc += ps + (sp << 8) + bswap16(l4len & 0xffffu);  // htons(proto) + htons(proto_len)
    }
  }
  s.l4_acc = acc;
  s.stream = kind != 0 && seg_end > (uint32_t)kStreamBase;
  if (FAST) s.stream = false;
}

// Verdict + record once the L4 sum is complete (mirrors ixgo rx_one order).
DEV void lane_finish(const KParams& p, const uint32_t (&d)[kPrefixDw], uint32_t L, LaneState& s) {
  const uint32_t etype = (byte_at(d, 12) << 8) | byte_at(d, 13);
  const uint32_t vh = byte_at(d, 14);
  const uint32_t ver = vh >> 4, ihl = vh & 15u;
  const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
  const uint32_t ip_off = (byte_at(d, 20) << 8) | byte_at(d, 21);
  const bool frag = (ip_off & 0x3fffu) != 0;

  s.l4_res = 0xffffu;
  if (s.l4_kind) {
    s.l4_res = (~fold16(s.l4_acc)) & 0xffffu;
    if (s.l4_kind == 1)
      s.flags |= IXG_RF_L4_CSUM_CHECKED | (s.l4_res == 0 ? IXG_RF_L4_CSUM_OK : 0u);
  }

  uint32_t v = 0, off = 0, len = 0, bucket = IXG_NO_BUCKET, tfl = 0;
  const bool csum_drop = !(p.flags & IXG_F_NO_CSUM_DROP);
  const uint32_t proto = s.proto, l4 = s.l4, l4len = s.l4len;
  if (csum_drop && (s.flags & IXG_RF_IP_CSUM_CHECKED) && !(s.flags & IXG_RF_IP_CSUM_OK)) {
    v = IXG_V_DROP_CSUM_IP;                                         // ixgbe.c:313-317
  } else if (csum_drop && (s.flags & IXG_RF_L4_CSUM_CHECKED) && !(s.flags & IXG_RF_L4_CSUM_OK)) {
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
        else if (s.l4_res != 0) v = IXG_V_DROP_ICMP_CSUM;           // icmp.c:82
        else if (s.icmp_type != 8) v = IXG_V_DROP_ICMP_TYPE;        // icmp.c:88-108
        else { v = IXG_V_ICMP_ECHO; off = l4; len = l4len; }
      } else {
        v = s.v6 ? IXG_V_DROP_IP6 : IXG_V_DROP_IP_PROTO;            // ip.c:106-107
      }
    }
  }
  s.verdict = v;
  s.l4_off = off & 0xffffu;
  s.l4_len = len & 0xffffu;
  s.bucket = bucket;
  s.tcp_flags = tfl;
}

DEV const uint8_t* frame_ptr(const KParams& p, uint32_t i) {
  return p.base + (p.off ? p.off[i] : (uint64_t)i * p.stride);
}

// load 16-byte chunks [K0, K1) of the prefix; chunk k only if 16k < L
template <int K0, int K1>
DEV void load_prefix(const uint8_t* f, uint32_t L, uint32_t (&d)[kPrefixDw]) {
#pragma unroll
  for (int k = K0; k < K1; k++) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if ((uint32_t)(16 * k) < L) v = *reinterpret_cast<const u32x4_a4*>(f + 16 * k);
    // bytes at offsets >= L read as zero (DESIGN.md "bytes beyond L")
    d[4 * k + 0] = v.x & ones((int)L - (16 * k + 0) < 0 ? 0 : (int)L - (16 * k + 0));
    d[4 * k + 1] = v.y & ones((int)L - (16 * k + 4) < 0 ? 0 : (int)L - (16 * k + 4));
    d[4 * k + 2] = v.z & ones((int)L - (16 * k + 8) < 0 ? 0 : (int)L - (16 * k + 8));
    d[4 * k + 3] = v.w & ones((int)L - (16 * k + 12) < 0 ? 0 : (int)L - (16 * k + 12));
  }
}

// Cooperative sum of [kStreamBase, seg_end) for the lanes with s.stream set.
DEV void stream_sums(const KParams& p, uint32_t pkt0, int lane, uint32_t* lds_list, uint32_t* lds_sum,
                     LaneState& s) {
  const uint64_t lm = __ballot(s.stream);
  if (lm == 0) return;
  const int nlong = __popcll(lm);
  // wave compaction: rank of this lane among the long lanes
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
  if (s.stream) lds_list[rank] = (uint32_t)lane;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int grp = lane / kGroup, gl = lane % kGroup;
  const uint32_t my_end = s.seg_end;
  for (int r0 = 0; r0 < nlong; r0 += 64 / kGroup) {
    const int k = r0 + grp;
    const bool act = k < nlong;
    const uint32_t owner = act ? lds_list[k] : 0u;
    const uint32_t end = (uint32_t)__shfl((int)my_end, (int)owner);
    const uint8_t* f = frame_ptr(p, pkt0 + owner);
    uint64_t acc = 0;
    // chunk c covers bytes [96 + 16c, 96 + 16c + 16); lane gl takes c = gl + 16t
    for (uint32_t c0 = 0;; c0 += kGroup * kStreamUnroll) {
      const bool more = act && (uint32_t)kStreamBase + 16u * c0 < end;
      if (!__any(more)) break;
      u32x4 v[kStreamUnroll];
#pragma unroll
      for (int t = 0; t < kStreamUnroll; t++) {
        const uint32_t pos = kStreamBase + 16u * (c0 + gl + kGroup * t);
        v[t] = u32x4{0u, 0u, 0u, 0u};
        if (act && pos < end) v[t] = *reinterpret_cast<const u32x4_a4*>(f + pos);
      }
#pragma unroll
      for (int t = 0; t < kStreamUnroll; t++) {
        const uint32_t pos = kStreamBase + 16u * (c0 + gl + kGroup * t);
        const int rem = (int)end - (int)pos;  // bytes of this chunk inside the segment
        acc += v[t].x & ones(rem < 0 ? 0 : rem);
        acc += v[t].y & ones(rem - 4 < 0 ? 0 : rem - 4);
        acc += v[t].z & ones(rem - 8 < 0 ? 0 : rem - 8);
        acc += v[t].w & ones(rem - 12 < 0 ? 0 : rem - 12);
      }
    }
    uint32_t a = fold32(acc);
#pragma unroll
    for (int m = 1; m < kGroup; m <<= 1) a = add1c(a, (uint32_t)__shfl_xor((int)a, m, kGroup));
    if (act && gl == 0) lds_sum[owner] = a;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (s.stream) s.l4_acc += lds_sum[lane];
}

template <bool FAST>
DEV void process(const KParams& p, const uint64_t* __restrict__ T, uint32_t i, bool valid, uint32_t L,
                 uint32_t (&d)[kPrefixDw], uint32_t pkt0, int lane, uint32_t* lds_list, uint32_t* lds_sum) {
  LaneState s;
  lane_parse<FAST>(p, T, d, L, s);
  if (!FAST) {
    if (!valid) s.stream = false;
    stream_sums(p, pkt0, lane, lds_list, lds_sum, s);
  }
  lane_finish(p, d, L, s);
  if (valid) {
    Rec r;
    r.w0 = (s.fg & 0xffffu) | (s.verdict << 16) | (s.flags << 24);
    r.w1 = s.l4_off | (s.l4_len << 16);
    r.w2 = s.rss;
    r.w3 = s.bucket | (s.tcp_flags << 16);
    u32x4 w = {r.w0, r.w1, r.w2, r.w3};
    *reinterpret_cast<u32x4*>(p.out + i) = w;
    if (p.csum) p.csum[i] = s.ip_res | (s.l4_res << 16);
  }
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock)
ixg_rx_kernel(KParams p) {
  __shared__ uint64_t T[12 * 256];
  __shared__ uint32_t lds_list[kWaves][64];
  __shared__ uint32_t lds_sum[kWaves][64];
  // stage the hash tables (24 KiB) once per persistent workgroup
  for (int k = threadIdx.x; k < 12 * 256 / 2; k += kBlock) {
    const u32x4 v = reinterpret_cast<const u32x4*>(p.tab)[k];
    reinterpret_cast<u32x4*>(T)[k] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t blk = blockIdx.x * kBlock; blk < p.n; blk += gridDim.x * kBlock) {
    const uint32_t pkt0 = blk + wave * 64;
    const uint32_t i = pkt0 + lane;
    const bool valid = i < p.n;
    const uint32_t L = valid ? p.len[i] : 0u;
    const uint8_t* f = valid ? frame_ptr(p, i) : p.base;
    uint32_t d[kPrefixDw];
    load_prefix<0, 4>(f, L, d);
#pragma unroll
    for (int j = 16; j < kPrefixDw; j++) d[j] = 0;
    const uint32_t etype = (byte_at(d, 12) << 8) | byte_at(d, 13);
    const uint32_t ip_len = (byte_at(d, 16) << 8) | byte_at(d, 17);
    const bool fast = !valid || (etype == 0x0800u && byte_at(d, 14) == 0x45u && ip_len >= 20 && 14 + ip_len <= 64);
    if (__all(fast)) {
      process<true>(p, T, i, valid, L, d, pkt0, lane, lds_list[wave], lds_sum[wave]);
    } else {
      load_prefix<4, 6>(f, L, d);
      process<false>(p, T, i, valid, L, d, pkt0, lane, lds_list[wave], lds_sum[wave]);
    }
  }
}

extern "C" int ixgrx_launch(const void* params, uint32_t grid, void* stream) {
  const KParams& p = *static_cast<const KParams*>(params);
  hipLaunchKernelGGL(ixg_rx_kernel, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}

extern "C" uint32_t ixgrx_kparams_size(void) { return (uint32_t)sizeof(KParams); }

extern "C" int ixgrx_blocks_per_cu(void) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ixg_rx_kernel, kBlock, 0) != hipSuccess || nb < 1)
    nb = 1;
  return nb;
}
extern "C" uint32_t ixgrx_block(void) { return (uint32_t)kBlock; }
