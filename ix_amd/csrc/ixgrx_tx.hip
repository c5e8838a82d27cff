// ixgrx_tx.hip - MI355X (gfx950) TX header build + checksums: the mirror of
// the RX transform. For each struct ixg_tx_seg the frame
// IX's TX paths build on the host -- the Ethernet header of ip_send_one
// (dp/net/ip.c:198-213), the IPv4 header of tcp_output_packet
// (dp/net/tcp_api.c:791-806) or of udp_output + ip_setup_header
// (dp/net/udp.c:114-128, dp/net/net.h:65-78), the segment bytes -- plus the
// checksums: the IP header's (chksum_internet, inc/asm/chksum.h:40-95) and
// TCP's (the seed of inet_chksum_pseudo, dp/lwip/inet_chksum.c:324-357, for
// a NIC that finishes it, or the full one the NIC would put on the wire).
//
// A wave takes 64 segments. Pass A, one lane per segment: descriptor, header
// dwords, IP checksum and the TCP pseudo-header term, into per-wave LDS.
// Pass B, G lanes per segment (G = 4 when every frame of the 64 is at most
// 96 bytes, else 16): lane t of a group loads body piece j = G*r + t of
// round r and writes output piece k = j + 2 (16 bytes at frame + 16k). The
// headers are 34 (TCP) or 42 (UDP) bytes, so every output piece is bytes
// 14..15 (TCP) or 6..15 (UDP) of body piece j - 1 (the previous lane's, by
// a shuffle) followed by the start of piece j; "body piece -1" is the
// header's last 16 bytes. Loads are aligned
// to the segment start (4-byte aligned), stores to the frame start (16-byte
// aligned). TCP's body sum is reduced across the group and patched into
// output piece 3 (frame bytes 48..63, the checksum at 50..51) last.
//
// No MFMA: HBM-bound byte moving (read the segment, write the frame).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_tx.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_a4 __attribute__((aligned(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

using TParams = ixg_tparams;

DEV uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

DEV uint32_t fold16(uint64_t s) {
  s = (s & 0xffffffffull) + (s >> 32);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  s = (s & 0xffffu) + (s >> 16);
  return (uint32_t)s;
}

DEV uint32_t ones(int k) { return k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u)); }

// sum of the first `rem` bytes of a 16-byte piece as LE dwords (rest zero)
DEV uint64_t piece_sum(const u32x4& v, int rem) {
  return (uint64_t)(v.x & ones(rem)) + (v.y & ones(rem - 4)) + (v.z & ones(rem - 8)) + (v.w & ones(rem - 12));
}

// (a >> 16) | (b << 16): bytes 2..3 of a, then bytes 0..1 of b
DEV uint32_t mid(uint32_t a, uint32_t b) { return __builtin_amdgcn_alignbyte(b, a, 2); }

// per-wave pass-A results, one entry per segment of the chunk
constexpr int kHdr = 11;  // frame bytes 0..43 as dwords
struct WaveTx {
  lds_u32* src_lo; lds_u32* src_hi; lds_u32* out_lo; lds_u32* out_hi;
  lds_u32* meta;   // K (bits 0..15) | udp (16) | valid (17) | tcp_full (18)
  lds_u32* seg_len;
  lds_u32* l4term; // TCP: the seed (offload) or the pseudo-header sum (full)
  lds_u32* hdr;    // [kHdr][64]
};

// Pass A's result for one segment (lane = segment)
struct Seg {
  uint32_t h[kHdr];
  uint64_t sa, oa;  // segment and frame addresses
  uint32_t K, seg_len, term;
  bool valid, udp, full;
};

// A segment's descriptor (struct ixg_tx_seg, 40 bytes) as loaded
struct TDesc {
  u32x4 a, b;
  uint32_t c;  // ttl | dmac_idx << 16 (rsvd2 is not loaded)
};

// descriptor loads (segment 0's for lanes past the end: always issued)
DEV TDesc tx_desc(const TParams& p, uint64_t i) {
  const uint32_t* dp = reinterpret_cast<const uint32_t*>(p.segs + (i < p.n ? i : 0u));
  return TDesc{*reinterpret_cast<const u32x4_a4*>(dp), *reinterpret_cast<const u32x4_a4*>(dp + 4), dp[8]};
}

// the checks of a descriptor and its output pieces K (0 when invalid)
DEV bool tx_valid(const TParams& p, uint64_t i, const TDesc& d, uint32_t& K) {
  const uint64_t seg_off = d.a.x | ((uint64_t)d.a.y << 32), out_off = d.a.z | ((uint64_t)d.a.w << 32);
  const uint32_t seg_len = d.b.z & 0xffffu, proto = (d.b.w >> 16) & 0xffu, dmi = d.c >> 16;
  const bool tcp = proto == 6u, udp = proto == 17u;
  const uint32_t l4 = seg_len + (udp ? 8u : 0u);
  const bool valid = i < p.n && (tcp || udp) && !(tcp && seg_len < 20u) && 20u + l4 <= 0xffffu &&
                     dmi < p.n_dmac && (seg_off & 3u) == 0u && (out_off & 15u) == 0u;
  K = valid ? (34u + l4 + 15u) >> 4 : 0u;
  return valid;
}

// What pass A needs from memory besides the descriptor: the next-hop MAC
// and, for a chunk the small path takes, the segment's first 32 bytes.
// Loaded one chunk ahead (tx_loop), so the descriptor -> data dependency
// costs no round trip of its own.
struct TPre {
  u32x2 dm;
  u32x4 b0, b1;
};

DEV void tx_pre(const TParams& p, uint64_t i, const TDesc& d, int lane, TPre& x) {
  uint32_t K;
  const bool valid = tx_valid(p, i, d, K);
  const bool small = __all(K <= 4u);
  const uint32_t dmi = d.c >> 16;
  x.dm = *reinterpret_cast<const u32x2*>(p.dmacs + 2u * (valid ? dmi : 0u));
  const uint64_t sa = reinterpret_cast<uint64_t>(p.seg_buf) + (d.a.x | ((uint64_t)d.a.y << 32));
  const uint64_t zero = reinterpret_cast<uint64_t>(p.zero) + 16u * (uint32_t)lane;
  const bool ld = small && valid;
  x.b0 = *reinterpret_cast<const u32x4_a4*>(ld ? sa : zero);
  x.b1 = *reinterpret_cast<const u32x4_a4*>(ld ? sa + 16u : zero);
}

// Pass A: lane = segment: header dwords, checksum terms.
DEV Seg tx_prepare(const TParams& p, uint32_t i, const TDesc& d, const TPre& x) {
  const bool in = i < p.n;
  const u32x4 a = d.a, b = d.b;
  const uint64_t seg_off = a.x | ((uint64_t)a.y << 32), out_off = a.z | ((uint64_t)a.w << 32);
  const uint32_t src = b.x, dst = b.y, seg_len = b.z & 0xffffu, sport = b.z >> 16;
  const uint32_t dport = b.w & 0xffffu, proto = (b.w >> 16) & 0xffu, tos = b.w >> 24;
  const uint32_t ttl = d.c & 0xffu;
  const bool tcp = proto == 6u, udp = proto == 17u;
  const uint32_t l4 = seg_len + (udp ? 8u : 0u);
  uint32_t K;
  const bool valid = tx_valid(p, i, d, K);
  const uint32_t flen = 34u + l4;
  const u32x2 dm = x.dm;
  const bool offload = (p.flags & IXG_TX_OFFLOAD) != 0u;
  // the header, dwords of frame bytes 0..43 (ip_send_one + tcp_output_packet
  // / ip_setup_header + udp_output)
  Seg sg;
  uint32_t (&h)[kHdr] = sg.h;
  h[0] = dm.x;
  h[1] = (dm.y & 0xffffu) | (p.smac_lo << 16);
  h[2] = (p.smac_lo >> 16) | (p.smac_hi << 16);
  h[3] = 0x08u | (0x45u << 16) | ((tcp ? tos : 0u) << 24);      // type 0x0800, vhl, tos
  h[4] = bswap16(20u + l4);                                      // len, id 0
  h[5] = ((tcp ? ttl : 64u) << 16) | (proto << 24);              // off 0, ttl, proto
  h[6] = (src & 0xffffu) << 16;                                  // chksum (below), src
  h[7] = (src >> 16) | ((dst & 0xffffu) << 16);
  h[8] = (dst >> 16) | (udp ? bswap16(sport) << 16 : 0u);
  h[9] = udp ? (bswap16(dport) | (bswap16(l4) << 16)) : 0u;      // UDP len, checksum 0
  h[10] = 0u;
  // chksum_internet over bytes 14..33 (LE 16-bit words), unless a TCP frame
  // leaves it to the NIC
  if (udp || !offload) {
    const uint64_t s = (uint64_t)(h[3] >> 16) + (h[4] & 0xffffu) + (h[4] >> 16) + (h[5] & 0xffffu) + (h[5] >> 16) +
                       (h[6] >> 16) + (h[7] & 0xffffu) + (h[7] >> 16) + (dst >> 16);
    h[6] |= (~fold16(s)) & 0xffffu;
  }
  uint32_t term = 0;
  if (tcp && offload) {
    // in_pseudo(src, dst, hton32(proto + tot_len)) (inet_chksum.c:324-340)
    const uint64_t s = (uint64_t)src + dst + __builtin_bswap32(6u + seg_len);
    uint32_t sum = (uint32_t)s + (uint32_t)(s >> 32);
    sum = (sum & 0xffffu) + (sum >> 16);
    term = sum > 0xffffu ? sum - 0xffffu : sum;
  } else if (tcp) {
    // pseudo header as inet_chksum_pseudo_partial adds it (:454-472, :436-437)
    term = (src & 0xffffu) + (src >> 16) + (dst & 0xffffu) + (dst >> 16) + (6u << 8) + bswap16(seg_len);
  }
  sg.K = K;
  sg.sa = reinterpret_cast<uint64_t>(p.seg_buf) + seg_off;
  sg.oa = reinterpret_cast<uint64_t>(p.out) + out_off;
  sg.seg_len = seg_len;
  sg.term = term;
  sg.valid = valid;
  sg.udp = udp;
  sg.full = tcp && !offload;
  if (in) p.out_len[i] = (uint16_t)(valid ? flen : 0u);
  return sg;
}

DEV void tx_publish(const Seg& sg, int lane, const WaveTx& w) {
  w.src_lo[lane] = (uint32_t)sg.sa;
  w.src_hi[lane] = (uint32_t)(sg.sa >> 32);
  w.out_lo[lane] = (uint32_t)sg.oa;
  w.out_hi[lane] = (uint32_t)(sg.oa >> 32);
  w.meta[lane] = sg.K | (sg.udp ? 1u << 16 : 0u) | (sg.valid ? 1u << 17 : 0u) | (sg.full ? 1u << 18 : 0u);
  w.seg_len[lane] = sg.seg_len;
  w.l4term[lane] = sg.term;
#pragma unroll
  for (int k = 0; k < kHdr; k++) w.hdr[k * 64 + lane] = sg.h[k];
}

DEV void store16(uint64_t addr, const u32x4& v) { *reinterpret_cast<u32x4*>(addr) = v; }
// the groups' body pieces: consecutive lanes fill whole lines, so streaming
// stores (3% on 1514-B frames; on the lane-per-segment small path, whose
// 16-byte pieces land in 64 different frames per instruction, they halve the
// rate, so that path keeps default-policy stores)
DEV void store16_nt(uint64_t addr, const u32x4& v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(addr)); }

// rounds in flight per segment group in the streaming pass (one 16-byte
// load per lane and round): 6 = every round of a 1514-B frame's 16-lane
// group at once (1514-B frames -7 %, mixed -2.5 % against 3 in a
// same-process A/B); the next group's are issued before this group's are
// consumed (tx_stream), a further -9 % on 1514-B and mixed frames
#ifndef IXG_TX_RIF
#define IXG_TX_RIF 6
#endif
constexpr int kTxRif = IXG_TX_RIF;

// lane t - 1's value within groups of G lanes (lane 0: lane G - 1's)
template <int G>
DEV uint32_t rot1(uint32_t v) {
  static_assert(G == 16 || G == 4, "DPP rotations within rows of 16 or quads");
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, G == 16 ? 0x121 : 0x93, 0xf, 0xf, false);
}

// Pass B: G lanes per segment, 64 / G segments at a time. Lane t of round r
// loads body piece j = G r + t (aligned to the segment) and writes output
// piece k = j + 2: bytes 14..15 (TCP) / 6..15 (UDP) of piece j - 1, then the
// start of piece j. Piece j - 1 is the previous lane's (a shuffle), for the
// group's first lane the previous round's last lane's (kept from that round),
// and before round 0 the header's last 16 bytes: every load is the lane's
// own piece (an earlier build also loaded piece j + 1 in the group's last
// lane: twice the loads and registers per round). TCP's sum (each lane sums
// its own piece) is reduced across the group and patched into output piece 3
// (frame bytes 48..63, the checksum at 50..51), stored last.
template <int G>
DEV void tx_stream(const TParams& p, int lane, const WaveTx& w) {
  const int g = lane / G, t = lane % G;
  const uint64_t zero = reinterpret_cast<uint64_t>(p.zero) + 16u * (uint32_t)lane;
  // the first kTxRif rounds' loads of segment si (always issued: the zero
  // page when there is nothing to read)
  auto first_loads = [&](int si, u32x4 (&v)[kTxRif]) {
    const uint32_t meta = w.meta[si];
    const int K = (int)(meta & 0xffffu);
    const int nr = ((meta >> 17) & 1u) ? (K - 2 + G - 1) / G : 0;
    const uint64_t src = ((uint64_t)w.src_hi[si] << 32) | w.src_lo[si];
#pragma unroll
    for (int q = 0; q < kTxRif; q++) {
      const int j = G * q + t;
      const bool act = q < nr && j + 2 < K;
      v[q] = *reinterpret_cast<const u32x4_a4*>(act ? src + 16u * (uint32_t)j : zero);
    }
  };
  // software pipeline over the segment groups: the next group's first
  // rounds are in flight while this group's are shifted and stored
  u32x4 nxt[kTxRif];
  first_loads(g, nxt);
  for (int s0 = 0; s0 < 64; s0 += 64 / G) {
    const int si = s0 + g;
    u32x4 cur[kTxRif];
#pragma unroll
    for (int q = 0; q < kTxRif; q++) cur[q] = nxt[q];
    if (s0 + 64 / G < 64) first_loads(si + 64 / G, nxt);
    const uint32_t meta = w.meta[si];
    const bool valid = (meta >> 17) & 1u, udp = (meta >> 16) & 1u, full = (meta >> 18) & 1u;
    const int K = (int)(meta & 0xffffu);
    const int seg_len = (int)w.seg_len[si];
    const uint64_t src = ((uint64_t)w.src_hi[si] << 32) | w.src_lo[si];
    const uint64_t out = ((uint64_t)w.out_hi[si] << 32) | w.out_lo[si];
    // header dwords this lane may need
    const int hb = udp ? 6 : 4;  // body piece -1 = frame bytes [H - 16, H): dwords hb..hb+4
    uint32_t hp[5];
#pragma unroll
    for (int k = 0; k < 5; k++) hp[k] = w.hdr[(hb + k) * 64 + si];
    u32x4 carry = {mid(hp[0], hp[1]), mid(hp[1], hp[2]), mid(hp[2], hp[3]), mid(hp[3], hp[4])};
    const int nr = valid ? (K - 2 + G - 1) / G : 0;  // output pieces 2..K-1
    uint64_t acc = 0;
    u32x4 held = {0u, 0u, 0u, 0u};
    // always-issued loads (the zero page when there is nothing to read)
    auto issue = [&](int r) {
      const int j = G * r + t;
      const bool act = r < nr && j + 2 < K;
      return *reinterpret_cast<const u32x4_a4*>(act ? src + 16u * (uint32_t)j : zero);
    };
    auto round = [&](int r, const u32x4& own) {
      const int j = G * r + t;
      const bool act = r < nr && j + 2 < K;
      // rotate the group's pieces by one lane (DPP row_ror:1 for 16-lane
      // groups, quad_perm [3,0,1,2] for 4-lane ones): lane t gets lane
      // t - 1's piece, lane 0 its group's last lane's, which is the next
      // round's lane-0 predecessor
      const u32x4 rot = {rot1<G>(own.x), rot1<G>(own.y), rot1<G>(own.z), rot1<G>(own.w)};
      const u32x4 prev = t == 0 ? carry : rot;
      carry = rot;
      u32x4 o;
      if (udp) {
        o = {mid(prev.y, prev.z), mid(prev.z, prev.w), mid(prev.w, own.x), mid(own.x, own.y)};
      } else {
        o = {mid(prev.w, own.x), mid(own.x, own.y), mid(own.y, own.z), mid(own.z, own.w)};
      }
      const int k = j + 2;
      if (act) {
        if (!udp && k == 3)
          held = o;  // holds the TCP checksum: stored after the reduction
        else
          store16_nt(out + 16u * (uint32_t)k, o);
      }
      if (act && r == 0 && t == 0) {
        store16(out, u32x4{w.hdr[0 * 64 + si], w.hdr[1 * 64 + si], w.hdr[2 * 64 + si], w.hdr[3 * 64 + si]});
        store16(out + 16u, u32x4{w.hdr[4 * 64 + si], w.hdr[5 * 64 + si], w.hdr[6 * 64 + si], w.hdr[7 * 64 + si]});
      }
      // each lane sums its own body piece: pieces 0..K-3 cover the segment
      // (K - 2 >= ceil(seg_len / 16))
      if (full && act) {
        u32x4 sv = own;
        if (j == 1) sv.x &= 0xffff0000u;  // the checksum field (segment bytes 16..17) counts as 0
        const int rem = seg_len - 16 * j;
        if (__all(!act || rem >= 16))
          acc += (uint64_t)sv.x + sv.y + sv.z + sv.w;
        else
          acc += piece_sum(sv, rem);
      }
    };
#pragma unroll
    for (int q = 0; q < kTxRif; q++) round(q, cur[q]);
    // segments longer than kTxRif rounds (not IX's MTU-sized ones): the
    // rest, one round at a time
    for (int r = kTxRif; __any(r < nr); r++) {
      const u32x4 v = issue(r);
      round(r, v);
    }
    if (!udp) {
#pragma unroll
      for (int m = 1; m < G; m <<= 1) {
        const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)acc, m, G);
        const uint32_t hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(acc >> 32), m, G);
        acc += ((uint64_t)hi32 << 32) | lo32;
      }
      if (valid && t == 1) {
        const uint32_t term = w.l4term[si];
        const uint32_t ck = full ? (~fold16(acc + term)) & 0xffffu : term;
        held.x = (held.x & 0xffffu) | (ck << 16);
        store16(out + 48u, held);
      }
    }
  }
}

// Every frame of the chunk fits 64 bytes (K <= 4: a TCP segment of at most
// 30 bytes, a UDP payload of at most 22): lane = segment, all in registers.
// Output pieces 0, 1 are header; piece 2 = header bytes [H-16, H) + body
// piece 0, piece 3 = body pieces 0 and 1 (as in tx_stream, j = -1 and 0).
// (b0, b1: the segment's first 32 bytes, prefetched by tx_pre; buf: the
// wave's 4 KiB of LDS for the coalesced store)
DEV void tx_small(const TParams& p, const Seg& sg, const u32x4& b0, const u32x4& b1, int lane, lds_u32* buf) {
  const uint32_t* h = sg.h;
  u32x4 pm1, o2, o3;
  if (sg.udp) {
    pm1 = {mid(h[6], h[7]), mid(h[7], h[8]), mid(h[8], h[9]), mid(h[9], h[10])};
    o2 = {mid(pm1.y, pm1.z), mid(pm1.z, pm1.w), mid(pm1.w, b0.x), mid(b0.x, b0.y)};
    o3 = {mid(b0.y, b0.z), mid(b0.z, b0.w), mid(b0.w, b1.x), mid(b1.x, b1.y)};
  } else {
    pm1 = {mid(h[4], h[5]), mid(h[5], h[6]), mid(h[6], h[7]), mid(h[7], h[8])};
    o2 = {mid(pm1.w, b0.x), mid(b0.x, b0.y), mid(b0.y, b0.z), mid(b0.z, b0.w)};
    o3 = {mid(b0.w, b1.x), mid(b1.x, b1.y), mid(b1.y, b1.z), mid(b1.z, b1.w)};
    const int L = (int)sg.seg_len;
    u32x4 c1 = b1;
    c1.x &= 0xffff0000u;  // the checksum field counts as 0
    const uint64_t acc = piece_sum(b0, L) + piece_sum(c1, L - 16);
    const uint32_t ck = sg.full ? (~fold16(acc + sg.term)) & 0xffffu : sg.term;
    o3.x = (o3.x & 0xffffu) | (ck << 16);
  }
  // 64 valid 64-byte frames back to back (packed echo replies): the wave's
  // 4 KiB go out through LDS as 4 fully coalesced 1 KiB stores instead of
  // 16-byte pieces into 64 different lines per store
  const uint64_t oa0 = __shfl(sg.oa, 0);
  if (__all(sg.valid && sg.K == 4u && sg.oa == oa0 + 64u * (uint32_t)lane)) {
    lds_u32* q = buf + 16 * lane;
    const u32x4 pc[4] = {u32x4{h[0], h[1], h[2], h[3]}, u32x4{h[4], h[5], h[6], h[7]}, o2, o3};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      q[4 * k + 0] = pc[k].x; q[4 * k + 1] = pc[k].y; q[4 * k + 2] = pc[k].z; q[4 * k + 3] = pc[k].w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const lds_u32* r = buf + 4 * (lane + 64 * k);
      store16(oa0 + 16u * (uint32_t)(lane + 64 * k), u32x4{r[0], r[1], r[2], r[3]});
    }
    // the next chunk's LDS writes must not pass these reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return;
  }
  if (sg.valid) {
    store16(sg.oa, u32x4{h[0], h[1], h[2], h[3]});
    store16(sg.oa + 16u, u32x4{h[4], h[5], h[6], h[7]});
    store16(sg.oa + 32u, o2);
    if (sg.K > 3u) store16(sg.oa + 48u, o3);
  }
}

// One chunk of 64 segments per wave (the grid has a wave per chunk: see
// ixgrx_tx_launch), so no loads are carried across chunks.
DEV void tx_chunk(const TParams& p, const WaveTx& w) {
  const int lane = threadIdx.x & 63;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  const uint32_t c = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (c >= nchunks) return;
  const uint32_t i = c * 64u + (uint32_t)lane;
  const TDesc d0 = tx_desc(p, i);
  TPre x0;
  tx_pre(p, i, d0, lane, x0);
  uint32_t K0;
  tx_valid(p, i, d0, K0);
  const Seg sg = tx_prepare(p, i, d0, x0);
  if (__all(K0 <= 4u)) {
    tx_small(p, sg, x0.b0, x0.b1, lane, w.src_lo);
    return;
  }
  tx_publish(sg, lane, w);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (__all(sg.K <= 6u))
    tx_stream<4>(p, lane, w);
  else
    tx_stream<16>(p, lane, w);
}

}  // namespace

// 3 waves/SIMD (161 VGPRs: two groups' rounds in registers); at 4 or 5 the
// pipelined streaming pass spills
#ifndef IXG_TX_WAVES
#define IXG_TX_WAVES 3
#endif
extern "C" __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(IXG_TX_WAVES)))
ixg_tx_build(TParams p) {
  __shared__ uint32_t sh[kWaves][(7 + kHdr) * 64];
  lds_u32* b = (lds_u32*)sh[threadIdx.x >> 6];
  const WaveTx w{b, b + 64, b + 128, b + 192, b + 256, b + 320, b + 384, b + 448};
  tx_chunk(p, w);
}

extern "C" int ixgrx_tx_launch(const void* params, uint32_t ncu, void* stream) {
  const TParams& p = *static_cast<const TParams*>(params);
  const uint64_t nchunks = ((uint64_t)p.n + 63u) / 64u;
  const uint64_t want = (nchunks + kWaves - 1) / kWaves;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ixg_tx_build, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
  const uint64_t cap = (uint64_t)ncu * (uint64_t)nb;
  // one wave per chunk, not a persistent grid: 1514-B frames -1.5 %, mixed
  // sizes -13 %, echo replies -8 % in a same-process A/B (the dispatcher
  // keeps every CU fed; a plain copy behaves the same, tools/probe_copy.hip)
  (void)cap;
  const uint32_t grid = (uint32_t)want;
  hipLaunchKernelGGL(ixg_tx_build, dim3(grid ? grid : 1u), dim3(kBlock), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}
