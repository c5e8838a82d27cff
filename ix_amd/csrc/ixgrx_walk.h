// ixgrx_walk.h - the PCB lookup of tcp_input (dp/net/tcp_in.c:233-323,
// 500-510) for one lane, shared by the demux kernel (ixgrx_demux.hip) and the
// RX kernels' fused demux (ixgrx_kernels.hip). Device code only.
#ifndef IXGRX_WALK_H
#define IXGRX_WALK_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"

namespace ixgwalk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The list snapshot of ixg_demux_load, in HBM (small; L2 / Infinity Cache).
struct Tables {
  const uint32_t* active_start;  // nfg*512 + 1
  // per active bucket one 64-byte line: {count, CSR start, TIME-WAIT count,
  // TIME-WAIT start} + the first three entries of the active list in list
  // order, so the common case (a short bucket) is ONE dependent load instead
  // of bounds then entries
  const uint32_t* bline;
  const ixg_pcb_key* active;
  // each group's TIME-WAIT list split into per-bucket runs in list order
  // (ixg_demux_load): a segment can only match a pcb of its own 4-tuple,
  // whose tcp_to_idx bucket is the segment's, so the first match in the
  // bucket's run is the first match in the group's list
  const ixg_pcb_key* tw;
  const ixg_listen_key* listen;
  uint32_t nfg;  // groups in the snapshot: local, then outbound (ixg_demux_group)
  uint32_t n_listen;
};

// A segment no active or TIME-WAIT pcb took: tcp_in.c:273-304 without
// SO_REUSE / LWIP_IPV6 (opt.h:1579,2016) breaks at the first lpcb on the
// port whose address is the segment's destination or ANY; the hlist loop
// variable keeps the last entry when nothing breaks, so a non-empty list
// always yields an lpcb (tcp_in.c:317-323); no listener: RST, or nothing for
// a segment that carries RST itself (tcp_in.c:500-510, TCP_RST = 0x04)
__device__ __forceinline__ void no_pcb(const Tables& t, uint32_t tflags, uint32_t dst, uint32_t ports, uint32_t& id,
                                       uint32_t& kind) {
  const uint32_t dport = ports >> 16;
  if (t.n_listen != 0) {
    uint32_t k = 0;
    for (; k < t.n_listen; k++) {
      const u32x4 v = reinterpret_cast<const u32x4*>(t.listen)[k];
      if ((v.y & 0xffffu) == dport && (v.x == dst || v.x == 0u)) break;
    }
    if (k == t.n_listen) k = t.n_listen - 1;
    id = reinterpret_cast<const u32x4*>(t.listen)[k].z;
    kind = IXG_D_LISTEN;
  } else {
    kind = (tflags & 0x04u) ? IXG_D_DROP : IXG_D_RESET;
    id = 0;
  }
}

// tcp_input_find_list (tcp_in.c:122-143): the first entry of [s, e) whose
// (remote port, local port, remote ip, local ip) equals the segment's
__device__ __forceinline__ bool find_list(const ixg_pcb_key* __restrict__ ent, uint32_t s, uint32_t e,
                                          uint32_t ports, uint32_t src, uint32_t dst, uint32_t& id) {
  for (uint32_t k = s; k < e; k++) {
    const u32x4 v = reinterpret_cast<const u32x4*>(ent)[k];
    if (v.z == ports && v.x == src && v.y == dst) {
      id = v.w;
      return true;
    }
  }
  return false;
}

// The 64-byte bucket line of the snapshot's group `fg` (ixg_demux_group), PCB bucket `bucket`
// (null when fg is not a group of the tables)
__device__ __forceinline__ const u32x4* bucket_line(const Tables& t, uint32_t fg, uint32_t bucket) {
  return fg < t.nfg ? reinterpret_cast<const u32x4*>(t.bline) + 4u * (fg * IXG_PCB_BUCKETS + bucket) : nullptr;
}

// The bucket lines of a wave's 64 lanes (`line`: the lane's line index,
// nlines or more: none), loaded 4 lanes per 64-byte line: 16 lines per wave
// instruction, 4 instructions. A lane loading its own line made each
// instruction touch 64 lines, 4 times over, and the L1's per-line work
// bounded the fused demux (C2: 0.349 -> 0.323 ms per launch). Piece k of a
// lane: bytes 16*(lane&3).. of the line of lane (lane>>2) + 16k; a line
// index past the table reads 0 without touching memory (buffer bounds).
__device__ __forceinline__ void lines_issue(const uint32_t* bline, uint32_t nlines, uint32_t line, int lane,
                                            u32x4 (&piece)[4]) {
  // (word 3: 32-bit data format, raw addressing)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bline), 0, (int)(nlines * 64u), 0x00020000);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t li = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * ((lane >> 2) + 16 * k), (int)line);
    piece[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (li < nlines ? li : nlines) * 64u + 16u * (uint32_t)(lane & 3),
                                                     0, 0);
  }
}

// The lane's own line {hd, e0, e1, e2} from the pieces of lines_issue,
// through 4 KiB of the wave's LDS (free on entry; free again on return).
// Line j's piece q sits in 16-byte unit 4j + (q ^ ((j >> 2) & 3)): the
// writes (16 lanes: 4 lines x 4 pieces) and the reads (16 lanes: 16 lines,
// one piece) each cover all 16 units of an LDS row, no bank conflicts.
__device__ __forceinline__ void lines_exchange(const u32x4 (&piece)[4], int lane,
                                               __attribute__((address_space(3))) uint32_t* buf, u32x4 (&ln)[4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t j = (uint32_t)(lane >> 2) + 16u * k, q = (uint32_t)lane & 3u;
    __attribute__((address_space(3))) uint32_t* w = buf + 4u * (4u * j + (q ^ ((j >> 2) & 3u)));
    w[0] = piece[k].x;
    w[1] = piece[k].y;
    w[2] = piece[k].z;
    w[3] = piece[k].w;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t j = (uint32_t)lane, sw = (j >> 2) & 3u;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const __attribute__((address_space(3))) uint32_t* r = buf + 4u * (4u * j + ((uint32_t)q ^ sw));
    ln[q] = u32x4{r[0], r[1], r[2], r[3]};
  }
  // (the caller's next writes to buf must not pass these reads)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The rest of a lookup once the bucket line's first three entries missed:
// the active list past them (start + 3 .. start + cnt), the group's
// TIME-WAIT list, then the listen list or the reset / drop verdict. fg not a
// group of the tables: straight to the listen list.
__device__ __forceinline__ void walk_rest(const Tables& t, uint32_t fg, uint32_t tflags, uint32_t src, uint32_t dst,
                                          uint32_t ports, const u32x4& hd, uint32_t& id, uint32_t& kind) {
  const uint32_t start = hd.y, cnt = hd.x;
  bool hit = false;
  id = 0;
  kind = IXG_D_NONE;
  if (fg < t.nfg) {
    if (cnt > 3u) hit = find_list(t.active, start + 3u, start + cnt, ports, src, dst, id);
    if (hit) {
      kind = IXG_D_ACTIVE;  // tcp_in.c:249-256
    } else if (hd.z && find_list(t.tw, hd.w, hd.w + hd.z, ports, src, dst, id)) {
      kind = IXG_D_TIMEWAIT;  // tcp_in.c:260-269
      hit = true;
    }
  }
  if (!hit) no_pcb(t, tflags, dst, ports, id, kind);
}

// A pending lookup's key, one dword: group (14 bits) | PCB bucket << 14 |
// TCP flags << 23. Groups >= 0x3ffd are markers: a TCP frame of no group
// of the tables (kGrpNone: straight to the listen list), a frame whose
// record is not IXG_V_TCP (kGrpNotTcp), no frame (kGrpNoFrame).
constexpr uint32_t kGrpNone = 0x3fffu, kGrpNotTcp = 0x3ffeu, kGrpNoFrame = 0x3ffdu;
__device__ __forceinline__ uint32_t lookup_key(uint32_t grp, uint32_t bucket, uint32_t tflags) {
  return grp | (bucket << 14) | (tflags << 23);
}

// The lookups a bucket line could not decide, queued per wave (lane j holds
// item j) and walked 64 at a time: one in ~50 segments of C2 (its PCB is
// past its bucket's first three entries) but in ~70 % of chunks, where a
// synchronous walk made the whole wave wait out its dependent loads
// (C2 demux: 12 % of the launch). An item is the frame index and its key;
// the walk reloads the bucket line's count and start.
// Frames: when base is set the 4-tuple is not queued but read back at the
// walk (fixed-stride frames of IPv4 ihl 5: bytes 26..37 of base + i *
// stride), which keeps the queue at 2 VGPRs.
struct SlowQ {
  uint32_t i, key, src, dst, ports;
  uint32_t n;  // items held (wave-uniform)
};
struct Frames {
  const uint8_t* base;  // null: the tuple is queued
  uint32_t stride;
};

// walk the queued items; their demux records go to out[i]
__device__ __forceinline__ void slowq_flush(const Tables& t, SlowQ& q, int lane, uint32_t* out, const Frames& f) {
  if (q.n == 0u) return;
  if ((uint32_t)lane < q.n) {
    uint32_t src = q.src, dst = q.dst, ports = q.ports;
    if (f.base) {  // bytes 24..39: d6..d9 of the frame
      typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
      const u32x4a v = *reinterpret_cast<const u32x4a*>(f.base + (uint64_t)q.i * f.stride + 24u);
      src = (v.x >> 16) | (v.y << 16);
      dst = (v.y >> 16) | (v.z << 16);
      const uint32_t sp = v.z >> 16, dp = v.w & 0xffffu;
      ports = (((sp & 0xffu) << 8) | (sp >> 8)) | ((((dp & 0xffu) << 8) | (dp >> 8)) << 16);
    }
    const uint32_t g = q.key & 0x3fffu;
    u32x4 hd = u32x4{0u, 0u, 0u, 0u};
    if (g < t.nfg) hd = reinterpret_cast<const u32x4*>(t.bline)[4u * (g * IXG_PCB_BUCKETS + ((q.key >> 14) & 0x1ffu))];
    uint32_t id, kind;
    walk_rest(t, g, q.key >> 23, src, dst, ports, hd, id, kind);
    typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
    reinterpret_cast<u32x2v*>(out)[q.i] = u32x2v{id, kind};
  }
  q.n = 0;
}

// The lookup of frame i (key: lookup_key) given its bucket line (hd,
// e0..e2). A frame the line decides (its PCB among the bucket's first three
// entries) has its record stored to out[i] now; an undecided TCP frame joins
// the queue (through buf, 2 KiB of the wave's LDS, free), walked first if it
// would overflow. Frames that are not TCP store nothing here.
__device__ __forceinline__ void walk_line(const Tables& t, SlowQ& q, uint32_t i, uint32_t key, uint32_t src,
                                          uint32_t dst, uint32_t ports, const u32x4& hd, const u32x4& e0,
                                          const u32x4& e1, const u32x4& e2, int lane,
                                          __attribute__((address_space(3))) uint32_t* buf, uint32_t* out,
                                          const Frames& f) {
  const uint32_t g = key & 0x3fffu;
  const bool tcp = g != kGrpNotTcp && g != kGrpNoFrame;
  const uint32_t cnt = g < t.nfg ? hd.x : 0u;
  const bool m0 = cnt > 0u && e0.z == ports && e0.x == src && e0.y == dst;
  const bool m1 = cnt > 1u && e1.z == ports && e1.x == src && e1.y == dst;
  const bool m2 = cnt > 2u && e2.z == ports && e2.x == src && e2.y == dst;
  const bool hit = m0 || m1 || m2;
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  if (tcp && hit)
    reinterpret_cast<u32x2v*>(out)[i] = u32x2v{m0 ? e0.w : (m1 ? e1.w : e2.w), (uint32_t)IXG_D_ACTIVE};  // tcp_in.c:249-256
  const bool need = tcp && !hit;
  const uint64_t m = __builtin_amdgcn_ballot_w64(need);
  if (m == 0u) return;
  const uint32_t nn = (uint32_t)__builtin_popcountll(m);
  if (q.n + nn > 64u) slowq_flush(t, q, lane, out, f);
  if (need) {
    const uint32_t pos = q.n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    __attribute__((address_space(3))) uint32_t* w = buf + 8u * pos;
    w[0] = i;
    w[1] = key;
    if (!f.base) {
      w[2] = src;
      w[3] = dst;
      w[4] = ports;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if ((uint32_t)lane >= q.n && (uint32_t)lane < q.n + nn) {
    const __attribute__((address_space(3))) uint32_t* r = buf + 8u * (uint32_t)lane;
    q.i = r[0];
    q.key = r[1];
    if (!f.base) {
      q.src = r[2];
      q.dst = r[3];
      q.ports = r[4];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  q.n += nn;
}

// The demux record (id | kind << 32 as two dwords) of an IXG_V_TCP frame in
// local flow group `fg` (fg_id - dev_idx*512), PCB bucket `bucket`
// (tcp_to_idx), TCP flags `tflags`; src/dst raw (network order as loaded
// LE), ports host order (sport | dport << 16). The same lookup as
// bucket_line + walk_finish, kept as one body: composed from the two, the
// general RX kernels lost 2.5 % on IMIX to register allocation.
__device__ __forceinline__ void walk(const Tables& t, uint32_t fg, uint32_t bucket, uint32_t tflags, uint32_t src,
                                     uint32_t dst, uint32_t ports, uint32_t& id, uint32_t& kind) {
  bool hit = false;
  id = 0;
  kind = IXG_D_NONE;
  if (fg < t.nfg) {
    const uint32_t a = fg * IXG_PCB_BUCKETS + bucket;
    const u32x4* line = reinterpret_cast<const u32x4*>(t.bline) + 4u * a;
    const u32x4 hd = line[0], e0 = line[1], e1 = line[2], e2 = line[3];
    const uint32_t cnt = hd.x;
    if (cnt > 0u && e0.z == ports && e0.x == src && e0.y == dst) {
      hit = true;
      id = e0.w;
    } else if (cnt > 1u && e1.z == ports && e1.x == src && e1.y == dst) {
      hit = true;
      id = e1.w;
    } else if (cnt > 2u && e2.z == ports && e2.x == src && e2.y == dst) {
      hit = true;
      id = e2.w;
    } else if (cnt > 3u) {
      hit = find_list(t.active, hd.y + 3u, hd.y + cnt, ports, src, dst, id);
    }
    if (hit) {
      kind = IXG_D_ACTIVE;  // tcp_in.c:249-256
    } else if (hd.z && find_list(t.tw, hd.w, hd.w + hd.z, ports, src, dst, id)) {
      kind = IXG_D_TIMEWAIT;  // tcp_in.c:260-269
      hit = true;
    }
  }
  if (!hit) no_pcb(t, tflags, dst, ports, id, kind);
}

}  // namespace ixgwalk

#endif
