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
  // per active bucket one 64-byte line: {count, CSR start, 0, 0} + the first
  // three entries of the list in list order, so the common case (a short
  // bucket) is ONE dependent load instead of bounds then entries
  const uint32_t* bline;
  const ixg_pcb_key* active;
  const uint32_t* tw_start;      // nfg + 1
  const ixg_pcb_key* tw;
  const ixg_listen_key* listen;
  uint32_t nfg;  // groups in the snapshot: local, then outbound (ixg_demux_group)
  uint32_t n_listen;
};

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

// The lookup given the frame's bucket line (hd, e0..e2; ignored when fg is
// not a group of the tables): the rest of walk below. Split out so a
// caller can load the line early and finish later.
__device__ __forceinline__ void walk_finish(const Tables& t, uint32_t fg, uint32_t tflags, uint32_t src, uint32_t dst,
                                            uint32_t ports, const u32x4& hd, const u32x4& e0, const u32x4& e1,
                                            const u32x4& e2, uint32_t& id, uint32_t& kind) {
  bool hit = false;
  id = 0;
  kind = IXG_D_NONE;
  if (fg < t.nfg) {
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
    } else if (find_list(t.tw, t.tw_start[fg], t.tw_start[fg + 1], ports, src, dst, id)) {
      kind = IXG_D_TIMEWAIT;  // tcp_in.c:260-269
      hit = true;
    }
  }
  if (!hit) {
    // tcp_in.c:273-304 without SO_REUSE / LWIP_IPV6 (opt.h:1579,2016): break
    // at the first lpcb on the port whose address is the segment's
    // destination or ANY; the hlist loop variable keeps the last entry when
    // nothing breaks, so a non-empty list always yields an lpcb
    const uint32_t dport = ports >> 16;
    if (t.n_listen != 0) {
      uint32_t k = 0;
      for (; k < t.n_listen; k++) {
        const u32x4 v = reinterpret_cast<const u32x4*>(t.listen)[k];
        if ((v.y & 0xffffu) == dport && (v.x == dst || v.x == 0u)) break;
      }
      if (k == t.n_listen) k = t.n_listen - 1;
      id = reinterpret_cast<const u32x4*>(t.listen)[k].z;
      kind = IXG_D_LISTEN;  // tcp_in.c:317-323
    } else {
      kind = (tflags & 0x04u) ? IXG_D_DROP : IXG_D_RESET;  // tcp_in.c:500-510 (TCP_RST = 0x04)
      id = 0;
    }
  }
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
    } else if (find_list(t.tw, t.tw_start[fg], t.tw_start[fg + 1], ports, src, dst, id)) {
      kind = IXG_D_TIMEWAIT;  // tcp_in.c:260-269
      hit = true;
    }
  }
  if (!hit) {
    // tcp_in.c:273-304 without SO_REUSE / LWIP_IPV6 (opt.h:1579,2016): break
    // at the first lpcb on the port whose address is the segment's
    // destination or ANY; the hlist loop variable keeps the last entry when
    // nothing breaks, so a non-empty list always yields an lpcb
    const uint32_t dport = ports >> 16;
    if (t.n_listen != 0) {
      uint32_t k = 0;
      for (; k < t.n_listen; k++) {
        const u32x4 v = reinterpret_cast<const u32x4*>(t.listen)[k];
        if ((v.y & 0xffffu) == dport && (v.x == dst || v.x == 0u)) break;
      }
      if (k == t.n_listen) k = t.n_listen - 1;
      id = reinterpret_cast<const u32x4*>(t.listen)[k].z;
      kind = IXG_D_LISTEN;  // tcp_in.c:317-323
    } else {
      kind = (tflags & 0x04u) ? IXG_D_DROP : IXG_D_RESET;  // tcp_in.c:500-510 (TCP_RST = 0x04)
      id = 0;
    }
  }
}

}  // namespace ixgwalk

#endif
