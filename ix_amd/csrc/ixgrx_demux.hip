// ixgrx_demux.hip - MI355X (gfx950) PCB demux: the step of tcp_input that
// follows the head (dp/net/tcp_in.c:233-323, 500-510), one lane per frame.
//
// Input: the frames and the 16-byte records ixg_rx_batch_dev produced for
// them. For an IXG_V_TCP record the lane reads the 4-tuple from the frame
// (IPv4 src/dst at bytes 26..33, ports at 14 + 4*ihl), then walks, in list
// order, the active list of (flow group, pcb_bucket), the flow group's
// TIME-WAIT list and the listen list, as tcp_input does. The lists are a CSR
// mirror of IX's hlists (include/ixgrx.h struct ixg_demux_tables) in HBM;
// they are small next to a batch and stay in L2 / Infinity Cache.
//
// A grid-stride loop over 64-frame chunks, three stages deep: the
// record and header bytes of chunk k+1 are loaded, the bucket lines of chunk
// k (ixgwalk::lines_issue, 4 lanes per line) are loaded, and the lookups of
// chunk k-1 are matched (their lines reach their lanes through the wave's
// LDS), so neither dependent load is waited for in the iteration that issues
// it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_demux.h"
#include "ixgrx_internal.h"
#include "ixgrx_walk.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2_a4 __attribute__((aligned(4)));

using DParams = ixg_dparams;

DEV uint32_t bswap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// what a chunk's lane carries from the load stage to the walk stage
struct Item {
  u32x4 rec;   // the ixg_rx_rec as four dwords
  u32x4 h0;    // frame bytes 12..27
  u32x4 h1;    // frame bytes 28..43
};

template <bool OFFS>
DEV uint64_t frame_off(const DParams& p, uint32_t i) {
  return OFFS ? p.off[i] : (uint64_t)i * p.stride;
}

// loads are always issued (a valid dummy address when there is nothing to
// read) so the compiler's vmcnt accounting stays exact across the pipeline
template <bool OFFS>
DEV void load_item(const DParams& p, uint32_t chunk, int lane, Item& it) {
  const uint32_t i = chunk * 64u + (uint32_t)lane;
  const bool valid = i < p.n;
  const uint32_t ic = valid ? i : 0u;
  it.rec = reinterpret_cast<const u32x4*>(p.rec)[ic];
  const uint8_t* f = p.base + frame_off<OFFS>(p, ic);
  it.h0 = *reinterpret_cast<const u32x4_a4*>(f + 12);
  it.h1 = *reinterpret_cast<const u32x4_a4*>(f + 28);
}

// a chunk's lookups in flight: lines loaded, matched an iteration later
struct Pend {
  u32x4 piece[4];  // ixgwalk::lines_issue's pieces
  uint32_t key;    // ixgwalk::lookup_key
  uint32_t src, dst, ports;
};
constexpr uint32_t kNoChunk = 0xffffffffu;

// the record and header bytes of frame i -> its lookup, bucket lines issued
template <bool OFFS>
DEV void prep_item(const DParams& p, uint32_t i, int lane, const Item& it, Pend& q) {
  const bool valid = i < p.n;
  const bool tcp = valid && ((it.rec.x >> 16) & 0xffu) == IXG_V_TCP;
  const uint32_t ng = p.nfg + p.n_out, nlines = ng * IXG_PCB_BUCKETS;
  const uint32_t fg = ixg_demux_group(it.rec.x & 0xffffu, p.fg_base, p.nfg, p.n_out);  // fgs[pkt->fg_id]
  const uint32_t bucket = it.rec.w & (IXG_PCB_BUCKETS - 1u);                          // tcp_to_idx (tcp_in.c:233)
  const uint32_t tflags = (it.rec.w >> 16) & 0xffu;
  const uint32_t ihl = (it.h0.x >> 16) & 15u;  // frame byte 14
  // src = bytes 26..29, dst = bytes 30..33 (raw, network order as loaded LE)
  q.src = (it.h0.w >> 16) | (it.h1.x << 16);
  q.dst = (it.h1.x >> 16) | (it.h1.y << 16);
  uint32_t sw = it.h1.y >> 16, dw = it.h1.z & 0xffffu;  // ports: L4 bytes 0..3 at 14 + 4*ihl
  if (tcp && ihl != 5u) {  // IP options: one more (dependent) load, rare
    const uint8_t* f = p.base + frame_off<OFFS>(p, i);
    const u32x2 v = *reinterpret_cast<const u32x2_a4*>(f + 12 + 4 * ihl);
    sw = v.x >> 16;
    dw = v.y & 0xffffu;
  }
  q.ports = bswap16(sw) | (bswap16(dw) << 16);  // tcp_in.c:230-231
  const bool look = tcp && fg < ng;
  q.key = ixgwalk::lookup_key(valid ? (tcp ? (look ? fg : ixgwalk::kGrpNone) : ixgwalk::kGrpNotTcp) : ixgwalk::kGrpNoFrame,
                              bucket, tflags);
  ixgwalk::lines_issue(p.bline, nlines, look ? fg * IXG_PCB_BUCKETS + bucket : nlines, lane, q.piece);
}

DEV ixgwalk::Tables tables(const DParams& p) {
  return ixgwalk::Tables{p.active_start, p.bline, p.active, p.tw, p.listen, p.nfg + p.n_out, p.n_listen};
}

// match chunk c's pending lookups (buf: the wave's 4 KiB of LDS); the ones
// the line cannot decide join the wave's queue sq
DEV void finish_chunk(const DParams& p, uint32_t c, const Pend& q, int lane,
                      __attribute__((address_space(3))) uint32_t* buf, ixgwalk::SlowQ& sq) {
  u32x4 ln[4];
  ixgwalk::lines_exchange(q.piece, lane, buf, ln);
  const uint32_t i = c * 64u + (uint32_t)lane;
  if ((q.key & 0x3fffu) == ixgwalk::kGrpNotTcp) reinterpret_cast<u32x2*>(p.out)[i] = u32x2{0u, (uint32_t)IXG_D_NONE};
  ixgwalk::walk_line(tables(p), sq, i, q.key, q.src, q.dst, q.ports, ln[0], ln[1], ln[2], ln[3], lane, buf,
                     reinterpret_cast<uint32_t*>(p.out), ixgwalk::Frames{nullptr, 0u});
}

template <bool OFFS>
DEV void demux_loop(const DParams& p) {
  __shared__ uint32_t sh_buf[kWaves][1024];
  const int lane = threadIdx.x & 63;
  __attribute__((address_space(3))) uint32_t* buf =
      (__attribute__((address_space(3))) uint32_t*)sh_buf[threadIdx.x >> 6];
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  uint32_t c = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  if (c >= nchunks) return;
  Item cur;
  load_item<OFFS>(p, c, lane, cur);
  Pend q;
  uint32_t cq = kNoChunk;  // the chunk whose lookups q holds
  ixgwalk::SlowQ sq;
  sq.n = 0;
  for (;;) {
    const uint32_t cn = c + nw;
    Item nxt;
    load_item<OFFS>(p, cn < nchunks ? cn : c, lane, nxt);
    if (cq != kNoChunk) finish_chunk(p, cq, q, lane, buf, sq);
    prep_item<OFFS>(p, c * 64u + (uint32_t)lane, lane, cur, q);
    cq = c;
    c = cn;
    if (c >= nchunks) break;
    cur = nxt;
  }
  finish_chunk(p, cq, q, lane, buf, sq);
  ixgwalk::slowq_flush(tables(p), sq, lane, reinterpret_cast<uint32_t*>(p.out), ixgwalk::Frames{nullptr, 0u});
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock) ixg_demux_s(DParams p) { demux_loop<false>(p); }
extern "C" __global__ void __launch_bounds__(kBlock) ixg_demux_o(DParams p) { demux_loop<true>(p); }

extern "C" int ixgrx_demux_launch(const void* params, uint32_t ncu, void* stream) {
  const DParams& p = *static_cast<const DParams*>(params);
  const uint64_t nchunks = ((uint64_t)p.n + 63u) / 64u;
  const uint64_t want = (nchunks + kWaves - 1) / kWaves;
  void (*k)(DParams) = p.off ? ixg_demux_o : ixg_demux_s;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
  // 8 resident grids' worth of blocks: 0.3265 -> 0.3169 ms over C2 against
  // one persistent grid (4x 0.3183, 16x 0.3218; round 4 same-process A/B,
  // profiles/r04/grid/)
  const uint64_t cap = (uint64_t)ncu * (uint64_t)nb * 8u;
  const uint32_t grid = (uint32_t)(want < cap ? want : cap);
  hipLaunchKernelGGL(k, dim3(grid ? grid : 1u), dim3(kBlock), 0, (hipStream_t)stream, p);
  return (int)hipGetLastError();
}
