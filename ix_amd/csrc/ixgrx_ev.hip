// ixgrx_ev.hip - MI355X (gfx950) event-record emission: the usys
// descriptors IX's stack writes for received data,
// produced on the device from the RX and demux records, dense and in frame
// order, so libix's event loop can consume them as they are:
//   udp_input -> usys_udp_recv  (dp/net/udp.c:81-88, inc/ix/syscall.h:360-365)
//   recv_a_pbuf -> usys_tcp_recv (dp/net/tcp_api.c:133-147, syscall.h:416-420)
// Four launches: per 64-frame chunk, count the events (ballot); per group
// of 64 chunks, one wave scans the chunk counts (bases within the group and
// the group's count); one block scans the group counts (so the output stays
// in frame order); per chunk, the event lanes put their 40-byte descriptors
// in LDS at their rank among the chunk's events (mbcnt) and the wave stores
// the chunk's contiguous run of descriptors with coalesced 8-byte stores.
// (A single block scanning every chunk count took 0.39 ms for 16M frames,
// stored lane by lane the descriptors 0.26 ms.)
//
// No MFMA: a few bytes in, 40 bytes out per event, HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_ev.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

using EParams = ixg_eparams;

struct Ev {
  bool on;
  uint32_t kind;  // 0 UDP, 1 TCP
  u32x4 rec;
  uint32_t id;
};

// which frames produce an event (include/ixgrx.h ixg_ev_batch_dev)
DEV Ev classify(const EParams& p, uint32_t i) {
  Ev e;
  const bool valid = i < p.n;
  const uint32_t ic = valid ? i : 0u;
  // non-temporal: the records and demux results are streamed through once
  // per pass (events 0.2934 -> 0.2825 ms in a same-process A/B,
  // profiles/r04/ev_nt/)
  e.rec = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p.rec) + ic);
  const uint32_t verdict = (e.rec.x >> 16) & 0xffu;
  const uint32_t plen = e.rec.y >> 16;
  u32x2 d = {0u, 0u};
  if (p.dmx) d = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p.dmx) + ic);
  e.id = d.x;
  const uint32_t dkind = d.y & 0xffu;
  const bool udp = verdict == IXG_V_UDP;
  const bool tcp = p.dmx && verdict == IXG_V_TCP && dkind == IXG_D_ACTIVE && plen > 0u && d.x < p.n_pcbs;
  e.on = valid && (udp || tcp);
  e.kind = tcp ? 1u : 0u;
  return e;
}

// a wave's k-th chunk: runs of kRunE consecutive chunks dealt out
// round-robin (kRunE = 1: grid-stride)
constexpr uint32_t kRunE = 1;
DEV uint32_t ev_chunk(uint32_t k, uint32_t nw, uint32_t nchunks) {
  const uint32_t w0 = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint64_t c64 = ((uint64_t)(k / kRunE) * nw + w0) * kRunE + k % kRunE;
  return c64 < nchunks ? (uint32_t)c64 : nchunks;
}

DEV uint32_t rank_of(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace

extern "C" __global__ void __launch_bounds__(kBlock) ixg_ev_count(EParams p) {
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  for (uint32_t k = 0, c = ev_chunk(0, nw, nchunks); c < nchunks; c = ev_chunk(++k, nw, nchunks)) {
    const Ev e = classify(p, c * 64u + (uint32_t)lane);
    const uint64_t m = __ballot(e.on);
    if (lane == 0) p.chunk_base[c] = (uint32_t)__popcll(m);
  }
}

// one wave per group of 64 chunks: the chunk counts -> bases within the
// group (exclusive scan), the group's count -> group_base
extern "C" __global__ void __launch_bounds__(kBlock) ixg_ev_group(EParams p) {
  const int lane = threadIdx.x & 63;
  const uint32_t nchunks = (p.n + 63u) >> 6, ngroups = (nchunks + 63u) >> 6;
  const uint32_t g = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= ngroups) return;
  const uint32_t c = g * 64u + (uint32_t)lane;
  const uint32_t v = c < nchunks ? p.chunk_base[c] : 0u;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += o;
  }
  if (c < nchunks) p.chunk_base[c] = incl - v;
  if (lane == 63) p.group_base[g] = incl;
}

// one block: exclusive scan of the group counts in place, total to *count
extern "C" __global__ void __launch_bounds__(1024) ixg_ev_scan(EParams p) {
  __shared__ uint32_t part[1024];
  const uint32_t nchunks = (p.n + 63u) >> 6, ngroups = (nchunks + 63u) >> 6;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ngroups + 1023u) / 1024u;
  const uint32_t b = t * per, e = b + per < ngroups ? b + per : ngroups;
  uint32_t s = 0;
  for (uint32_t k = b; k < e; k++) s += p.group_base[k];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024u; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;  // exclusive
  for (uint32_t k = b; k < e; k++) {
    const uint32_t c = p.group_base[k];
    p.group_base[k] = run;
    run += c;
  }
  if (t == 1023u) *p.count = part[1023];
}

typedef __attribute__((address_space(3))) uint64_t lds_u64;

extern "C" __global__ void __launch_bounds__(kBlock) ixg_ev_emit(EParams p) {
  __shared__ uint64_t sh[kWaves][64 * 5];
  lds_u64* buf = (lds_u64*)sh[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * kWaves;
  const uint32_t nchunks = (p.n + 63u) >> 6;
  // the chunk bases were written by the kernels before this one: scalar
  // loads through the constant address space (counted on lgkmcnt, so they
  // never wait for the records in flight)
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  uint32_t k = 0, c = ev_chunk(0, nw, nchunks);
  if (c >= nchunks) return;
  Ev e = classify(p, c * 64u + (uint32_t)lane);
  for (;;) {
    // the next chunk's records and demux records are loaded before this
    // chunk's descriptors are built (one chunk of software pipelining)
    const uint32_t cn = ev_chunk(++k, nw, nchunks);
    const Ev en = classify(p, cn * 64u + (uint32_t)lane);  // (i >= n past the end: nothing valid)
    const uint32_t i = c * 64u + (uint32_t)lane;
    const uint64_t m = __ballot(e.on);
    if (m == 0) {
      if (cn >= nchunks) break;
      c = cn;
      e = en;
      continue;
    }
    const uint32_t base = *(cu32*)(p.group_base + (c >> 6)) + *(cu32*)(p.chunk_base + c), r = rank_of(m);
    if (e.on) {
      const uint64_t foff = p.off ? p.off[i] : (uint64_t)i * p.stride;
      const uint64_t fio = p.iomap_base + foff;  // iomap(frame start)
      const uint32_t fg = e.rec.x & 0xffffu, l4_off = e.rec.y & 0xffffu, l4_len = e.rec.y >> 16;
      ixg_bsys_desc d;
      if (e.kind) {  // usys_tcp_recv(handle, cookie, iomap(payload), len)
        const ixg_ev_pcb pc = p.pcbs[e.id];
        d.sysnr = IXG_USYS_TCP_RECV;
        d.arga = ((uint64_t)fg << 48) | (pc.pcb_idx & 0xffffffffffffull);
        d.argb = pc.cookie;
        d.argc = fio + l4_off;
        d.argd = l4_len;
      } else {  // usys_udp_recv(iomap(data), udp->len, iomap(ip_tuple at the frame start))
        d.sysnr = IXG_USYS_UDP_RECV;
        d.arga = fio + l4_off;
        d.argb = l4_len;
        d.argc = fio;
        d.argd = 0;
        if (p.flags & IXG_EV_UDP_TUPLE) {
          // udp.c:81-86: {ntoh32(src), ntoh32(dst), ntoh16(sport), ntoh16(dport)}
          uint8_t* f = p.base + foff;
          const uint32_t* w = reinterpret_cast<const uint32_t*>(f + 24);  // bytes 24..31 (4-aligned)
          const uint32_t w6 = w[0], w7 = w[1], w8 = w[2];
          const uint32_t src = (w6 >> 16) | (w7 << 16), dst = (w7 >> 16) | (w8 << 16);  // raw bytes 26..33
          // the UDP header starts at l4 = l4_off - 8 = 2 mod 4: ports from the
          // aligned dwords at l4 - 2 and l4 + 2
          const uint32_t A = *reinterpret_cast<const uint32_t*>(f + l4_off - 10);
          const uint32_t B = *reinterpret_cast<const uint32_t*>(f + l4_off - 6);
          const uint32_t sport = (((A >> 16) & 0xffu) << 8) | (A >> 24);
          const uint32_t dport = ((B & 0xffu) << 8) | ((B >> 8) & 0xffu);
          uint32_t* o = reinterpret_cast<uint32_t*>(f);
          o[0] = __builtin_bswap32(src);
          o[1] = __builtin_bswap32(dst);
          o[2] = sport | (dport << 16);
        }
      }
      lds_u64* q = buf + 5 * r;
      q[0] = d.sysnr;
      q[1] = d.arga;
      q[2] = d.argb;
      q[3] = d.argc;
      q[4] = d.argd;
      if (p.frame_idx) p.frame_idx[base + r] = i;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the chunk's descriptors are one contiguous run: 8-byte pieces, lane
    // by lane (5 per descriptor, at most 5 stores per lane), non-temporal:
    // the descriptors are written once, and left dirty in the caches they
    // were paid for again by the next launch's count pass (0.2819 -> 0.2578
    // ms per launch in a same-process A/B, profiles/r05/ev_nt_store/; the
    // frame indices and chunk counts as non-temporal stores too: 0.2796;
    // count and group scan fused into one launch, a wave per 64 chunks:
    // 0.2618-0.2667 ms, slower)
    uint64_t* out = reinterpret_cast<uint64_t*>(p.ev + base);
    const uint32_t nq = 5u * (uint32_t)__popcll(m);
    for (uint32_t q = (uint32_t)lane; q < nq; q += 64u) __builtin_nontemporal_store((uint64_t)buf[q], out + q);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (cn >= nchunks) break;
    c = cn;
    e = en;
  }
}

extern "C" int ixgrx_ev_launch(const void* params, uint32_t ncu, void* stream) {
  const EParams& p = *static_cast<const EParams*>(params);
  const uint64_t nchunks = ((uint64_t)p.n + 63u) / 64u;
  const uint64_t want = (nchunks + kWaves - 1) / kWaves;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ixg_ev_emit, kBlock, 0) != hipSuccess || nb < 1) nb = 1;
  const uint64_t cap = (uint64_t)ncu * (uint64_t)nb;
  const uint32_t grid = (uint32_t)(want < cap ? want : cap);
  hipStream_t s = (hipStream_t)stream;
  const uint64_t ngroups = (nchunks + 63u) / 64u;
  hipLaunchKernelGGL(ixg_ev_count, dim3(grid ? grid : 1u), dim3(kBlock), 0, s, p);
  hipLaunchKernelGGL(ixg_ev_group, dim3((uint32_t)((ngroups + kWaves - 1) / kWaves)), dim3(kBlock), 0, s, p);
  hipLaunchKernelGGL(ixg_ev_scan, dim3(1), dim3(1024), 0, s, p);
  hipLaunchKernelGGL(ixg_ev_emit, dim3(grid ? grid : 1u), dim3(kBlock), 0, s, p);
  return (int)hipGetLastError();
}
