/* ixgrx_internal.h - private structures shared by the C host library and
 * the HIP kernels (not part of the public ABI). */
#ifndef IXGRX_INTERNAL_H
#define IXGRX_INTERNAL_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_kparams {
	const uint8_t *base;
	const uint64_t *off;
	const uint16_t *len;
	struct ixg_rx_rec *out;
	uint32_t *csum;
	const uint64_t *tab;   /* 12 x 256: lo = Toeplitz, hi = CRC-32C contribution */
	const uint32_t *tab6;  /* IXG_TAB6_WORDS Toeplitz contributions of tuple bytes 12..35 (IXG_F_IPV6), or NULL */
	const uint32_t *tab32; /* tab's low words (Toeplitz), 12 x 256 */
	const uint16_t *tab16; /* tab's high words' low halves (CRC-32C; the bucket needs 9 bits), 12 x 256 */
	uint32_t stride;
	uint32_t n;
	uint32_t crc_const;
	uint32_t flags;
	uint32_t fg_base;      /* dev_idx * 512 */
	uint32_t fg_mask;      /* nb_rx_fgs - 1 */
	uint8_t *defer;        /* per 64-packet chunk: 0 = done by the fixed-shape
	                          kernel, IXG_CLS_SHORT / IXG_CLS_LONG = left for
	                          that general kernel; NULL = the long general
	                          kernel does everything */
	uint32_t *present;     /* [IXG_PRESENT_WORDS]: present[k] == epoch (k = 1, 2)
	                          iff some chunk of class k was deferred in this
	                          launch; present[0] == epoch iff the sampler (or
	                          the self-sampling short kernel) ran,
	                          and then present[3] is the launch's IXG_MODE_*;
	                          present[6] != 0: most sampled chunks are big
	                          (the long kernel walks its chunks strided) */
	uint32_t epoch;        /* per-launch stamp (never 0) */
	uint32_t force_mode;   /* IXG_MODE_* for the sampler to write instead of
	                          sampling (tests), or IXG_MODE_AUTO */
	/* fused PCB demux (ixg_rx_demux_batch_dev): dmx != NULL turns it on */
	struct ixg_demux_rec *dmx;
	const uint32_t *active_start;
	const uint32_t *bline;        /* nfg*512 bucket lines (ixgrx_walk.h) */
	const struct ixg_pcb_key *active;
	const struct ixg_pcb_key *tw;
	const struct ixg_listen_key *listen;
	uint32_t nfg;          /* the snapshot's local flow groups */
	uint32_t n_out;        /* ... and its outbound groups, after them (ixg_demux_group) */
	uint32_t n_listen;
	const uint8_t *zero;   /* IXG_ZERO_PAGE zero bytes: stand-in source for
	                          loads that must read nothing */
	/* flow director (ixg_rx_set_fdir), always present: a header of 4 u32
	 * {mask, fg = IXG_ETH_MAX_TOTAL_FG + cpu_id, 0, 0} (mask 0 = no filters)
	 * followed by mask+1 slots of 4 u32 {src, dst, sport | dport << 16 (host
	 * order), 1 = used}: open addressing, slot = ixg_fdir_hash(...) & mask,
	 * linear probing */
	const uint32_t *fdir;
	uint32_t host_mem;     /* the frames are in host memory (the asynchronous path's
	                          DIRECT mode): every load crosses the host link, so
	                          the span-staged short kernel runs one wave per chunk
	                          (latency-bound) instead of one per 64 chunks */
	uint32_t overlap;      /* fixed-stride batches: frames may run up to 64 bytes
	                          past their slot (the host paths' staging, whose
	                          skipped MAC bytes overlap the previous frame) */
	uint32_t self_sample;  /* set by ixgrx_launch for the span-staged short
	                          kernel when it runs first: it samples the
	                          launch's mode itself and publishes it */
	uint32_t long_only;    /* every frame is at least 256 bytes (the host's
	                          IXG_LF_LONG): with host_mem, the host-memory
	                          big-frame kernel takes the batch */
	/* the fused tcp_input head (ixg_rx_tcpx_batch_dev): ext != NULL turns
	 * it on, in the kernels ixgrx_tcpx_fusable accepts */
	struct ixg_tcp_ext *ext;
	uint32_t xflags;       /* IXG_TCPX_* */
	uint32_t rsvd;
};

/* the flow-director table's hash (host and device agree on it) */
#ifdef __HIPCC__
#define IXG_HD __host__ __device__
#else
#define IXG_HD
#endif
IXG_HD static inline uint32_t ixg_fdir_hash(uint32_t src, uint32_t dst, uint32_t ports)
{
	uint32_t h = src * 0x9E3779B1u ^ dst * 0x85EBCA77u ^ ports * 0xC2B2AE3Du;
	return h ^ (h >> 15) ^ (h >> 27);
}
typedef struct ixg_kparams ixg_kparams;

/* The demux snapshot's group of a record's fg_id (struct ixg_demux_tables):
 * a local flow group (fg_id - dev_idx*512 < nfg), or the outbound group of
 * CPU fg_id - IXG_ETH_MAX_TOTAL_FG (< n_out), stored after the local ones
 * (eth_input's cur_fg = fgs[pkt->fg_id], dp/net/ip.c:125, for a frame the
 * flow director steered, ethfg.c:502-505); IXG_NO_GROUP when the snapshot
 * has no such group (the lookup then goes straight to the listen list). */
#define IXG_NO_GROUP 0xfffffffeu
IXG_HD static inline uint32_t ixg_demux_group(uint32_t fg_id, uint32_t fg_base, uint32_t nfg, uint32_t n_out)
{
	if (fg_id >= IXG_ETH_MAX_TOTAL_FG)
		return fg_id - IXG_ETH_MAX_TOTAL_FG < n_out ? nfg + (fg_id - IXG_ETH_MAX_TOTAL_FG) : IXG_NO_GROUP;
	return fg_id - fg_base < nfg ? fg_id - fg_base : IXG_NO_GROUP;
}

#define IXG_ZERO_PAGE 4096u
#define IXG_PRESENT_WORDS 8u

/* deferred chunk classes: SHORT = every frame shorter than 112 bytes (the
 * whole L4 segment lies in the 96-byte prefix + one 16-byte piece, no
 * streaming), LONG = anything else */
#define IXG_CLS_SHORT 1u
#define IXG_CLS_LONG 2u
#define IXG_CLS_ANY 3u   /* a long-kernel build that takes both classes */
#define IXG_SHORT_MAX 112u

/* how a launch splits the work, chosen on the device by the sampler kernel
 * from the lengths of up to 64 evenly spread chunks (u64-offset batches and
 * strides > 64 B; coalesced fixed-stride batches are always FAST):
 * FAST  = the fixed-shape kernel first, then deferred short / long chunks;
 * SHORT = the short kernel walks every chunk, deferring long ones;
 * LONG  = the long kernel walks every chunk. */
#define IXG_MODE_FAST 0u
#define IXG_MODE_SHORT 1u
#define IXG_MODE_LONG 2u
#define IXG_MODE_AUTO 0xffffffffu

/* The IPv6-extension Toeplitz tables (ixg_kparams.tab6): the contribution
 * of each value of tuple bytes 12..35 (24 x 256 u32 = 24 KiB); tuple bytes
 * 0..11 use the IPv4 tables' Toeplitz words (the same key offsets) */
#define IXG_TAB6_FIRST 12u
#define IXG_TAB6_WORDS (24u * 256u)

/* implemented in ixgrx_kernels.hip */
/* enqueue one batch: the fixed-shape kernel (when p->defer) and the general
 * kernel; grids are sized from the device's CU count and each kernel's
 * occupancy */
int ixgrx_launch(const void *params, uint32_t ncu, void *stream);
/* enqueue the completion stamp: *flag = v (coherent pinned host memory), after
 * everything enqueued before it on the stream; flag[2..3] = the device's wall
 * clock (wall_clock64) when it ran, stored before flag[0] (flag: 16 bytes) */
int ixgrx_stamp(uint32_t *flag, uint32_t v, void *stream);
uint32_t ixgrx_kparams_size(void);
/* 1 when ixgrx_launch writes p->ext itself (the coalesced fixed-shape
 * kernel's layout in the default split, no fused demux); else the caller
 * runs the separate tcp_input-head pass after the launch */
int ixgrx_tcpx_fusable(const void *params);
uint32_t ixgrx_block(void);

#ifdef __cplusplus
}
#endif
#endif
