/* ixgrx_ctx.h - the RX context (private to the C host library: ixgrx_host.c,
 * ixgrx_async.c). */
#ifndef IXGRX_CTX_H
#define IXGRX_CTX_H

#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <stddef.h>
#include <stdint.h>

#include "../../include/ixgrx.h"
#include "ixgrx_internal.h"

/* per-launch kernel state that concurrent launches must not share: the
 * defer flags and the class stamps */
struct ixg_dstate {
	uint8_t *d_defer;    /* one flag per 64-packet chunk */
	size_t defer_cap;
	uint32_t *d_present; /* [IXG_PRESENT_WORDS] (ixg_kparams.present) */
	uint32_t epoch;      /* last launch's stamp */
	uint16_t *d_lenc;    /* [64 * defer_cap] lengths of a uniform-length run, all lenc */
	uint32_t lenc;       /* the value d_lenc holds (0: not filled) */
};

#define IXG_MAX_REGIONS 32u

/* one stage of the pipelined host path (ixg_rx_batch_mbufs): pinned
 * staging, device buffers, its own stream and defer state */
#define IXG_SLOTS 2
struct ixg_slot {
	struct ixg_dstate ds;
	hipStream_t stream;
	hipEvent_t done;
	int ready;           /* every buffer below allocated (slot_init) */
	int busy;            /* work enqueued, records not yet taken */
	uint32_t first, n;   /* the chunk of the caller's batch it holds */
	uint8_t *h_buf, *d_buf; /* one H2D image: frames | offsets | lengths (ixg_stage) */
	uint64_t *h_off;     /* gather scratch */
	uint16_t *h_len;
	struct ixg_rx_rec *h_rec, *d_rec;
};

/* A gathered run laid out for ONE host-to-device copy (ixg_stage_finish):
 * the frames [0, frames_end) with IXG_TAIL_PAD zero bytes after the last,
 * then the u64 offsets (packed runs only), then the u16 lengths. A run
 * whose frames all stage the same byte count is a fixed-stride batch (no
 * offsets): frame k at k * stride, frames running into the next slot by the
 * skipped MAC bytes and the bytes past ixg_stage_ext (at most 64), which the
 * launch is told (ixg_kparams.overlap). */
struct ixg_stage {
	size_t h2d;          /* bytes to copy */
	uint64_t base;       /* runs with in-place frames: the address offsets are
	                        relative to (0: the image itself) */
	size_t o_off, o_len; /* where the offsets / lengths start in the image */
	uint32_t stride;     /* fixed-stride run: the stride; else 0 */
	uint32_t lmin;       /* the shortest frame's length */
	uint32_t lconst;     /* fixed-stride run of equal lengths: the length, not
	                        in the image (the kernels read it from
	                        ixg_dstate.d_lenc); else 0 */
};
/* stage capacity: bytes the image needs for n frames of `span` gathered bytes */
#define IXG_STAGE_BYTES(span, n) ((((span) + 12u + IXG_TAIL_PAD + 16u) & ~(size_t)7) + (size_t)(n) * 10u)

struct ixg_ctx {
	int device;
	struct ixg_rx_cfg cfg;
	uint32_t crc_const;
	uint32_t ncu;        /* compute units: persistent grids are sized from it */
	int force_general;   /* IXG_SPLIT_GENERAL: skip the fixed-shape kernel (ixg_rx_set_split) */
	uint32_t force_mode; /* IXG_MODE_* forced by ixg_rx_set_split, or IXG_MODE_AUTO */
	struct ixg_dstate ds; /* the synchronous and device-resident paths' */
	struct ixg_slot slot[IXG_SLOTS];
	uint8_t *d_zero;     /* IXG_ZERO_PAGE bytes of zeros */
	uint64_t *d_tab;
	uint32_t *d_tab6;
	uint32_t *d_tab32;   /* d_tab split: Toeplitz words, CRC low halves */
	uint16_t *d_tab16;
	hipStream_t stream; /* for the synchronous host paths */
	/* host-path device staging (ixg_rx_batch_host, ixg_demux_batch_host) */
	uint8_t *d_frames;
	size_t d_frames_cap;
	uint64_t *d_off;
	uint16_t *d_len;
	struct ixg_rx_rec *d_out;
	uint32_t *d_csum;
	size_t d_n_cap;
	/* PCB demux tables (ixg_demux_load) */
	int demux_loaded;
	uint32_t dmx_nfg, dmx_nout, dmx_nlisten;
	uint32_t *d_astart;
	struct ixg_pcb_key *d_active, *d_tw;
	struct ixg_listen_key *d_listen;
	uint32_t *d_bline;           /* nfg*512 bucket lines of 64 B (ixgrx_walk.h) */
	struct ixg_demux_rec *d_dmx; /* host-path output staging */
	size_t d_dmx_cap;
	/* TX (ixg_tx_set_macs) */
	uint32_t *d_dmacs;           /* rows of 2 dwords */
	uint32_t n_dmac;
	uint32_t smac_lo, smac_hi;
	uint8_t *d_txbuf, *d_txout;  /* host-path staging */
	size_t d_txbuf_cap, d_txout_cap;
	struct ixg_tx_seg *d_txsegs;
	uint16_t *d_txlen;
	size_t d_txn_cap;
	/* event emission scratch: per-chunk counts / bases */
	uint32_t *d_evbase;
	size_t evbase_cap;
	/* flow-director perfect filters (ixg_rx_set_fdir) */
	uint32_t *d_fdir;            /* header + slots (ixgrx_internal.h); never NULL */
	size_t fdir_cap;             /* slots d_fdir holds (grow-only)*/
	/* the asynchronous host path (ixgrx_async.c) */
	struct ixg_async *async;
	/* host memory registered for in-place reads (ixg_rx_register_memory):
	 * frames of mbufs inside [lo, hi - IXG_MBUF_STRIDE - IXG_TAIL_PAD] are
	 * read by the kernels where they are (device address = host + delta) */
	struct ixg_region {
		uintptr_t lo, hi;
		intptr_t delta;
	} reg[IXG_MAX_REGIONS];
	uint32_t nreg;
	/* the echo replies' source addresses (ixg_rx_set_icmp_reply) */
	uint8_t icmp_mac[6];
	uint32_t icmp_host;
};

/* The asynchronous path's echo-request candidates of one batch
 * (IXG_ASYNC_ICMP_REFLECT): record index and the frame's device address in
 * its registered mbuf, both in pinned host memory the kernel reads. */
struct ixg_icmp_items {
	uint32_t n;
	const uint32_t *idx;
	const uint64_t *addr;
};


#define HIPCHK(x)                       \
	do {                            \
		if ((x) != hipSuccess)  \
			return -EIO;    \
	} while (0)

/* library-internal functions: not exported from libixgrx.so */
#define IXG_INTERNAL __attribute__((visibility("hidden")))

/* ixgrx_host.c; lflags: IXG_LF_* */
#define IXG_LF_OVERLAP 1u /* fixed stride, frames overlap the next slot (ixg_kparams.overlap) */
#define IXG_LF_HOST 2u    /* frames in host memory (ixg_kparams.host_mem) */
#define IXG_LF_LONG 4u    /* every frame long: the general kernel alone, no short-kernel pass */
/* a staged run whose frames are all at least this long goes to the general
 * kernel alone (IXG_LF_LONG): no chunk of it can be short, so the short
 * kernel's pass would only defer every chunk */
#ifndef IXG_LONG_ONLY_LEN
#define IXG_LONG_ONLY_LEN 256u /* >= 96: the host-memory big-frame kernel reads every prefix unmasked */
#endif
IXG_INTERNAL int ixg_launch_ds(struct ixg_ctx *c, struct ixg_dstate *ds, const uint8_t *base, const uint64_t *off,
		  const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out, uint32_t *csum,
		  struct ixg_demux_rec *dmx, uint32_t lflags, hipStream_t s);
/* ixg_launch_ds with the tcp_input head (ext != NULL: ixg_rx_tcpx_batch_dev) */
/* the echo replies of ixg_rx_icmp_batch_dev (CFG.mac, CFG.host_addr in host order) */
struct ixg_icmp_fuse {
	uint8_t mac[6];
	uint32_t host_addr;
};
IXG_INTERNAL int ixg_launch_x(struct ixg_ctx *c, struct ixg_dstate *ds, const uint8_t *base, const uint64_t *off,
			      const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out, uint32_t *csum,
			      struct ixg_demux_rec *dmx, struct ixg_tcp_ext *ext, uint32_t xflags, uint32_t lflags,
			      const struct ixg_icmp_fuse *ic, hipStream_t s);
IXG_INTERNAL void ixg_dstate_free(struct ixg_dstate *ds);
/* the per-chunk defer flags for batches of up to nchunks chunks (grown, never
 * shrunk; growing frees the old buffer, which waits for the device) */
IXG_INTERNAL int ixg_dstate_reserve(struct ixg_dstate *ds, size_t nchunks);

/* The bytes of a frame the path can read: [0, ixg_stage_ext(f, L)). For an
 * IPv4 frame (ethertype 0x0800, version 4) nothing past
 * max(14 + ip_len, l4 + 20), l4 = 14 + 4 ihl, is read by any check or sum:
 * ip_input's checks read the header (dp/net/ip.c:63-87), the L4 sums and
 * tcp_input / udp_input / icmp_input stop at the IP total length
 * (dp/lwip/misc.c:57-67, dp/net/udp.c:53-60, dp/net/icmp.c:78-92), and the
 * NIC's RSS reads the ports at l4 (a TCP header's 20 bytes cover the doff and
 * flags a record reports even for a short segment). The Ethernet pad past
 * 14 + ip_len (C2's 64-B frames: 6 bytes) is therefore not staged. Other
 * frames (ARP, IPv6, anything dropped on the ethertype): all L bytes. */
static inline size_t ixg_stage_ext(const uint8_t *f, size_t L)
{
	if (L < 34 || f[12] != 0x08 || f[13] != 0x00 || (f[14] >> 4) != 4)
		return L;
	size_t e = 14u + (((size_t)f[16] << 8) | f[17]);
	const size_t h = 14u + 4u * (size_t)(f[14] & 15u) + 20u;
	if (e < h)
		e = h;
	return e < L ? e : L;
}

/* The IX-layout gather both host paths use: frames out of mbufs (len =
 * size_t at +0, data at +64, inc/ix/mbuf.h:73-90) into staging, the MAC
 * addresses (bytes 0..11, which nothing on the path reads) skipped. Frame k
 * of the run gets the 4-aligned offset pos[k] and its bytes [12, E) land at
 * frames + pos[k] + 12, E = ixg_stage_ext(frame, L); pos[k+1] = pos[k] +
 * round4(max(E, 12) - 12), so a frame's bytes 0..11 overlap its
 * predecessor's tail, and its bytes [E, L), which nothing reads, are the
 * next frame's. Writes n offsets and lengths, returns the staged span (pos
 * of the frame after the last) and raises *hi to the end of the furthest
 * frame (pos[k] + L): the image's readable bytes must reach it. */
IXG_INTERNAL size_t ixg_gather_mbufs(uint8_t *frames, size_t pos0, void *const *mbufs, uint32_t n, uint32_t avail,
				     uint64_t *off, uint16_t *len, size_t *hi);

/* How many mbufs ahead the gathers prefetch (the header line with mbuf->len
 * and the frame's first line): `avail` (>= n) is how many valid pointers
 * mbufs[] holds, so a caller gathering in short steps still prefetches into
 * the frames of its next steps. 32 measured best over 6/12/24/32/48 on 2M
 * cold mbufs. */
#define IXG_MBUF_PREFETCH 32u

/* -EINVAL when an mbuf's len exceeds IXG_MBUF_DATA_LEN (mbuf.h) */
IXG_INTERNAL int ixg_check_mbufs(void *const *mbufs, uint32_t n);

/* The asynchronous path's gather with registered regions (zero copy): a
 * frame whose mbuf lies in one of c's registered regions is not copied; its
 * off[k] is its data's device address | IXG_OFF_ABS. Other frames are
 * gathered as by ixg_gather_mbufs (off[k] = staging position). Returns the
 * staged span; *nabs counts the in-place frames and *link grows by the bytes
 * the kernels will read of them over the host link (their lengths, rounded
 * up to 64-byte requests). */
#define IXG_OFF_ABS (1ull << 63)
IXG_INTERNAL size_t ixg_gather_mbufs_zc(const struct ixg_ctx *c, uint8_t *frames, size_t pos, void *const *mbufs,
				       uint32_t n, uint32_t avail, uint64_t *off, uint16_t *len, size_t *hi,
				       uint32_t *nabs, size_t *link);

/* lay out the image of a gathered run (span, hi: ixg_gather_mbufs): a fixed
 * stride when the offsets are k * stride, else the u64 offsets */
IXG_INTERNAL void ixg_stage_finish(uint8_t *buf, size_t span, size_t hi, const uint64_t *off, const uint16_t *len,
				  uint32_t n, struct ixg_stage *st);
/* the same for a run with in-place frames (ixg_gather_mbufs_zc, nabs > 0):
 * the image's offsets are relative to st->base, the lowest frame address of
 * the run (staged frames: buf's device address + position). off[] is left as
 * gathered, so a launch that fails can lay the run out again. */
IXG_INTERNAL void ixg_stage_finish_abs(uint8_t *buf, size_t span, size_t hi, const uint64_t *off,
				      const uint16_t *len, uint32_t n, struct ixg_stage *st);

/* enqueue one staged image on `s`: its H2D copy, the kernels, the echo
 * reflect over `ic`'s candidates (if any), the D2H copy of the records into
 * h_rec; direct: the kernels read the pinned image and write h_rec
 * themselves (no copies). done_flag != NULL: then the completion stamp,
 * *done_flag = done_val (coherent pinned host memory), after all of it.
 * Returns -EIO when nothing that changes an mbuf was enqueued (the batch may
 * be launched again). Once the reflect is enqueued a later failure completes
 * the batch synchronously (stream wait, records, the word stored from the
 * host); if even that fails, -EPIPE: the batch must not be launched again. */
IXG_INTERNAL int ixg_stage_launch(struct ixg_ctx *c, struct ixg_dstate *ds, const struct ixg_stage *st, uint8_t *h_buf,
		     uint8_t *d_buf, uint32_t n, struct ixg_rx_rec *d_rec, struct ixg_rx_rec *h_rec, int direct,
		     const struct ixg_icmp_items *ic, uint32_t *done_flag, uint32_t done_val, hipStream_t s);

/* ixgrx_async.c */
IXG_INTERNAL void ixg_async_free(struct ixg_ctx *c);
/* launch the OPEN asynchronous batch and wait for every batch in flight
 * (their kernels read the context's device tables: ixg_rx_set_fdir) */
IXG_INTERNAL int ixg_async_quiesce(struct ixg_ctx *c);

#endif
