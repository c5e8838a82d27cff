/*
 * ixgrx.h - C ABI of the MI355X-native RX parse + checksum + flow-hash engine.
 *
 * This is the drop-in boundary for IX's receive-side per-packet transform:
 * the work that dp/net + dp/lwip do on every frame between the driver poll
 * and the TCP state machine. IX has no plugin API for this path; the two
 * seams it replaces are
 *
 *   1. the driver vtable  struct eth_rx_queue { poll, ready }
 *        (/root/reference/inc/ix/ethqueue.h:47-64), whose ixgbe implementation
 *        fills mbuf->len / mbuf->fg_id from the RX descriptor (RSS) and drops
 *        packets on the NIC checksum verdict (dp/drivers/ixgbe.c:286-376);
 *   2. the direct call  eth_input(struct eth_rx_queue *, struct mbuf *)
 *        (inc/ix/mbuf.h:232-234, dp/net/ip.c:120-141) made per packet by
 *        eth_process_recv_queue (dp/core/ethqueue.c:91-110), which runs
 *        ip_input (dp/net/ip.c:63-114), the tcp_input head
 *        (dp/lwip/misc.c:57-67, dp/net/tcp_in.c:157-241), udp_input
 *        (dp/net/udp.c:53-89) and icmp_input (dp/net/icmp.c:78-115).
 *
 * One call turns a batch of frames into one 16-byte record per frame, in
 * input order. No C++ or HIP types appear here: streams are passed as void*
 * (a hipStream_t), device buffers as plain pointers.
 *
 * Threading follows IX's per-CPU model: one context per host thread; calls on
 * one context are not thread-safe. The library never frees an input frame
 * and modifies one only when asked to: the reference rewrites TCP header
 * fields to host order in place (tcp_in.c:230-238; IXG_TCPX_INPLACE of
 * ixg_tcp_ext_batch_dev) and UDP writes an ip_tuple over the frame start
 * (udp.c:81-86; IXG_EV_UDP_TUPLE of ixg_ev_batch_dev).
 */
#ifndef IXGRX_H
#define IXGRX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IXGRX_ABI_VERSION 3

/* Constants of the reference this ABI is bit-exact against. */
#define IXG_ETH_MAX_NUM_FG 512u    /* inc/ix/ethfg.h:38 ETH_MAX_NUM_FG */
#define IXG_ETH_MAX_TOTAL_FG 8192u /* inc/ix/ethfg.h:40-41 ETH_MAX_NUM_FG * NETHDEV (16): the
                                      outbound flow groups follow, one per CPU (:135-138) */
#define IXG_PCB_BUCKETS 512u       /* inc/ix/ethfg.h:42 TCP_ACTIVE_PCBS_MAX_BUCKETS */
#define IXG_PCB_HASH_SEED 0xa36bdcbeu /* inc/lwip/lwip/tcp_impl.h:371 */
#define IXG_MBUF_HEADER_LEN 64u    /* inc/ix/mbuf.h MBUF_HEADER_LEN: data at mbuf+64 */
#define IXG_MBUF_DATA_LEN 2048u    /* inc/ix/mbuf.h MBUF_DATA_LEN */
#define IXG_MBUF_STRIDE 2112u      /* MBUF_LEN, element stride of the mbuf mempool */
#define IXG_RSS_KEY_LEN 40u

/* Bytes that must be readable past the end of the last frame of a device
 * batch (the kernels load 16-byte chunks and may run up to 15 bytes past L). */
#define IXG_TAIL_PAD 64u

/* ---- configuration -------------------------------------------------- */

/* cfg.flags */
#define IXG_F_NO_CSUM_DROP (1u << 0) /* report checksum flags but never turn a
                                        bad checksum into a DROP verdict (IX
                                        with hw_ip_checksum=0) */
#define IXG_F_IPV6 (1u << 1)         /* extension: parse IPv6 TCP/UDP instead
                                        of the reference's ethertype drop */

struct ixg_rx_cfg {
	uint8_t rss_key[IXG_RSS_KEY_LEN]; /* Toeplitz key; IX leaves the NIC/DPDK
	                                     default (dp/drivers/common.c:136-168) */
	uint16_t nb_rx_fgs; /* RETA size, power of two <= 512 (common.c:257) */
	uint16_t dev_idx;   /* fg_id = dev_idx*512 + local fg (dp/core/init.c:456-462) */
	uint32_t flags;     /* IXG_F_* */
};

/* ---- the record ------------------------------------------------------- */

/* verdict: what IX's RX path does with the frame. Deliveries are < 0x80. */
enum ixg_verdict {
	IXG_V_TCP = 0x01,       /* -> tcp_input body (tcp_in.c:243-): l4_off/l4_len
	                           = TCP payload after the doff strip (tcp_in.c:222),
	                           pcb_bucket = tcp_to_idx (tcp_in.c:233) */
	IXG_V_UDP = 0x02,       /* -> usys_udp_recv(data, len) (udp.c:88): l4_off =
	                           UDP header + 8, l4_len = udp->len (header-inclusive,
	                           as the reference reports it) */
	IXG_V_ICMP_ECHO = 0x03, /* -> icmp_reflect (icmp.c:89-92): l4_off = ICMP
	                           header, l4_len = ip_len - ihl*4 */
	IXG_V_ARP = 0x04,       /* -> arp_input (ip.c:134-135): l4_off = 14,
	                           l4_len = L - 14 */
	IXG_V_TCP6 = 0x05,      /* IXG_F_IPV6 only: IPv6 TCP, fields as IXG_V_TCP */
	IXG_V_UDP6 = 0x06,      /* IXG_F_IPV6 only: IPv6 UDP, fields as IXG_V_UDP */

	/* drops: the caller frees the mbuf (ip.c:112-113,137) */
	IXG_V_DROP_ETHERTYPE = 0x80,  /* ip.c:136-137 (IPv6, VLAN, other) */
	IXG_V_DROP_IP_SHORT = 0x81,   /* ip.c:68  L < 14 + 20 */
	IXG_V_DROP_IP_VERSION = 0x82, /* ip.c:71  version != 4 */
	IXG_V_DROP_IP_IHL = 0x83,     /* ip.c:74  ihl < 5 */
	IXG_V_DROP_IP_FRAG = 0x84,    /* ip.c:78  MF set or offset != 0 */
	IXG_V_DROP_IP_LEN = 0x85,     /* ip.c:85  ip_len < ihl*4 */
	IXG_V_DROP_IP_TRUNC = 0x86,   /* ip.c:87  14 + ip_len > L */
	IXG_V_DROP_IP_PROTO = 0x87,   /* ip.c:106 proto not TCP/UDP/ICMP */
	IXG_V_DROP_TCP_SHORT = 0x88,  /* tcp_in.c:189 l4len < 20 */
	IXG_V_DROP_TCP_HDRLEN = 0x89, /* tcp_in.c:222 doff*4 > l4len */
	IXG_V_DROP_UDP_LEN = 0x8a,    /* udp.c:59 udp->len past the frame */
	IXG_V_DROP_ICMP_SHORT = 0x8b, /* icmp.c:80 len < 8 */
	IXG_V_DROP_ICMP_CSUM = 0x8c,  /* icmp.c:82 chksum_internet != 0 */
	IXG_V_DROP_ICMP_TYPE = 0x8d,  /* icmp.c:93-108 not an echo request */
	IXG_V_DROP_CSUM_IP = 0x8e,    /* NIC IPCS&IPE (ixgbe.c:313-317) */
	IXG_V_DROP_CSUM_L4 = 0x8f,    /* NIC L4CS&TCPE (ixgbe.c:320-324) */
	IXG_V_DROP_IP6 = 0x90,        /* IXG_F_IPV6: malformed/unsupported IPv6 */
};

/* rec.flags */
#define IXG_RF_IP_CSUM_CHECKED 0x01u
#define IXG_RF_IP_CSUM_OK 0x02u
#define IXG_RF_L4_CSUM_CHECKED 0x04u
#define IXG_RF_L4_CSUM_OK 0x08u
#define IXG_RF_RSS 0x10u /* rss_hash was computed (non-fragmented IPv4 TCP/UDP) */
#define IXG_RF_FDIR 0x20u /* matched a flow-director perfect filter (ixg_rx_set_fdir): fg_id is
                             the CPU's outbound flow group, not the RSS group */
#define IXG_RF_REPLY 0x40u /* IXG_V_ICMP_ECHO on the asynchronous path with
                              IXG_ASYNC_ICMP_REFLECT: the mbuf already holds
                              the echo reply icmp_input builds (icmp.c:44-71,
                              88-91); the callee only sends it (eth_send_one) */

#define IXG_NO_BUCKET 0xffffu

struct ixg_rx_rec {
	uint16_t fg_id;      /* dev_idx*512 + (rss_hash & (nb_rx_fgs-1)) (ixgbe.c:329-335), or with
	                        IXG_RF_FDIR the outbound group ETH_MAX_TOTAL_FG + cpu_id */
	uint8_t verdict;     /* enum ixg_verdict */
	uint8_t flags;       /* IXG_RF_* */
	uint16_t l4_off;     /* payload offset from the frame start (see verdicts) */
	uint16_t l4_len;     /* payload length as the reference reports it */
	uint32_t rss_hash;   /* raw Toeplitz hash (compute_toeplitz_hash, tcp_api.c:581-604); 0 if !IXG_RF_RSS */
	uint16_t pcb_bucket; /* tcp_to_idx (tcp_impl.h:381-387) for IXG_V_TCP, else IXG_NO_BUCKET */
	uint8_t tcp_flags;   /* TCPH_FLAGS (tcp_in.c:240) for IXG_V_TCP/TCP6, else 0 */
	uint8_t rsvd;        /* 0 */
};

/* Optional per-frame checksum residuals (debug/parity): bits 0-15 =
 * chksum_internet over the IP header, bits 16-31 = pseudo-header L4
 * residual (inet_chksum_pseudo_partial). 0xffff in a half = not computed. */
typedef uint32_t ixg_csum_t;

/* ---- frames ------------------------------------------------------------ */

/* A device-resident batch. Frame i starts at base + off[i] (or base +
 * i*stride when off == NULL) and is len[i] bytes long (mbuf->len: CRC
 * stripped, ethdev.c:50). Frame starts must be 4-byte aligned. Bytes at
 * offsets >= len[i] are treated as zero. IXG_TAIL_PAD bytes past the last
 * frame must be readable. */
struct ixg_rx_frames {
	const void *base;
	const uint64_t *off; /* device array of n byte offsets, or NULL */
	const uint16_t *len; /* device array of n frame lengths */
	uint32_t stride;     /* used when off == NULL; multiple of 4 */
	uint32_t rsvd;
};

/* ---- entry points ---------------------------------------------------- */

/* Create a context on HIP device `device`. 0 or -errno. */
int ixg_rx_init(const struct ixg_rx_cfg *cfg, int device, void **ctx);
void ixg_rx_fini(void *ctx);

/* Device-resident batch: records into device memory `d_out` (n entries),
 * optional residuals into `d_csum` (n entries or NULL), enqueued on `stream`
 * (a hipStream_t, NULL = default stream). Asynchronous. 0 or -errno. */
int ixg_rx_batch_dev(void *ctx, const struct ixg_rx_frames *frames, uint32_t n,
		     struct ixg_rx_rec *d_out, ixg_csum_t *d_csum, void *stream);

/* Host batch in IX's own layout: n mbuf pointers (len = size_t at +0, frame
 * data at +64, inc/ix/mbuf.h:73-90). Frames are gathered into pinned
 * staging without their MAC addresses (bytes 0..11, which nothing on the
 * path reads), copied to the device as one image per chunk, processed, and
 * the records copied back to host `out`. Synchronous (pipelined over two
 * stages for large batches). 0 or -errno. */
int ixg_rx_batch_mbufs(void *ctx, void *const *mbufs, uint32_t n, struct ixg_rx_rec *out);

/* ---- the asynchronous host path: IX's run loop never waits on the GPU ---- */

/* IX hands at most eth_rx_max_batch (64) frames per sys_bpoll iteration to
 * eth_input (dp/core/ethqueue.c:71,117-149), then runs timers and TX
 * (dp/core/syscall.c:187-196). These calls replace that per-packet loop
 * without a GPU round trip per iteration: submit gathers a CPU's frames of
 * many iterations into one staged batch (pinned memory, MAC bytes skipped),
 * which is launched when it is full or its oldest frame has waited
 * max_wait_us; poll returns finished records, with their mbufs, in the order
 * the frames were submitted. Neither call waits on the GPU (poll only with
 * wait != 0). One context per CPU, as everywhere in this ABI. */
struct ixg_rx_async_cfg {
	uint32_t batch_frames; /* launch a batch once it holds this many frames */
	uint32_t batch_bytes;  /* ... or this many frame bytes (>= 4096) */
	uint32_t max_wait_us;  /* ... or its oldest frame has waited this long
	                          (checked on every submit and poll) */
	uint32_t depth;        /* batches in the ring: in flight or not yet
	                          polled, 1..IXG_ASYNC_MAX_DEPTH */
	uint32_t flags;        /* IXG_ASYNC_* */
};
#define IXG_ASYNC_DIRECT (1u << 0) /* the kernels read the pinned staging and
                                      write the pinned records themselves
                                      over the host link: no copies */
#define IXG_ASYNC_ICMP_REFLECT (1u << 1) /* echo requests whose mbufs lie in a
                                      registered region (ixg_rx_register_memory)
                                      are turned into their replies in the
                                      mbuf on the device, after the parse and
                                      before poll returns them: the record
                                      carries IXG_RF_REPLY. The reply's MAC and
                                      address: ixg_rx_set_icmp_reply */
#define IXG_ASYNC_MAX_DEPTH 16u
#define IXG_ASYNC_DEF_FRAMES 16384u
#define IXG_ASYNC_DEF_BYTES (512u << 10)
#define IXG_ASYNC_DEF_WAIT_US 50u
#define IXG_ASYNC_DEF_DEPTH 2u
#define IXG_ASYNC_DEF_FLAGS IXG_ASYNC_DIRECT

/* Configure (or re-configure, with nothing pending) the context's
 * asynchronous path; cfg NULL = the defaults above. Optional: the first
 * submit applies the defaults. 0 or -errno (-EBUSY: frames pending). */
int ixg_rx_async_init(void *ctx, const struct ixg_rx_async_cfg *cfg);

/* Take n mbufs (len @0, data @+64; at most 2048 data bytes each) into the
 * open batch, launching batches as they fill. Returns the number accepted
 * (< n when every batch of the ring is in flight or unpolled: poll, then
 * submit the rest; the caller keeps those mbufs, as IX keeps frames queued
 * on its RX queue) or -errno. The library keeps the mbuf pointers until poll
 * returns them and never writes to or frees an mbuf. A launch that fails
 * after frames of this call were accepted does not undo them: the call
 * returns the count, the frames stay in the open batch (launched again by a
 * later submit, flush or poll), and the next submit, poll or flush returns
 * the launch's -errno once. */
int ixg_rx_submit_mbufs(void *ctx, void *const *mbufs, uint32_t n);

/* Launch the open batch now (e.g. before idling). 0 or -errno. */
int ixg_rx_flush(void *ctx);

/* Up to max finished frames, oldest first: mbufs[i] as submitted and its
 * record recs[i]. wait = 0: never blocks; wait != 0: launches the open batch
 * and blocks until at least one record is ready (returns 0 at once when
 * nothing is pending). Returns the count or -errno. */
int ixg_rx_poll(void *ctx, void **mbufs, struct ixg_rx_rec *recs, uint32_t max, int wait);

/* Frames submitted and not yet returned by poll, or -errno. */
int ixg_rx_async_pending(void *ctx);

/* The source addresses of the echo replies IXG_ASYNC_ICMP_REFLECT builds:
 * CFG.mac and CFG.host_addr (host order, as IX's cfg holds it; icmp.c:50-55).
 * Applies to batches launched after the call. 0 or -errno. Replaces, on the
 * asynchronous path, the per-packet icmp_reflect call of icmp_input
 * (dp/net/icmp.c:88-92): ixg_icmp_reflect_dev's kernel over the batch's echo
 * requests, the frames read and rewritten in their mbufs. */
int ixg_rx_set_icmp_reply(void *ctx, const uint8_t mac[6], uint32_t host_addr);

/* Where a context's asynchronous path spends its host time (cumulative since
 * ixg_rx_async_init or the last reset; for tuning IX's loop, e.g. the thread
 * count or the batch size). Times are host nanoseconds measured with the TSC
 * inside the calls. */
struct ixg_rx_async_stats {
	uint64_t frames_submitted; /* accepted by submit */
	uint64_t frames_returned;  /* handed back by poll */
	uint64_t frames_refused;   /* offered to submit, not accepted (every batch busy) */
	uint64_t submit_calls, poll_calls;
	uint64_t batches;          /* launched */
	uint64_t batches_by_time;  /* ... of which before they were full (max_wait_us passed, flush, poll with wait) */
	uint64_t gather_ns;        /* submit: copying frames into the pinned staging */
	uint64_t launch_ns;        /* enqueuing batches: copies, kernels, completion stamp */
	uint64_t poll_ns;          /* poll: completion checks and copying records out */
	uint64_t wait_ns;          /* poll with wait != 0: blocked on the GPU */
	uint64_t launch_max_ns;    /* the longest single batch launch */
	uint64_t image_bytes;      /* staged images of the launched batches: frame bytes, offsets,
	                              lengths (what the kernels or the copies read over the link) */
	uint64_t inplace_bytes;    /* in-place (zero-copy) frames of the launched batches, in
	                              64-B requests */
	uint64_t frames_launched;  /* frames of the launched batches */
	/* The batch whose first frame waited longest from its gather to the poll
	 * that returned its last frame (the worst frame latency of the window),
	 * split where the time went: open = first frame gathered -> batch
	 * launched; gpu = launched -> the completion stamp ran on the device (its
	 * wall clock, calibrated to CLOCK_MONOTONIC at ixg_rx_async_init; 0 when
	 * unknown); visible = stamp ran -> the library saw the completion word
	 * (the thread was not polling, or was asleep in the wait); returned =
	 * seen -> the last frame handed back by poll. open + gpu + visible +
	 * returned = total. wait: time poll(wait) blocked on this batch; outside:
	 * the longest interval between two calls into the library while the batch
	 * was pending (the caller's own work, or the thread off its CPU).
	 * naps / nap_max: the naps poll(wait) took on it and the longest one (a
	 * nap asks for 10 us: one of milliseconds is the thread off its CPU, many
	 * short ones a completion word that was not there yet). */
	uint64_t worst_total_ns, worst_open_ns, worst_gpu_ns, worst_visible_ns, worst_returned_ns;
	uint64_t worst_wait_ns, worst_outside_ns;
	uint64_t worst_naps, worst_nap_max_ns;
	uint64_t nap_max_ns;       /* the longest single nap of poll(wait) in the window */
};
/* Copy the counters to *out (may be NULL) and, reset != 0, zero them. 0 or -errno. */
int ixg_rx_async_stats(void *ctx, struct ixg_rx_async_stats *out, int reset);

/* Zero copy: make host memory that holds mbufs (IX's mbuf mempool, its 2 MB
 * pages, dp/core/mempool.c:198-243) readable by the kernels (page-locked and
 * mapped, hipHostRegister). With IXG_ASYNC_DIRECT, a submitted frame of at
 * least IXG_ZC_MIN_LEN bytes whose whole mbuf plus IXG_TAIL_PAD bytes lies
 * inside a registered region is then not gathered: the kernels read it where
 * it is, over the host link, and the CPU only stages its pointer and length.
 * Shorter frames, and frames outside every region, are gathered as before
 * (a short frame costs the CPU a few ns to copy, while the kernels' reads
 * of it in place cost host-link requests: DESIGN.md 5). Up to 32 regions per context, none overlapping; they
 * stay registered until ixg_rx_unregister_memory (-EBUSY while frames are
 * pending) or ixg_rx_fini. 0 or -errno. */
#define IXG_ZC_MIN_LEN 256u
int ixg_rx_register_memory(void *ctx, void *base, size_t bytes);
int ixg_rx_unregister_memory(void *ctx, void *base);

/* Host batch from a packed host buffer (same layout rules as
 * ixg_rx_frames, but host pointers). Synchronous. `csum` may be NULL. */
int ixg_rx_batch_host(void *ctx, const void *frames, const uint64_t *off,
		      const uint16_t *len, uint32_t stride, uint32_t n,
		      struct ixg_rx_rec *out, ixg_csum_t *csum);

/* The RSS/PCB hash tables the kernels use (12 x 256 x u64: low word =
 * Toeplitz contribution, high word = CRC-32C contribution) and the CRC
 * constant term, built from cfg on the host. For tests. */
int ixg_rx_hash_tables(const struct ixg_rx_cfg *cfg, uint64_t *tab12x256, uint32_t *crc_const);

int ixg_abi_version(void);
const char *ixg_strerror(int err);

/* ---- flow director: the outbound connections' perfect filters ---------- */

/* One perfect filter as get_port_with_fdir installs it for an outbound
 * (bsys_tcp_connect) connection (dp/net/tcp_api.c:630-643): IPv4 TCP frames
 * from the connection's remote address/port (src) to its local address/port
 * (dst). */
struct ixg_fdir_filter {
	uint32_t src_ip;   /* raw, network byte order (frame bytes 26..29) */
	uint32_t dst_ip;   /* raw (frame bytes 30..33) */
	uint16_t src_port; /* host order */
	uint16_t dst_port; /* host order */
};

/* Replace the context's filter set (n = 0: none, the default; IX removes
 * them one by one, remove_fdir_filter tcp_api.c:606-619). A non-fragmented
 * IPv4 TCP frame whose 4-tuple equals a filter's gets the NIC's FLM status:
 * the driver sets fg_id = MBUF_INVALID_FG_ID (dp/drivers/ixgbe.c:329-330,
 * i40e.c:380-381), which eth_recv_handle_fg_transition turns into
 * outbound_fg_idx() = ETH_MAX_TOTAL_FG + cpu_id (dp/core/ethfg.c:502-505,
 * inc/ix/ethfg.h:135-138). The record carries that fg_id and IXG_RF_FDIR;
 * everything else about the frame is unchanged. cpu_id: the IX CPU the
 * filters steer to (the queue of the CPU that connected). The table lives in
 * device memory and the kernels read it at run time, so a launch captured in
 * a HIP graph sees the current filters, unless the set grew past every
 * earlier one (the table then moves: capture again). Before it writes the
 * table the call waits for every launch the library made for this context:
 * its own stream, the pipelined mbuf path, and the asynchronous ring, whose
 * open batch it launches first, so frames submitted before the call are
 * matched against the filters in force when they were submitted. The
 * caller's own launches on its streams (ixg_rx_batch_dev and graphs) it
 * cannot see: finish those first. 0 or -errno. */
int ixg_rx_set_fdir(void *ctx, const struct ixg_fdir_filter *filters, uint32_t n, uint16_t cpu_id);

/* How the context's RX launches divide a batch between the kernels
 * (DESIGN.md 4.1). AUTO, the default, is the only setting a drop-in needs:
 * the others exist so tests can pin every kernel against the same oracle
 * (each gives bit-identical records, only slower on some layouts). Nothing
 * else (no environment variable) changes the launch plan. */
enum ixg_split {
	IXG_SPLIT_AUTO = 0,    /* mode sampled on the device / coalesced fixed-shape first */
	IXG_SPLIT_FAST = 1,    /* fixed-shape kernel first, deferred chunks after */
	IXG_SPLIT_SHORT = 2,   /* short kernel walks every chunk, defers long ones */
	IXG_SPLIT_LONG = 3,    /* long kernel walks every chunk */
	IXG_SPLIT_GENERAL = 4, /* long kernel alone, no defer flags */
};
/* 0 or -EINVAL. Applies to the context's later launches. */
int ixg_rx_set_split(void *ctx, uint32_t split);

/* How the context's last device-resident or host launch (ixg_rx_batch_dev,
 * ixg_rx_batch_host) split its batch, as the device decided it (DESIGN.md
 * 4.1): info[0] = IXG_MODE_* (0 fast, 1 short, 2 long; 0xffffffff when no
 * sampler ran: coalesced fixed-stride batches, always fast), info[1] = 1
 * when most sampled chunks were big (the long kernel then walks its chunks
 * strided), info[2] = 1 when the sampling kernel ran. For tuning and tests;
 * the caller finishes the launch first (this call synchronizes only the
 * context's own stream). 0 or -errno. */
int ixg_rx_launch_info(void *ctx, uint32_t info[3]);

/* ---- host-side dispatch: the eth_input replacement ------------------- */

/* Callbacks a run-to-completion loop supplies; each receives the mbuf and
 * its record. `drop` frees (mbuf_free). Mirrors the callees of eth_input /
 * ip_input (ip.c:92-110,132-137) and of the tcp_input head. */
struct ixg_rx_ops {
	void (*tcp)(void *user, void *mbuf, const struct ixg_rx_rec *rec);
	void (*udp)(void *user, void *mbuf, const struct ixg_rx_rec *rec);
	void (*icmp_echo)(void *user, void *mbuf, const struct ixg_rx_rec *rec);
	void (*arp)(void *user, void *mbuf, const struct ixg_rx_rec *rec);
	void (*drop)(void *user, void *mbuf, const struct ixg_rx_rec *rec);
};

/* Dispatch n records in input order; returns the number delivered
 * (non-drop). Replaces the per-packet eth_input loop of eth_process_recv
 * (dp/core/ethqueue.c:117-149). */
uint32_t ixg_rx_dispatch(void *const *mbufs, const struct ixg_rx_rec *recs, uint32_t n,
			 const struct ixg_rx_ops *ops, void *user);

/* ---- the rest of the tcp_input head: seqno/ackno/wnd/tcplen ------------- */

/* What tcp_input computes for a segment after the doff strip and before the
 * PCB lookup (dp/net/tcp_in.c:230-241): the header fields converted to host
 * order, kept in its LWIP_Context, and tcplen. One per frame, in input order;
 * all zero unless the record's verdict is IXG_V_TCP (or IXG_V_TCP6 under
 * IXG_F_IPV6, the same conversions at L4 offset 54). */
struct ixg_tcp_ext {
	uint32_t seqno;    /* ntohl(tcphdr->seqno) (tcp_in.c:236) */
	uint32_t ackno;    /* ntohl(tcphdr->ackno) (:237) */
	uint16_t wnd;      /* ntohs(tcphdr->wnd) (:238) */
	uint16_t tcplen;   /* p->tot_len after the strip + 1 if FIN or SYN (:241), u16 as lwIP keeps it */
	uint16_t src_port; /* ntohs(tcphdr->src): the remote port (:230) */
	uint16_t dst_port; /* ntohs(tcphdr->dest): the local port (:231) */
};

/* flags of ixg_tcp_ext_batch_dev */
#define IXG_TCPX_INPLACE (1u << 0) /* also rewrite each such segment's header as
                                      tcp_input leaves it: src, dest, seqno,
                                      ackno and wnd in host order, in place
                                      (tcp_in.c:230-238), so the unmodified
                                      rest of tcp_input (tcp_process,
                                      tcp_receive) can read the frame */

/* Device-resident: frames (as for ixg_rx_batch_dev; with IXG_TCPX_INPLACE
 * writable) and the records ixg_rx_batch_dev produced for them; one
 * ixg_tcp_ext per frame into d_ext. Asynchronous on `stream`. 0 or -errno. */
int ixg_tcp_ext_batch_dev(void *ctx, const struct ixg_rx_frames *frames, const struct ixg_rx_rec *d_rec,
			  uint32_t n, struct ixg_tcp_ext *d_ext, uint32_t flags, void *stream);

/* RX and the tcp_input head in one pass: d_out as ixg_rx_batch_dev, d_ext
 * (and, with IXG_TCPX_INPLACE, the frames) as ixg_tcp_ext_batch_dev over
 * those records. For a coalesced fixed-stride batch (stride <= 64 B, a
 * 16-byte aligned base: 64-byte frames) the RX kernel writes each
 * ixg_tcp_ext from the header bytes it has just parsed, with no second read
 * of the frames or the records; other layouts run the two passes on
 * `stream`. Replaces the pair ixg_rx_batch_dev + ixg_tcp_ext_batch_dev
 * (dp/net/ip.c:120-141 through dp/net/tcp_in.c:230-241 per frame).
 * Asynchronous on `stream`. 0 or -errno. */
int ixg_rx_tcpx_batch_dev(void *ctx, const struct ixg_rx_frames *frames, uint32_t n, struct ixg_rx_rec *d_out,
			  struct ixg_tcp_ext *d_ext, uint32_t flags, void *stream);

/* ---- ICMP echo reflect ---------------------------------------------------- */

/* For every frame whose record is IXG_V_ICMP_ECHO, rewrite the frame in place
 * into the echo reply icmp_input leaves in the mbuf for eth_send_one
 * (dp/net/icmp.c:44-71,88-91): ICMP type ICMP_ECHOREPLY; Ethernet destination
 * = the old source, source = mac (CFG.mac); IP destination = the old source,
 * source = hton32(host_addr) (CFG.host_addr, host order as IX's cfg holds
 * it); the ICMP checksum = chksum_internet over the record's l4_len bytes.
 * As in the reference, the IP header checksum is left as it was (the reply
 * goes out with ol_flags 0): it stays valid when host_addr is the request's
 * destination. Other frames are untouched. Device-resident frames (any
 * alignment) and the records ixg_rx_batch_dev produced for them (8-byte
 * aligned); asynchronous on `stream`. 0 or -errno. */
int ixg_icmp_reflect_dev(void *ctx, const struct ixg_rx_frames *frames, const struct ixg_rx_rec *d_rec, uint32_t n,
			 const uint8_t mac[6], uint32_t host_addr, void *stream);

/* ixg_rx_batch_dev and then ixg_icmp_reflect_dev in one call: the records
 * of the frames, and every IXG_V_ICMP_ECHO frame rewritten in place into its
 * echo reply as above, its record carrying IXG_RF_REPLY (eth_input ->
 * icmp_input -> icmp_reflect per echo request, dp/net/ip.c:120-141,
 * dp/net/icmp.c:44-71,88-92). Arguments as ixg_rx_batch_dev plus the
 * reply's mac / host_addr. Asynchronous on `stream`. 0 or -errno. */
int ixg_rx_icmp_batch_dev(void *ctx, const struct ixg_rx_frames *frames, uint32_t n, struct ixg_rx_rec *d_out,
			  const uint8_t mac[6], uint32_t host_addr, void *stream);

/* ---- PCB demux: the tcp_input step after the head ---- */

/* For each IXG_V_TCP record, find the PCB the segment belongs to, exactly as
 * tcp_input does (dp/net/tcp_in.c:233-323, 500-510): the active list of the
 * frame's flow group at bucket tcp_to_idx (tcp_in.c:249,
 * tcp_input_find_list :122-143), then the flow group's TIME-WAIT list
 * (:260), then the per-CPU listen list (:273-304), else a RST. The tables
 * are a snapshot of IX's lists, mirrored to the device by ixg_demux_load;
 * entries keep list order, so "first match" is the reference's match. */

/* One PCB as tcp_input_find_list compares it (tcp_in.c:134-138). */
struct ixg_pcb_key {
	uint32_t remote_ip;   /* pcb->remote_ip.addr: raw, network byte order */
	uint32_t local_ip;    /* pcb->local_ip.addr */
	uint16_t remote_port; /* pcb->remote_port: host order */
	uint16_t local_port;  /* pcb->local_port */
	uint32_t id;          /* the caller's handle for the PCB (returned as is) */
};

/* One LISTEN pcb as the listen walk compares it (tcp_in.c:274-303). */
struct ixg_listen_key {
	uint32_t local_ip;   /* lpcb->local_ip.addr; 0 = IP_ADDR_ANY */
	uint16_t local_port; /* host order */
	uint16_t rsvd;
	uint32_t id;
	uint32_t rsvd2;
};

/* A snapshot of one context's demux lists (host arrays; ixg_demux_load copies
 * them). Groups are the context's local flow groups (fg_id - dev_idx*512,
 * g < nfg) followed by n_out outbound groups: the per-CPU groups
 * ETH_MAX_TOTAL_FG + cpu_id (inc/ix/ethfg.h:135-138) whose active and
 * TIME-WAIT lists hold the connections the CPU opened (bsys_tcp_connect,
 * dp/net/tcp_api.c:694), whose frames the flow director steers there
 * (ixg_rx_set_fdir): group nfg + cpu_id for cpu_id < n_out. */
#define IXG_MAX_OUTBOUND 1024u
struct ixg_demux_tables {
	uint32_t nfg;                       /* local flow groups in the snapshot (<= 512) */
	uint32_t n_listen;
	const uint32_t *active_start;       /* (nfg+n_out)*512 + 1 offsets: entries of
	                                       fgs[g]->active_tbl[b].pcbs (ethfg.h:83) in
	                                       list order are active[active_start[g*512+b] ..
	                                       active_start[g*512+b+1]) */
	const struct ixg_pcb_key *active;
	const uint32_t *tw_start;           /* nfg + n_out + 1 offsets into tw[]: fgs[g]->tw_pcbs */
	const struct ixg_pcb_key *tw;
	const struct ixg_listen_key *listen; /* percpu tcp_cpu_lists.listen_pcbs, list order */
	uint32_t n_out;                     /* outbound groups (CPUs) in the snapshot (<= IXG_MAX_OUTBOUND) */
	uint32_t rsvd;
};

/* demux.kind */
enum ixg_demux_kind {
	IXG_D_NONE = 0,     /* not an IXG_V_TCP record */
	IXG_D_ACTIVE = 1,   /* tcp_in.c:249-256: tcp_process on pcb `id` */
	IXG_D_TIMEWAIT = 2, /* tcp_in.c:260-269: tcp_timewait_input on pcb `id` */
	IXG_D_LISTEN = 3,   /* tcp_in.c:317-323: tcp_listen_input on lpcb `id`. As in the
	                       reference's hlist walk, a non-empty listen list with no
	                       port/address match yields its LAST entry (the loop
	                       variable keeps the last node when no `break` ran) */
	IXG_D_RESET = 4,    /* tcp_in.c:500-507: no PCB, tcp_rst sent */
	IXG_D_DROP = 5,     /* tcp_in.c:503,509: no PCB, the segment carries RST: freed */
};

struct ixg_demux_rec {
	uint32_t id;  /* the matched entry's id (0 for NONE/RESET/DROP) */
	uint8_t kind; /* enum ixg_demux_kind */
	uint8_t rsvd[3];
};

/* Load (replace) the context's demux tables. 0 or -errno. */
int ixg_demux_load(void *ctx, const struct ixg_demux_tables *t);

/* Device-resident: frames (as for ixg_rx_batch_dev) and the records that
 * ixg_rx_batch_dev produced for them, in HBM; demux records into d_out.
 * Asynchronous on `stream`. 0 or -errno (-ENOENT: no tables loaded). */
int ixg_demux_batch_dev(void *ctx, const struct ixg_rx_frames *frames, const struct ixg_rx_rec *d_rec,
			uint32_t n, struct ixg_demux_rec *d_out, void *stream);

/* RX and demux in one pass (the demux fused into the RX kernels: the lookup
 * runs from the parse state, with no second pass over frames or records):
 * d_out as ixg_rx_batch_dev, d_dmx as ixg_demux_batch_dev. Asynchronous on
 * `stream`. 0 or -errno (-ENOENT: no tables loaded). */
int ixg_rx_demux_batch_dev(void *ctx, const struct ixg_rx_frames *frames, uint32_t n, struct ixg_rx_rec *d_out,
			   struct ixg_demux_rec *d_dmx, void *stream);

/* Host variant of ixg_demux_batch_dev (copies in, runs, copies out). */
int ixg_demux_batch_host(void *ctx, const void *frames, const uint64_t *off, const uint16_t *len,
			 uint32_t stride, uint32_t n, const struct ixg_rx_rec *rec,
			 struct ixg_demux_rec *out);

/* ---- TX: header build + checksums, the mirror transform ---- */

/* One outgoing segment, as the reference's two TX paths receive it:
 *  - proto 6: tcp_output_packet (dp/net/tcp_api.c:773-826) gets a pbuf chain
 *    holding the TCP header lwIP built + payload (seg bytes here), and the
 *    pcb's local/remote IP, tos and ttl;
 *  - proto 17: udp_output (dp/net/udp.c:102-130) gets the payload (seg bytes)
 *    and an ip_tuple {dst_ip, src_port, dst_port}; the source IP is
 *    CFG.host_addr, tos 0 and ttl 64 (ip_setup_header, dp/net/net.h:65-78).
 * The Ethernet header is ip_send_one's (dp/net/ip.c:192-219): dhost = the
 * ARP entry of the next hop (here dmac[dmac_idx] of the MAC table), shost =
 * CFG.mac, type 0x0800. */
struct ixg_tx_seg {
	uint64_t seg_off;   /* device byte offset of the segment bytes, 4-aligned */
	uint64_t out_off;   /* frame start in the output buffer, 16-aligned */
	uint32_t src_ip;    /* raw, network byte order (pcb->local_ip.addr) */
	uint32_t dst_ip;    /* raw, network byte order */
	uint16_t seg_len;   /* TCP: header + payload; UDP: payload (<= 1472) */
	uint16_t src_port;  /* UDP: host order (ip_tuple); TCP: unused */
	uint16_t dst_port;  /* UDP: host order; TCP: unused */
	uint8_t proto;      /* 6 or 17 */
	uint8_t tos;
	uint8_t ttl;
	uint8_t rsvd;
	uint16_t dmac_idx;  /* index into the context's destination MAC table */
	uint32_t rsvd2;
};

/* flags of ixg_tx_batch_dev */
#define IXG_TX_OFFLOAD (1u << 0) /* leave a TCP frame's checksums as IX leaves
                                    them for the NIC (PKT_TX_IP_CKSUM |
                                    PKT_TX_TCP_CKSUM, tcp_api.c:815-817): IP
                                    checksum 0 and the TCP checksum field =
                                    inet_chksum_pseudo's seed
                                    (dp/lwip/inet_chksum.c:323-360). Default:
                                    both computed, as the NIC puts them on
                                    the wire. UDP is the same in both: IP
                                    checksum by chksum_internet (udp.c:121),
                                    UDP checksum 0 (udp.c:127). */

/* The MAC addresses: src = CFG.mac, dmacs = n_dmac next-hop addresses (the
 * ARP table rows segments refer to by dmac_idx). 0 or -errno. */
int ixg_tx_set_macs(void *ctx, const uint8_t src_mac[6], const uint8_t *dmacs, uint32_t n_dmac);

/* Build n frames: frame i = Ethernet + IPv4 (+ UDP) header + the segment
 * bytes, written at out + segs[i].out_off, with out_len[i] = its length
 * (14 + 20 + seg_len, + 8 for UDP). Bytes from the frame end up to the next
 * 16-byte boundary may be overwritten. segs, seg_buf, out, out_len are
 * device pointers. Asynchronous on `stream`. 0 or -errno (-EINVAL: bad
 * proto/length/alignment is reported per frame as out_len 0). */
int ixg_tx_batch_dev(void *ctx, const void *seg_buf, const struct ixg_tx_seg *segs, uint32_t n, void *out,
		     uint16_t *out_len, uint32_t flags, void *stream);

/* Host variant: host seg_buf (seg_buf_len bytes), host segs, host out
 * (large enough for every out_off + round_up(frame, 16)), host out_len.
 * Synchronous. */
int ixg_tx_batch_host(void *ctx, const void *seg_buf, size_t seg_buf_len, const struct ixg_tx_seg *segs,
		      uint32_t n, void *out, size_t out_size, uint16_t *out_len, uint32_t flags);

/* ---- event records: the usys descriptors libix consumes ---- */

/* struct bsys_desc (inc/ix/syscall.h:101-104), 40 bytes packed */
struct ixg_bsys_desc {
	uint64_t sysnr;
	uint64_t arga, argb, argc, argd;
};
#define IXG_USYS_UDP_RECV 0u /* inc/ix/syscall.h:319 */
#define IXG_USYS_TCP_RECV 4u /* :323 */

/* What recv_a_pbuf needs of a PCB (dp/net/tcp_api.c:125-147): its index in
 * the pcb mempool (the low 48 bits of the flow handle, tcpapi_to_handle
 * :125-131) and the application's cookie. Indexed by ixg_pcb_key.id. */
struct ixg_ev_pcb {
	uint64_t pcb_idx;
	uint64_t cookie;
};

/* flags of ixg_ev_batch_dev */
#define IXG_EV_UDP_TUPLE (1u << 0) /* also write udp_input's struct ip_tuple
                                      (host-order src/dst IP and ports) over the
                                      first 12 bytes of each UDP frame, as
                                      dp/net/udp.c:81-86 does */

/* Emit, in frame order, the descriptors the reference's stack writes into the
 * per-CPU usys array for a batch (dense, as usys_next hands them out):
 *  - IXG_V_UDP: udp_input's usys_udp_recv (udp.c:88, syscall.h:360-365):
 *    {USYS_UDP_RECV, iomap(payload), udp->len, iomap(frame start: the
 *    ip_tuple), 0};
 *  - IXG_V_TCP whose demux record is IXG_D_ACTIVE with a non-empty payload:
 *    recv_a_pbuf's usys_tcp_recv (tcp_api.c:133-147, syscall.h:416-420) for
 *    the segment delivered in order as one pbuf: {USYS_TCP_RECV,
 *    (fg_id << 48) | pcb_idx, cookie, iomap(payload), payload length}. The
 *    TCP state machine (tcp_process) that decides in-order delivery stays on
 *    the host: these are the descriptors for in-order segments.
 * iomap(frame i + x) = iomap_base + frame offset of i + x (frames laid out as
 * the device batch: a mirror of the mbuf arena gives IX's
 * mempool_pagemem_to_iomap, inc/ix/mempool.h:259-263). d_dmx may be NULL (no
 * TCP events); d_frame_idx (may be NULL) receives each event's frame index.
 * *d_count (device u32) receives the number of events. Asynchronous. */
int ixg_ev_batch_dev(void *ctx, const struct ixg_rx_frames *frames, const struct ixg_rx_rec *d_rec,
		     const struct ixg_demux_rec *d_dmx, const struct ixg_ev_pcb *d_pcbs, uint32_t n_pcbs,
		     uint32_t n, uint64_t iomap_base, uint32_t flags, struct ixg_bsys_desc *d_ev,
		     uint32_t *d_frame_idx, uint32_t *d_count, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* IXGRX_H */
