/* ref_capture.h - what the reference harness observes (test infrastructure). */
#ifndef REF_CAPTURE_H
#define REF_CAPTURE_H
#include <stdint.h>

enum { REF_NONE = 0, REF_TCP, REF_UDP, REF_ARP, REF_ICMP_REFLECT };

struct ref_capture {
	int kind;        /* which callee eth_input reached (REF_NONE: none) */
	long l4_off;     /* L4 header pointer - frame start, as passed to the callee */
	uint16_t l4_len; /* tcp_input_tmp's pbuf length */
	int freed;       /* mbuf_free reached mempool_free_2 (= dropped) */
};

extern struct ref_capture ref_cap;

int ref_ix_init(void);
/* eth_recv_handle_fg_transition (dp/core/ethfg.c:502-523) on CPU `cpu`: the
 * fg_id it leaves, 0xffffffff when the frame would not be processed here */
uint32_t ref_fg_transition(uint32_t fg_id, unsigned int cpu);
void ref_eth_input(void *mbuf);
uint16_t ref_chksum_internet(const void *buf, int len);
void ref_set_host(const uint8_t mac[6], uint32_t host_addr);

uint16_t ref_pseudo_partial(const void *seg, uint16_t len, uint8_t proto, uint16_t proto_len,
			    uint32_t src_raw, uint32_t dst_raw);
uint16_t ref_pseudo6_partial(const void *seg, uint16_t len, uint8_t proto, uint16_t proto_len,
			     const void *src16, const void *dst16);
int ref_pbuf_header_rom(uint16_t len, int16_t inc, uint16_t *new_len);
int ref_tcp_to_idx(uint32_t local_raw, uint32_t remote_raw, uint16_t local_port, uint16_t remote_port);
uint32_t ref_toeplitz(const uint8_t *key, uint32_t src_raw, uint32_t dst_raw, uint16_t sport_raw,
		      uint16_t dport_raw);

/* a PCB as the demux harness hands it to ref_find_list (ref_tcpin.c) */
struct ref_pcb {
	uint32_t remote_ip, local_ip; /* raw, network order */
	uint16_t remote_port, local_port; /* host order */
};
int ref_find_list(const struct ref_pcb *pcbs, int n, uint32_t src_raw, uint32_t dst_raw, uint16_t src_port,
		  uint16_t dst_port);

/* TX: reference frame builds and the offload seed */
void ref_tx_set_macs(const uint8_t src[6], const uint8_t dst[6]);
uint32_t ref_tcp_frame(uint32_t local_raw, uint32_t remote_raw, uint8_t tos, uint8_t ttl, const void *seg,
		       uint16_t len, uint8_t *out);
uint32_t ref_udp_frame(uint32_t src_raw, uint32_t dst_raw, uint16_t sport, uint16_t dport, const void *payload,
		       uint16_t len, uint8_t *out);
uint16_t ref_pseudo_seed(uint32_t src_raw, uint32_t dst_raw, uint8_t proto, uint16_t tot_len);

/* event records: the reference's usys encoders and iomap */
#include <stddef.h>
void ref_ev_set_iomap(uint64_t iomap_offset);
uint64_t ref_iomap(const void *p);
void ref_ev_udp(void *addr, size_t len, void *id, uint64_t out[5]);
void ref_ev_tcp(uint64_t handle, unsigned long cookie, void *addr, size_t len, uint64_t out[5]);

/* the tcp_input head run for real (ref_tcphead.c): what tcp_rst received */
struct ref_tcphead_cap {
	int rst_called;
	uint32_t rst_seqno, rst_ackno; /* tcp_rst(ackno, seqno + tcplen, ...) (tcp_in.c:505) */
	uint16_t rst_local_port, rst_remote_port;
};
extern struct ref_tcphead_cap ref_th;
/* runs tcp_input over one segment with empty PCB lists; returns 1 when the
 * segment passed the head. hdr_out: the segment's first 16 bytes afterwards
 * (converted in place); tot_len_after: the pbuf length after the strip */
int ref_tcp_head(const uint8_t *seg, uint16_t seg_len, uint32_t src_raw, uint32_t dst_raw, uint8_t hdr_out[16],
		 uint16_t *tot_len_after);
#endif
