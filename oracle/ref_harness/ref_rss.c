/*
 * ref_rss.c - the reference's software Toeplitz hash.
 *
 * TEST INFRASTRUCTURE ONLY. compute_toeplitz_hash is static in
 * dp/net/tcp_api.c:581-604, so the file is included unmodified and only the
 * wrapper's reachable code is kept by --gc-sections (no stubs needed).
 */
#include "/root/reference/dp/net/tcp_api.c"

#include "ref_capture.h"

uint32_t ref_toeplitz(const uint8_t *key, uint32_t src_raw, uint32_t dst_raw, uint16_t sport_raw,
		      uint16_t dport_raw)
{
	return compute_toeplitz_hash(key, src_raw, dst_raw, sport_raw, dport_raw);
}

/* The reference's TCP TX frame build: tcp_output_packet
 * (dp/net/tcp_api.c:773-826) on a one-pbuf chain holding the segment, for a
 * pcb with the given addresses, tos and ttl; ip_send_one (ip.c) queues the
 * mbuf on the harness's TX queue (ref_tx_take). */
void *ref_cur_fg(void);
uint32_t ref_tx_take(uint8_t *out);

uint32_t ref_tcp_frame(uint32_t local_raw, uint32_t remote_raw, uint8_t tos, uint8_t ttl, const void *seg,
		       uint16_t len, uint8_t *out)
{
	static struct tcp_pcb pcb;
	struct pbuf p;
	memset(&pcb, 0, sizeof(pcb));
	memset(&p, 0, sizeof(p));
	pcb.local_ip.addr = local_raw;
	pcb.remote_ip.addr = remote_raw;
	pcb.tos = tos;
	pcb.ttl = ttl;
	p.payload = (void *)seg;
	p.len = p.tot_len = len;
	p.type = PBUF_ROM;
	if (tcp_output_packet((struct eth_fg *)ref_cur_fg(), &pcb, &p))
		return 0;
	return ref_tx_take(out);
}
