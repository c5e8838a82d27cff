/*
 * ref_lwip.c - lwIP-side translation unit of the reference harness.
 *
 * TEST INFRASTRUCTURE ONLY. Compiles the reference's dp/lwip/inet_chksum.c
 * (inet_chksum_pseudo_partial + lwip_standard_chksum) and dp/lwip/pbuf.c
 * (pbuf_header) unmodified, and uses tcp_to_idx / hash_crc32c_* from the
 * reference headers (inc/lwip/lwip/tcp_impl.h:381-387, inc/ix/hash.h). Only
 * the functions reachable from the wrappers below survive --gc-sections.
 */
#include "/root/reference/dp/lwip/inet_chksum.c"
#include "/root/reference/dp/lwip/pbuf.c"
#include <lwip/tcp_impl.h>

#include "ref_capture.h"

uint16_t ref_pseudo_partial(const void *seg, uint16_t len, uint8_t proto, uint16_t proto_len,
			    uint32_t src_raw, uint32_t dst_raw)
{
	/* the PBUF_ROM pbuf tcp_input_tmp builds: payload = L4 header, len = tot_len */
	struct pbuf p;
	ip_addr_t s, d;
	memset(&p, 0, sizeof(p));
	p.payload = (void *)seg;
	p.len = p.tot_len = len;
	p.type = PBUF_ROM;
	s.addr = src_raw;
	d.addr = dst_raw;
	return inet_chksum_pseudo_partial(&p, proto, proto_len, len, &s, &d);
}

int ref_pbuf_header_rom(uint16_t len, int16_t inc, uint16_t *new_len)
{
	static uint8_t dummy[1 << 16];
	struct pbuf p;
	memset(&p, 0, sizeof(p));
	p.payload = dummy;
	p.len = p.tot_len = len;
	p.type = PBUF_ROM;
	int r = pbuf_header(&p, inc);
	*new_len = p.len;
	return r;
}

int ref_tcp_to_idx(uint32_t local_raw, uint32_t remote_raw, uint16_t local_port, uint16_t remote_port)
{
	ipX_addr_t l, r;
	memset(&l, 0, sizeof(l));
	memset(&r, 0, sizeof(r));
	l.addr = local_raw;
	r.addr = remote_raw;
	return tcp_to_idx(&l, &r, local_port, remote_port);
}

/* pbuf.c's unreachable allocators reference these; never called here */

/* inet_chksum_pseudo (inet_chksum.c:353-357): the TX offload seed */
uint16_t ref_pseudo_seed(uint32_t src_raw, uint32_t dst_raw, uint8_t proto, uint16_t tot_len)
{
	struct pbuf p;
	ip_addr_t s, d;
	memset(&p, 0, sizeof(p));
	p.tot_len = tot_len;
	s.addr = src_raw;
	d.addr = dst_raw;
	return inet_chksum_pseudo(&p, proto, tot_len, &s, &d);
}
