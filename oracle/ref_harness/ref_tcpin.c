/*
 * ref_tcpin.c - tcp_input side translation unit of the reference harness.
 *
 * TEST INFRASTRUCTURE ONLY. Compiles the reference's dp/net/tcp_in.c
 * unmodified; only tcp_input_find_list (tcp_in.c:122-143) is reached, so
 * --gc-sections drops the rest of the file and its callees. The wrapper
 * builds an hlist of struct tcp_pcb (inc/ix/list.h:687-732) in the given
 * list order and runs the reference walk over it.
 */
#include "/root/reference/dp/net/tcp_in.c"

#include "ref_capture.h"

#define REF_MAX_LIST 4096

int ref_find_list(const struct ref_pcb *pcbs, int n, uint32_t src_raw, uint32_t dst_raw, uint16_t src_port,
		  uint16_t dst_port)
{
	static struct tcp_pcb pool[REF_MAX_LIST];
	struct hlist_head head;
	struct LWIP_Context ctx;
	struct tcp_hdr hdr;
	ipX_addr_t s, d;

	if (n > REF_MAX_LIST)
		return -2;
	hlist_init_head(&head);
	for (int k = n - 1; k >= 0; k--) { /* add_head in reverse: list order = pcbs[0..n) */
		memset(&pool[k], 0, sizeof(pool[k]));
		pool[k].remote_ip.addr = pcbs[k].remote_ip;
		pool[k].local_ip.addr = pcbs[k].local_ip;
		pool[k].remote_port = pcbs[k].remote_port;
		pool[k].local_port = pcbs[k].local_port;
		pool[k].state = ESTABLISHED;
		hlist_add_head(&head, &pool[k].link);
	}
	memset(&ctx, 0, sizeof(ctx));
	memset(&hdr, 0, sizeof(hdr));
	hdr.src = src_port; /* host order, as after tcp_in.c:230-231 */
	hdr.dest = dst_port;
	ctx.tcphdr = &hdr;
	memset(&s, 0, sizeof(s));
	memset(&d, 0, sizeof(d));
	s.addr = src_raw;
	d.addr = dst_raw;
	struct tcp_pcb *r = tcp_input_find_list(&ctx, &head, &s, &d);
	return r ? (int)(r - pool) : -1;
}
