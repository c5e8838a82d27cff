/*
 * ref_tcphead_stubs.c - link-time test doubles for ref_tcphead.c.
 *
 * TEST INFRASTRUCTURE ONLY. tcp_input (dp/net/tcp_in.c) references the rest
 * of the TCP stack (tcp.c, tcp_out.c, the timer wheel, the event upcall).
 * With empty PCB lists none of it runs: a segment either fails the head
 * (`dropped`, pbuf_free) or takes the no-PCB path, whose one callee is
 * tcp_rst (tcp_in.c:503-506) -> tcp_rst_impl, the capture point here. Every
 * other symbol aborts if reached, so a capture can never silently come from
 * a stubbed path. No headers of the reference are included: the symbols are
 * matched by name at link time. oracle/Makefile links this file and
 * ref_tcphead.c into one object and keeps only the entry points global, so
 * these doubles never stand in for the real functions other harness units
 * link (tcp_api.c's lwip_tcp_event in ref_rss.c).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ref_capture.h"

/* tcp_rst_impl(cur_fg, seqno, ackno, local_ip, remote_ip, local_port,
 * remote_port) (inc/lwip/lwip/tcp_impl.h:604-617, LWIP_IPV6 off) */
void tcp_rst_impl(void *cur_fg, uint32_t seqno, uint32_t ackno, void *local_ip, void *remote_ip,
		  uint16_t local_port, uint16_t remote_port)
{
	(void)cur_fg;
	(void)local_ip;
	(void)remote_ip;
	ref_th.rst_called++;
	ref_th.rst_seqno = seqno;
	ref_th.rst_ackno = ackno;
	ref_th.rst_local_port = local_port;
	ref_th.rst_remote_port = remote_port;
}

static void unreached(const char *what)
{
	fprintf(stderr, "ref_tcphead: tcp_input reached %s with empty PCB lists\n", what);
	abort();
}

#define UNREACHED(name) \
	void name(void) { unreached(#name); }

UNREACHED(lwip_tcp_event)
UNREACHED(tcp_abandon)
UNREACHED(tcp_abort)
UNREACHED(tcp_alloc)
UNREACHED(tcp_eff_send_mss_impl)
UNREACHED(tcp_enqueue_flags)
UNREACHED(tcp_output)
UNREACHED(tcp_pcb_purge)
UNREACHED(tcp_pcb_remove)
UNREACHED(tcp_process_refused_data)
UNREACHED(tcp_rexmit)
UNREACHED(tcp_rexmit_fast)
UNREACHED(tcp_seg_copy)
UNREACHED(tcp_seg_free)
UNREACHED(tcp_segs_free)
UNREACHED(tcp_send_empty_ack)
UNREACHED(tcp_unified_timer_handler)
UNREACHED(tcp_update_rcv_ann_wnd)
UNREACHED(timer_add)
UNREACHED(timer_add_abs)
UNREACHED(timer_now)

/* data symbols tcp_in.c declares extern: never read on the head paths */
uint8_t tcp_persist_backoff[8];
uint8_t tcp_pcb_mempool[256];
