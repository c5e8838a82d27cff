/*
 * ref_tcphead.c - the reference's tcp_input head, run for real.
 *
 * TEST INFRASTRUCTURE ONLY. Compiles dp/net/tcp_in.c unmodified and runs its
 * tcp_input (tcp_in.c:157-241: length check, doff strip, the in-place
 * conversion of the TCP header to host order, seqno/ackno/wnd/flags/tcplen
 * into the LWIP_Context) over one segment, with empty PCB lists: every
 * segment that passes the head falls through to the no-PCB path
 * (tcp_in.c:500-507), whose tcp_rst(ackno, seqno + tcplen, ...) is the
 * capture point (ref_tcphead_stubs.c). What the head left behind is read
 * back: the converted header bytes in the segment buffer, the pbuf's length
 * after the strip, and the tcp_rst arguments.
 *
 * The pbuf is the one tcp_input_tmp builds (dp/lwip/misc.c:57-67): PBUF_ROM,
 * payload = the TCP header, len = tot_len = ip_len - ihl*4. It is set up here
 * with ref = 2 so the reference's pbuf_free (tcp_in.c:509/515) only drops a
 * reference and the harness can read it afterwards.
 */
#include "/root/reference/dp/net/tcp_in.c"

#include "ref_capture.h"

/* per-CPU state tcp_input reads: the listen list (tcp_in.c:274), empty */
DEFINE_PERCPU(struct tcp_global_percpu_lists, tcp_cpu_lists);

/* pbuf_free's release path (memp.h:70-76), which a pbuf held with ref = 2
 * never takes; it is linked in now that pbuf_free is reachable */
DEFINE_PERCPU(struct mempool, pbuf_mempool);
void mem_free(void *mem)
{
	(void)mem;
	abort();
}

struct ref_tcphead_cap ref_th;

int ref_tcp_head(const uint8_t *seg_in, uint16_t seg_len, uint32_t src_raw, uint32_t dst_raw,
		 uint8_t hdr_out[16], uint16_t *tot_len_after)
{
	static uint8_t seg[1 << 16];
	static struct eth_fg fg; /* active_tbl / tw_pcbs: empty hlists (zeroed) */
	struct pbuf p;
	ip_addr_t s, d;

	memset(&fg, 0, sizeof(fg));
	memset(seg, 0, 64);
	memcpy(seg, seg_in, seg_len);
	memset(&p, 0, sizeof(p));
	p.payload = seg;
	p.len = p.tot_len = seg_len;
	p.type = PBUF_ROM;
	p.ref = 2;
	s.addr = src_raw;
	d.addr = dst_raw;
	memset(&ref_th, 0, sizeof(ref_th));
	tcp_input(&fg, &p, &s, &d);
	memcpy(hdr_out, seg, 16);
	*tot_len_after = p.tot_len;
	/* passed the head: pbuf_header moved the payload past the header, or
	 * the header length was 0 (a strip of nothing, which cannot fail) */
	return p.payload != (void *)seg || (seg_len >= 20 && (seg_in[12] >> 4) == 0);
}
