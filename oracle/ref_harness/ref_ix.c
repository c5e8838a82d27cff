/*
 * ref_ix.c - IX-side translation unit of the reference harness.
 *
 * TEST INFRASTRUCTURE ONLY. Compiles the reference's own dp/net/ip.c
 * (eth_input, ip_input) and dp/net/icmp.c (icmp_input) unmodified, straight
 * from /root/reference (the include paths come from oracle/Makefile), and
 * supplies link-time test doubles for the IX runtime symbols they reference:
 * per-CPU data normally defined in dp/core (cpu_id, mbuf_mempool, eth_txqs),
 * the flow-group table (fgs), and capture points for the callees eth_input
 * dispatches to (tcp_input_tmp, udp_input, arp_input) and for the mempool
 * slow path that mbuf_free reaches (mempool_free_2 = "dropped").
 *
 * dp/net/udp.c is NOT compiled: it includes <ix/vm.h> -> <mmu-x86.h> from
 * the un-vendored Dune submodule (deps/dune is empty), so it is unbuildable
 * here; its two-line length check is restated in harness_main.c.
 */
#include "/root/reference/dp/net/ip.c"
#include "/root/reference/dp/net/icmp.c"

#include "ref_capture.h"

/* ---- per-CPU data (normally in dp/core/cpu.c, mbuf.c, ethqueue.c) ---- */
DEFINE_PERCPU(unsigned int, cpu_id);
DEFINE_PERCPU(struct mempool, mbuf_mempool);
DEFINE_PERCPU(struct eth_tx_queue *, eth_txqs[NETHDEV]);

/* ---- globals (normally dp/core/ethfg.c, cfg.c, control_plane.c) ---- */
struct eth_fg *fgs[ETH_MAX_TOTAL_FG + NCPU];
struct cfg_parameters CFG;
int cycles_per_us = 1000;

static struct eth_fg the_fg;           /* cur_cpu = 0 == percpu cpu_id */
static struct eth_tx_queue the_txq;    /* TX capture for icmp_reflect */
struct ref_capture ref_cap;

/* ---- capture points ---- */
void mempool_free_2(struct mempool *m, void *ptr)
{
	(void)m;
	(void)ptr;
	ref_cap.freed++;
}

void tcp_input_tmp(struct eth_fg *cur_fg, struct mbuf *pkt, struct ip_hdr *iphdr, void *tcphdr)
{
	(void)cur_fg;
	ref_cap.kind = REF_TCP;
	ref_cap.l4_off = (long)((uint8_t *)tcphdr - mbuf_mtod(pkt, uint8_t *));
	/* the pbuf length tcp_input_tmp allocates (dp/lwip/misc.c:61) */
	ref_cap.l4_len = (uint16_t)(ntoh16(iphdr->len) - iphdr->header_len * 4);
}

void udp_input(struct mbuf *pkt, struct ip_hdr *iphdr, struct udp_hdr *udphdr)
{
	(void)iphdr;
	ref_cap.kind = REF_UDP;
	ref_cap.l4_off = (long)((uint8_t *)udphdr - mbuf_mtod(pkt, uint8_t *));
}

void arp_input(struct mbuf *pkt, struct arp_hdr *hdr)
{
	ref_cap.kind = REF_ARP;
	ref_cap.l4_off = (long)((uint8_t *)hdr - mbuf_mtod(pkt, uint8_t *));
}

void logk(int level, const char *fmt, ...)
{
	(void)level;
	(void)fmt;
}

/* ---- entry points used by harness_main.c ---- */
static uint8_t percpu_area[1 << 16] __attribute__((aligned(64)));
static void *gs_block[8];

#include <asm/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

int ref_ix_init(void)
{
	gs_block[0] = percpu_area; /* %gs:0 = this CPU's percpu offset (inc/ix/cpu.h:58-65) */
	if (syscall(SYS_arch_prctl, ARCH_SET_GS, (unsigned long)gs_block))
		return -1;
	the_fg.cur_cpu = 0;
	fgs[0] = &the_fg;
	the_txq.cap = 1 << 30;
	percpu_get(eth_txqs)[0] = &the_txq;
	return 0;
}

/* Run the reference eth_input on one IX-layout mbuf (2112-B element, data at
 * +64, len at +0). Fills ref_cap. The frame is mutated only by icmp_reflect. */
void ref_eth_input(void *mbuf)
{
	struct mbuf *m = (struct mbuf *)mbuf;
	int txq_before = the_txq.len;
	memset(&ref_cap, 0, sizeof(ref_cap));
	ref_cap.kind = REF_NONE;
	m->fg_id = 0;
	/* fresh mempool state per call so every mbuf_free reaches mempool_free_2 */
	memset(&percpu_get(mbuf_mempool), 0, sizeof(struct mempool));
	eth_input(NULL, m);
	if (the_txq.len != txq_before) {
		ref_cap.kind = REF_ICMP_REFLECT;
		the_txq.len = 0;
	}
}

uint16_t ref_chksum_internet(const void *buf, int len)
{
	return chksum_internet((const char *)buf, len);
}
