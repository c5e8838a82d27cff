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
/* weak: ixref_rx links dp/core/ethfg.c (ref_ethfg.c), which defines it */
__attribute__((weak)) struct eth_fg *fgs[ETH_MAX_TOTAL_FG + NCPU];
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

/* harness_bench.c: the tcp_input head run in place of the capture */
void (*ref_tcp_hook)(const uint8_t *frame, const uint8_t *tcphdr, uint16_t len);

void tcp_input_tmp(struct eth_fg *cur_fg, struct mbuf *pkt, struct ip_hdr *iphdr, void *tcphdr)
{
	(void)cur_fg;
	if (ref_tcp_hook) {
		/* the pbuf length tcp_input_tmp allocates (dp/lwip/misc.c:61) */
		ref_tcp_hook(mbuf_mtod(pkt, uint8_t *), (const uint8_t *)tcphdr,
			     (uint16_t)(ntoh16(iphdr->len) - iphdr->header_len * 4));
		return;
	}
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

/* eth_input on a pre-filled mbuf with nothing around it (harness_bench.c):
 * the per-CPU mbuf mempool stays zeroed (ref_ix_init), so a drop's mbuf_free
 * takes the mempool_free_2 stub and never writes into the arena */
void ref_eth_input_raw(void *mbuf)
{
	eth_input(NULL, (struct mbuf *)mbuf);
}

/* icmp_reflect's source MAC and IP address (CFG.mac, CFG.host_addr, host
 * order as cfg.c stores it) */
void ref_set_host(const uint8_t mac[6], uint32_t host_addr)
{
	memcpy(&CFG.mac, mac, 6);
	CFG.host_addr.addr = host_addr;
}

uint16_t ref_chksum_internet(const void *buf, int len)
{
	return chksum_internet((const char *)buf, len);
}

/* ---- TX test doubles (the reference's TX path) ---- */
/* mempool slow path (mbuf_alloc_local -> mempool_alloc_2 when the per-CPU
 * free list is empty, as it always is here): one zeroed IX mbuf element */
static uint8_t tx_mbuf[2112] __attribute__((aligned(64)));
void *mempool_alloc_2(struct mempool *m)
{
	(void)m;
	memset(tx_mbuf, 0, sizeof(tx_mbuf));
	return tx_mbuf;
}
void mbuf_default_done(struct mbuf *m) { (void)m; }

/* the ARP table row ip_send_one finds (dp/net/ip.c:208) */
static struct eth_addr arp_mac;
int arp_lookup_mac(struct ip_addr *addr, struct eth_addr *mac)
{
	(void)addr;
	*mac = arp_mac;
	return 0;
}
int arp_add_pending_pkt(struct ip_addr *dst_addr, struct eth_fg *fg, struct mbuf *mbuf, size_t len)
{
	(void)dst_addr;
	(void)fg;
	(void)mbuf;
	(void)len;
	return -1;
}

void ref_tx_set_macs(const uint8_t src[6], const uint8_t dst[6])
{
	memcpy(&CFG.mac, src, 6);
	memcpy(&arp_mac, dst, 6);
}

void *ref_cur_fg(void) { return &the_fg; }

/* The frame the last eth_send_one queued (its mbuf data and mbuf->len);
 * returns the length, 0 when nothing was queued. */
uint32_t ref_tx_take(uint8_t *out)
{
	if (!the_txq.len)
		return 0;
	struct mbuf *m = the_txq.bufs[the_txq.len - 1];
	the_txq.len = 0;
	the_txq.cap = 1 << 30;
	memcpy(out, mbuf_mtod(m, uint8_t *), m->len);
	return (uint32_t)m->len;
}

/* [UDP] udp_output (dp/net/udp.c:114-128) is unbuildable here (udp.c needs
 * Dune's mmu-x86.h); its header writes are restated over the reference's own
 * ip_setup_header (dp/net/net.h:65-78) and chksum_internet, and the frame is
 * queued through the reference's ip_send_one's Ethernet fill-in instead of
 * udp_output's inline copy of it (udp.c:115-117, the same three writes). */
uint32_t ref_udp_frame(uint32_t src_raw, uint32_t dst_raw, uint16_t sport, uint16_t dport, const void *payload,
		       uint16_t len, uint8_t *out)
{
	struct mbuf *pkt = mbuf_alloc_local();
	struct eth_hdr *ethhdr = mbuf_mtod(pkt, struct eth_hdr *);
	struct ip_hdr *iphdr = mbuf_nextd(ethhdr, struct ip_hdr *);
	struct udp_hdr *udphdr = mbuf_nextd(iphdr, struct udp_hdr *);
	size_t full_len = len + sizeof(struct udp_hdr);
	struct ip_addr dst;
	ip_setup_header(iphdr, IPPROTO_UDP, ntoh32(src_raw), ntoh32(dst_raw), full_len);
	iphdr->chksum = chksum_internet((void *)iphdr, sizeof(struct ip_hdr));
	udphdr->src_port = hton16(sport);
	udphdr->dst_port = hton16(dport);
	udphdr->len = hton16(full_len);
	udphdr->chksum = 0;
	memcpy(udphdr + 1, payload, len);
	dst.addr = ntoh32(dst_raw);
	if (ip_send_one(&the_fg, &dst, pkt, sizeof(struct eth_hdr) + sizeof(struct ip_hdr) + full_len))
		return 0;
	return ref_tx_take(out);
}
