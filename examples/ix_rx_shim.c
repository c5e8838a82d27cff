/*
 * ix_rx_shim.c - how IX's run-to-completion loop would call libixgrx.
 *
 * A compile-checked sketch of INTEGRATION.md: it replaces the per-packet
 * eth_input() loop of eth_process_recv (dp/core/ethqueue.c:117-149) with one
 * batched call. The mbuf type and the callees below are minimal stand-ins
 * for IX's (inc/ix/mbuf.h:73-90, dp/net/ip.c) so this file builds on its own;
 * in IX the same code sits in dp/core/ethqueue.c with IX's headers.
 *
 * build: gcc -O2 -Iinclude examples/ix_rx_shim.c -Lix_amd -lixgrx -o ix_rx_shim
 * run:   ./ix_rx_shim     (needs a GPU; exits 2 with a message without one)
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ixgrx.h"

/* ---- stand-ins for IX (inc/ix/mbuf.h:73-90) ---------------------------- */
struct mbuf {
	size_t len;              /* @0: frame length, CRC stripped */
	struct mbuf *next;       /* @8 */
	uint8_t pad0[12];
	uint16_t fg_id;          /* @28 */
	uint16_t ol_flags;       /* @30 */
	uint8_t pad1[32];
	uint8_t data[2048];      /* @64: frame bytes (mbuf_mtod) */
};

struct stats {
	unsigned tcp, udp, icmp, icmp_sent, arp, drop;
};

/* what IX's callees receive; each replaces a call made inside eth_input */
static void on_tcp(void *u, void *m, const struct ixg_rx_rec *r)
{
	/* IX: the pbuf that tcp_input_tmp (dp/lwip/misc.c:57-67) builds, already
	 * stripped to the payload: payload = mtod + r->l4_off, len = r->l4_len;
	 * PCB lookup starts at bucket r->pcb_bucket (tcp_in.c:249); mbuf->fg_id
	 * = r->fg_id. */
	((struct mbuf *)m)->fg_id = r->fg_id;
	((struct stats *)u)->tcp++;
}
static void on_udp(void *u, void *m, const struct ixg_rx_rec *r)
{
	/* IX: usys_udp_recv(mtod + r->l4_off, r->l4_len, ...) (udp.c:88) */
	(void)m; (void)r;
	((struct stats *)u)->udp++;
}
static void on_icmp(void *u, void *m, const struct ixg_rx_rec *r)
{
	/* IX: with IXG_RF_REPLY (the asynchronous path with
	 * IXG_ASYNC_ICMP_REFLECT) the mbuf already holds the reply:
	 * eth_send_one(percpu_get(eth_num_queues)..., m, len) (icmp.c:71);
	 * otherwise icmp_reflect on the mbuf (icmp.c:89-92) */
	(void)m;
	if (r->flags & IXG_RF_REPLY)
		((struct stats *)u)->icmp_sent++;
	((struct stats *)u)->icmp++;
}
static void on_arp(void *u, void *m, const struct ixg_rx_rec *r)
{
	/* IX: arp_input(mbuf, mtod + 14) (ip.c:134-135) */
	(void)m; (void)r;
	((struct stats *)u)->arp++;
}
static void on_drop(void *u, void *m, const struct ixg_rx_rec *r)
{
	/* IX: mbuf_free(m) (ip.c:112-113,137); r->verdict says why */
	(void)m; (void)r;
	((struct stats *)u)->drop++;
}

static const struct ixg_rx_ops ix_ops = {on_tcp, on_udp, on_icmp, on_arp, on_drop};

/* The replacement for eth_process_recv's inner loop: up to `n` mbufs taken
 * round-robin from the RX queues (as eth_process_recv_queue does), one
 * batched transform, then the callees in input order. */
static int eth_process_recv_batch(void *ctx, struct mbuf **pkts, uint32_t n, struct ixg_rx_rec *recs,
				  struct stats *st)
{
	int rc = ixg_rx_batch_mbufs(ctx, (void *const *)pkts, n, recs);
	if (rc)
		return rc;
	ixg_rx_dispatch((void *const *)pkts, recs, n, &ix_ops, st);
	return 0;
}

/* one valid 60-byte Eth/IPv4/TCP frame (checksums filled in below) */
static void make_frame(uint8_t *f, uint32_t i)
{
	memset(f, 0, 60);
	f[12] = 0x08;
	f[14] = 0x45;
	f[17] = 40;          /* ip_len */
	f[22] = 64;          /* ttl */
	f[23] = 6;           /* TCP */
	uint32_t src = 0x0a000001u + i, dst = 0x0a000002u;
	for (int k = 0; k < 4; k++) {
		f[26 + k] = (uint8_t)(src >> (24 - 8 * k));
		f[30 + k] = (uint8_t)(dst >> (24 - 8 * k));
	}
	f[34] = (uint8_t)((1024 + i) >> 8); f[35] = (uint8_t)(1024 + i);
	f[36] = 0x00; f[37] = 80;
	f[46] = 0x50; f[47] = 0x10; /* doff 5, ACK */
	uint32_t s = 0;
	for (int k = 14; k < 34; k += 2) s += (uint32_t)(f[k] << 8 | f[k + 1]);
	while (s >> 16) s = (s & 0xffff) + (s >> 16);
	f[24] = (uint8_t)(~s >> 8); f[25] = (uint8_t)~s;
	s = 6 + 20; /* pseudo header: proto + TCP length */
	for (int k = 26; k < 34; k += 2) s += (uint32_t)(f[k] << 8 | f[k + 1]);
	for (int k = 34; k < 54; k += 2) s += (uint32_t)(f[k] << 8 | f[k + 1]);
	while (s >> 16) s = (s & 0xffff) + (s >> 16);
	f[50] = (uint8_t)(~s >> 8); f[51] = (uint8_t)~s;
}

int main(void)
{
	enum { N = 64 }; /* eth_rx_max_batch default */
	struct ixg_rx_cfg cfg;
	memset(&cfg, 0, sizeof(cfg));
	for (int k = 0; k < 40; k++)
		cfg.rss_key[k] = (uint8_t)(0x6d + 7 * k);
	cfg.nb_rx_fgs = 128;
	void *ctx = NULL;
	int rc = ixg_rx_init(&cfg, 0, &ctx);
	if (rc) {
		fprintf(stderr, "ixg_rx_init: %s (%d)\n", ixg_strerror(rc), rc);
		return 2;
	}
	struct mbuf *pkts[N];
	struct ixg_rx_rec recs[N];
	for (uint32_t i = 0; i < N; i++) {
		pkts[i] = aligned_alloc(64, sizeof(struct mbuf));
		memset(pkts[i], 0, sizeof(struct mbuf));
		pkts[i]->len = 60;
		make_frame(pkts[i]->data, i);
	}
	struct stats st = {0};
	rc = eth_process_recv_batch(ctx, pkts, N, recs, &st);
	printf("rc=%d tcp=%u udp=%u icmp=%u arp=%u drop=%u\n", rc, st.tcp, st.udp, st.icmp, st.arp, st.drop);
	for (uint32_t i = 0; i < N; i++)
		free(pkts[i]);
	ixg_rx_fini(ctx);
	return rc == 0 && st.tcp == N ? 0 : 1;
}
