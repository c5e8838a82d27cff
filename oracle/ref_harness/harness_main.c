/*
 * harness_main.c - drive the reference's own RX code over a frame file.
 *
 * TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ixref_rx; used by
 * tests/golden/make_golden.py to produce the committed golden vectors).
 * No reference header is included here: every reference function is reached
 * through the ref_* wrappers of the ref_*.c translation units.
 *
 * Per frame: the frame is placed in a zeroed IX mbuf (2112-B element, len at
 * +0, data at +64: inc/ix/mbuf.h:73-90), the reference eth_input runs on it
 * and the harness observes which callee it reached and with which L4
 * pointer. Values come from the reference's functions: chksum_internet,
 * inet_chksum_pseudo_partial, ip6_chksum_pseudo_partial, pbuf_header,
 * tcp_to_idx, compute_toeplitz_hash. What the tree does not hold is restated
 * here and flagged:
 *   [NIC]  the driver's checksum/RSS applicability rules (DESIGN.md "NIC rules")
 *   [UDP]  udp.c:59's length check (udp.c is unbuildable: needs Dune's mmu-x86.h)
 *   [TCP]  the tcp_input head glue around pbuf_header (tcp_in.c:189,221-222,240)
 *   [WHY]  drop reason codes, each confirmed by the reference: the blamed field
 *          is repaired and eth_input run again (confirm_drop)
 *   [V6]   the IPv6 extension (reference drops 0x86DD); Toeplitz over 36 bytes
 *          is compute_toeplitz_hash's loop generalised, parity unpinned
 *   [FDIR] the NIC's flow-director perfect match (the 4-tuple of a
 *          non-fragmented IPv4 TCP frame equals an installed filter); what
 *          the stack then does with the FLM status is the reference's own
 *          eth_recv_handle_fg_transition (ref_ethfg.c)
 *
 * Input file  (LE): "IXGRXIN1", u32 n, u32 cfg_flags, u16 nb_rx_fgs, u16 dev_idx,
 *                   u8 key[40], u16 len[n], u32 off[n], u32 blob_len, blob,
 *                   optionally "FDIR", u32 nf, u16 cpu_id, u16 0,
 *                   struct ixg_fdir_filter[nf], and/or "HOST", u8 mac[6],
 *                   u16 0, u32 host_addr (CFG.mac / CFG.host_addr for
 *                   icmp_reflect; host order).
 * Output file (LE): "IXGRXOUT", u32 n, struct ixg_rx_rec[n] (16 B), u32 csum[n],
 *                   u8 confirm[n] (0: eth_input did not drop the frame; 1: it
 *                   did and confirm_drop pinned the reason; 2: not pinned),
 *                   "TCPX", struct ixg_tcp_ext[n], u8 hdr[n][16] (the rest of
 *                   the tcp_input head from the reference's own tcp_input,
 *                   ref_tcphead.c: its LWIP_Context fields and the segment's
 *                   first 16 bytes as it converted them in place),
 *                   "ICMP", u8 reflected[n], then each frame as eth_input left
 *                   it in its mbuf (len[i] bytes each: icmp_reflect rewrote
 *                   the ICMP_ECHO ones in place, dp/net/icmp.c:44-71).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/ixgrx.h"
#include "ref_capture.h"

static void die(const char *m, uint32_t i)
{
	fprintf(stderr, "ixref_rx: %s (frame %u)\n", m, i);
	exit(2);
}

static uint8_t Bz(const uint8_t *f, uint32_t L, uint32_t i) { return i < L ? f[i] : 0; }
static uint16_t B16z(const uint8_t *f, uint32_t L, uint32_t i)
{
	return (uint16_t)((Bz(f, L, i) << 8) | Bz(f, L, i + 1));
}
static uint32_t raw32(const uint8_t *p)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}
static uint16_t raw16(const uint8_t *p)
{
	uint16_t v;
	memcpy(&v, p, 2);
	return v;
}

/* [V6] bit-serial Toeplitz over n bytes, same loop as tcp_api.c:593-601 */
static uint32_t toeplitz_n(const uint8_t *key, const uint8_t *in, int n)
{
	uint32_t r = 0, kp = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) | ((uint32_t)key[2] << 8) | key[3];
	for (int i = 0; i < n; i++)
		for (int j = 128; j; j >>= 1) {
			if (in[i] & j)
				r ^= kp;
			kp <<= 1;
			if (key[i + 4] & j)
				kp |= 1;
		}
	return r;
}

static void drop(struct ixg_rx_rec *r, uint8_t v)
{
	r->verdict = v;
	r->l4_off = r->l4_len = 0;
	r->pcb_bucket = IXG_NO_BUCKET;
	r->tcp_flags = 0;
}

/* [WHY] the reason eth_input/ip_input/icmp_input dropped an IPv4/other frame */
static uint8_t drop_reason(const uint8_t *f, uint32_t L)
{
	uint16_t et = B16z(f, L, 12);
	if (et != 0x0800)
		return IXG_V_DROP_ETHERTYPE;
	uint32_t ver = Bz(f, L, 14) >> 4, ihl = Bz(f, L, 14) & 15, ip_len = B16z(f, L, 16);
	if (L < 34) return IXG_V_DROP_IP_SHORT;
	if (ver != 4) return IXG_V_DROP_IP_VERSION;
	if (ihl < 5) return IXG_V_DROP_IP_IHL;
	if (B16z(f, L, 20) & 0x3FFF) return IXG_V_DROP_IP_FRAG;
	if (ip_len < ihl * 4) return IXG_V_DROP_IP_LEN;
	if (14 + ip_len > L) return IXG_V_DROP_IP_TRUNC;
	uint8_t proto = Bz(f, L, 23);
	if (proto == 1) {
		uint32_t l4 = 14 + ihl * 4, n = ip_len - ihl * 4;
		if (n < 8) return IXG_V_DROP_ICMP_SHORT;
		if (ref_chksum_internet(f + l4, (int)n)) return IXG_V_DROP_ICMP_CSUM;
		return IXG_V_DROP_ICMP_TYPE;
	}
	return IXG_V_DROP_IP_PROTO;
}

static void put16(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}

/* the ICMP message's checksum rewritten so chksum_internet over it is 0 */
static void icmp_fix(uint8_t *g, uint32_t l4, uint32_t n)
{
	g[l4 + 2] = g[l4 + 3] = 0;
	uint16_t c = ref_chksum_internet(g + l4, (int)n);
	memcpy(g + l4 + 2, &c, 2);
}

/* [WHY] pin: mend the one field (or length) drop reason `why` blames.
 * Returns 0 when the reason has no repair. */
static int repair(uint8_t *g, uint32_t *L, uint8_t why)
{
	const uint32_t ihl = g[14] & 15, l4 = 14 + ihl * 4;
	uint32_t ip_len = ((uint32_t)g[16] << 8) | g[17];
	switch (why) {
	case IXG_V_DROP_ETHERTYPE: /* (a frame shorter than its Ethernet header grows) */
		put16(g + 12, 0x0800);
		if (*L < 14)
			*L = 14;
		return 1;
	case IXG_V_DROP_IP_SHORT: *L = 34; return 1; /* the frame grows (zero bytes) */
	case IXG_V_DROP_IP_VERSION: g[14] = (uint8_t)(0x40 | ihl); return 1;
	case IXG_V_DROP_IP_IHL: g[14] = (uint8_t)((g[14] & 0xF0) | 5); return 1;
	case IXG_V_DROP_IP_FRAG: g[20] &= 0x40; g[21] = 0; return 1; /* DF kept */
	case IXG_V_DROP_IP_LEN: put16(g + 16, ihl * 4); return 1;
	case IXG_V_DROP_IP_TRUNC:
		if (14 + ip_len <= IXG_MBUF_DATA_LEN)
			*L = 14 + ip_len;
		else
			put16(g + 16, *L - 14 >= ihl * 4 ? *L - 14 : ihl * 4);
		if (*L < l4)
			*L = l4;
		return 1;
	case IXG_V_DROP_IP_PROTO: g[23] = 17; return 1;
	case IXG_V_DROP_ICMP_SHORT:
		put16(g + 16, ihl * 4 + 8);
		if (*L < l4 + 8)
			*L = l4 + 8;
		icmp_fix(g, l4, 8);
		return 1;
	case IXG_V_DROP_ICMP_CSUM: icmp_fix(g, l4, ip_len - ihl * 4); return 1;
	case IXG_V_DROP_ICMP_TYPE: g[l4] = 8; icmp_fix(g, l4, ip_len - ihl * 4); return 1;
	}
	return 0;
}

/* [WHY] pin: a restated drop reason is confirmed by the reference itself.
 * The blamed field is repaired and the reference eth_input runs again; the
 * frame must then be delivered, or dropped for a strictly later reason (the
 * order of the checks in eth_input/ip_input/icmp_input, ip.c:63-114,
 * icmp.c:78-115), whose field is repaired in turn, until the reference
 * delivers it. Returns the number of repairs, 0 when not confirmed. */
static int confirm_drop(const uint8_t *frame, uint32_t L, uint8_t why, uint8_t *mbuf)
{
	uint8_t g[IXG_MBUF_DATA_LEN + 64];
	memset(g, 0, sizeof(g));
	memcpy(g, frame, L);
	for (int step = 1; step <= 16; step++) {
		if (!repair(g, &L, why) || L > IXG_MBUF_DATA_LEN)
			return 0;
		size_t len = L;
		memset(mbuf, 0, IXG_MBUF_STRIDE);
		memcpy(mbuf, &len, sizeof(len));
		memcpy(mbuf + IXG_MBUF_HEADER_LEN, g, L);
		ref_eth_input(mbuf);
		if (ref_cap.kind != REF_NONE)
			return step;
		const uint8_t next = drop_reason(g, L);
		if (next <= why)
			return 0;
		why = next;
	}
	return 0;
}

static const struct ixg_fdir_filter *fdir;
static uint32_t n_fdir;
static unsigned int fdir_cpu;

/* the rest of the tcp_input head (tcp_in.c:230-241) for the frame one() just
 * classified: ixg_tcp_ext and the segment's first 16 bytes as the head leaves
 * them (converted to host order in place); zero for every other verdict */
static struct ixg_tcp_ext th_ext;
static uint8_t th_hdr[16];
/* the frame as eth_input left it (icmp_reflect rewrites echo requests) */
static uint8_t after[IXG_MBUF_DATA_LEN];
static uint8_t reflected;

static uint16_t h16(const uint8_t *p)
{
	uint16_t v;
	memcpy(&v, p, 2);
	return v;
}
static uint32_t h32(const uint8_t *p)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}

/* fill th_ext from a header already in host order and the post-strip length */
static void ext_from(const uint8_t *hdr, uint16_t tot_len, uint8_t tcp_flags)
{
	th_ext.seqno = h32(hdr + 4);
	th_ext.ackno = h32(hdr + 8);
	th_ext.wnd = h16(hdr + 14);
	/* tcp_in.c:241: TCP_FIN 0x01, TCP_SYN 0x02 */
	th_ext.tcplen = (uint16_t)(tot_len + ((tcp_flags & 0x03) ? 1 : 0));
	th_ext.src_port = h16(hdr);
	th_ext.dst_port = h16(hdr + 2);
}

/* [V6] the extension's TCP: the reference never parses IPv6; the head's
 * conversions restated over the segment at 54 */
static void ext_v6(const uint8_t *f, uint16_t tot_len, uint8_t tcp_flags)
{
	const uint8_t *t = f + 54;
	th_hdr[0] = t[1], th_hdr[1] = t[0], th_hdr[2] = t[3], th_hdr[3] = t[2];
	for (int k = 0; k < 4; k++) {
		th_hdr[4 + k] = t[7 - k];
		th_hdr[8 + k] = t[11 - k];
	}
	th_hdr[12] = t[12], th_hdr[13] = t[13], th_hdr[14] = t[15], th_hdr[15] = t[14];
	ext_from(th_hdr, tot_len, tcp_flags);
}

static void one(const struct ixg_rx_cfg *cfg, const uint8_t *frame, uint32_t L, uint8_t *mbuf,
		struct ixg_rx_rec *r, uint32_t *csum, uint8_t *confirm, uint32_t idx)
{
	uint8_t f[2048 + 64];
	uint16_t ip_res = 0xffff, l4_res = 0xffff;
	uint32_t rss = 0;
	uint8_t flags = 0;

	memset(r, 0, sizeof(*r));
	memset(&th_ext, 0, sizeof(th_ext));
	memset(th_hdr, 0, sizeof(th_hdr));
	memcpy(after, frame, L);
	reflected = 0;
	*confirm = 0;
	r->pcb_bucket = IXG_NO_BUCKET;
	memset(f, 0, sizeof(f));
	memcpy(f, frame, L); /* a pristine copy: icmp_reflect rewrites the mbuf */

	uint16_t et = B16z(f, L, 12);
	uint32_t ver = f[14] >> 4, ihl = f[14] & 15, ip_len = B16z(f, L, 16), l4 = 14 + ihl * 4;
	uint8_t proto = f[23];
	int frag = (B16z(f, L, 20) & 0x3FFF) != 0;
	int v6 = et == 0x86DD && (cfg->flags & IXG_F_IPV6);

	/* [NIC] IP header checksum */
	int hdr_ok = et == 0x0800 && ver == 4 && ihl >= 5 && l4 <= L;
	if (hdr_ok) {
		ip_res = ref_chksum_internet(f + 14, (int)(ihl * 4));
		flags |= IXG_RF_IP_CSUM_CHECKED | (ip_res == 0 ? IXG_RF_IP_CSUM_OK : 0);
	}
	/* [NIC] RSS */
	if (hdr_ok && !frag && (proto == 6 || proto == 17) && l4 + 4 <= L) {
		rss = ref_toeplitz(cfg->rss_key, raw32(f + 26), raw32(f + 30), raw16(f + l4), raw16(f + l4 + 2));
		flags |= IXG_RF_RSS;
	} else if (v6 && L >= 58 && (f[14] >> 4) == 6 && (f[20] == 6 || f[20] == 17)) {
		uint8_t in[36];
		memcpy(in, f + 22, 32);
		memcpy(in + 32, f + 54, 4);
		rss = toeplitz_n(cfg->rss_key, in, 36);
		flags |= IXG_RF_RSS;
	}
	r->rss_hash = rss;
	r->fg_id = (uint16_t)(cfg->dev_idx * 512u + (rss & (uint32_t)(cfg->nb_rx_fgs - 1)));
	/* [FDIR] a perfect-filter match sets FLM: the driver's fg_id is
	 * MBUF_INVALID_FG_ID (ixgbe.c:329-330), then eth_recv maps it */
	if (n_fdir && hdr_ok && !frag && proto == 6 && l4 + 4 <= L) {
		for (uint32_t k = 0; k < n_fdir; k++)
			if (fdir[k].src_ip == raw32(f + 26) && fdir[k].dst_ip == raw32(f + 30) &&
			    fdir[k].src_port == B16z(f, L, l4) && fdir[k].dst_port == B16z(f, L, l4 + 2)) {
				uint32_t fg = ref_fg_transition(0xFFFF, fdir_cpu);
				if (fg > 0xffff)
					die("outbound flow group not processed on its CPU", idx);
				r->fg_id = (uint16_t)fg;
				flags |= IXG_RF_FDIR;
				break;
			}
	}

	/* [NIC] L4 checksum */
	int l4c = 0;
	if (hdr_ok && !frag && (proto == 6 || proto == 17) && ip_len >= ihl * 4 && 14 + ip_len <= L) {
		uint32_t n = ip_len - ihl * 4;
		if ((proto == 6 && n >= 20) || (proto == 17 && n >= 8 && B16z(f, L, l4 + 6) != 0)) {
			l4_res = ref_pseudo_partial(f + l4, (uint16_t)n, proto, (uint16_t)n, raw32(f + 26), raw32(f + 30));
			l4c = 1;
		}
	}
	uint32_t plen = B16z(f, L, 18);
	int v6ok = v6 && L >= 54 && (f[14] >> 4) == 6 && 54 + plen <= L;
	if (v6ok && ((f[20] == 6 && plen >= 20) || (f[20] == 17 && plen >= 8))) {
		l4_res = ref_pseudo6_partial(f + 54, (uint16_t)plen, f[20], (uint16_t)plen, f + 22, f + 38);
		l4c = 1;
	}
	if (l4c)
		flags |= IXG_RF_L4_CSUM_CHECKED | (l4_res == 0 ? IXG_RF_L4_CSUM_OK : 0);
	r->flags = flags;

	/* ICMP residual word: chksum_internet as icmp_input computes it */
	if (et == 0x0800 && L >= 34 && ver == 4 && ihl >= 5 && !frag && ip_len >= ihl * 4 &&
	    14 + ip_len <= L && proto == 1 && ip_len - ihl * 4 >= 8)
		l4_res = ref_chksum_internet(f + l4, (int)(ip_len - ihl * 4));
	*csum = (uint32_t)ip_res | ((uint32_t)l4_res << 16);

	/* the driver drops on the NIC verdict (ixgbe.c:312-324,349) */
	if (!(cfg->flags & IXG_F_NO_CSUM_DROP)) {
		if ((flags & IXG_RF_IP_CSUM_CHECKED) && !(flags & IXG_RF_IP_CSUM_OK)) {
			drop(r, IXG_V_DROP_CSUM_IP);
			return;
		}
		if ((flags & IXG_RF_L4_CSUM_CHECKED) && !(flags & IXG_RF_L4_CSUM_OK)) {
			drop(r, IXG_V_DROP_CSUM_L4);
			return;
		}
	}

	if (v6) {
		/* [V6] extension; the reference eth_input drops this frame */
		if (!v6ok || (f[20] != 6 && f[20] != 17)) {
			drop(r, IXG_V_DROP_IP6);
			return;
		}
		uint32_t n = plen;
		if (f[20] == 6) {
			if (n < 20) { drop(r, IXG_V_DROP_TCP_SHORT); return; }
			uint8_t doff = f[54 + 12] >> 4;
			uint16_t nl;
			if (ref_pbuf_header_rom((uint16_t)n, (int16_t)-(doff * 4), &nl)) { drop(r, IXG_V_DROP_TCP_HDRLEN); return; }
			r->verdict = IXG_V_TCP6;
			r->l4_off = (uint16_t)(54 + doff * 4);
			r->l4_len = nl;
			r->tcp_flags = f[54 + 13] & 0x3f;
			ext_v6(f, nl, r->tcp_flags);
		} else {
			uint16_t ulen = B16z(f, L, 54 + 4);
			if (54 + ulen > L) { drop(r, IXG_V_DROP_UDP_LEN); return; }
			r->verdict = IXG_V_UDP6;
			r->l4_off = 54 + 8;
			r->l4_len = ulen;
		}
		return;
	}

	/* the reference eth_input, for real */
	size_t len = L;
	memset(mbuf, 0, IXG_MBUF_STRIDE);
	memcpy(mbuf, &len, sizeof(len));
	memcpy(mbuf + IXG_MBUF_HEADER_LEN, f, L);
	ref_eth_input(mbuf);

	switch (ref_cap.kind) {
	case REF_NONE: {
		if (!ref_cap.freed)
			die("eth_input neither delivered nor freed", idx);
		uint8_t why = drop_reason(f, L);
		drop(r, why);
		*confirm = (uint8_t)(confirm_drop(f, L, why, mbuf) ? 1 : 2);
		return;
	}
	case REF_TCP: {
		if (ref_cap.freed)
			die("tcp delivered and freed", idx);
		uint32_t off = (uint32_t)ref_cap.l4_off;
		uint16_t n = ref_cap.l4_len;
		if (off != l4)
			die("tcp l4 offset mismatch", idx);
		/* the reference's own tcp_input over the segment tcp_input_tmp
		 * hands it (ref_tcphead.c): passed or dropped, and what the head
		 * converted in place */
		uint16_t tot_after = 0;
		const int passed = ref_tcp_head(f + off, n, raw32(f + 26), raw32(f + 30), th_hdr, &tot_after);
		/* [TCP] tcp_input head (tcp_in.c:189,221-222), which the real head must agree with */
		if (n < 20) {
			if (passed) die("tcp_input passed a segment shorter than 20", idx);
			memset(th_hdr, 0, sizeof(th_hdr));
			drop(r, IXG_V_DROP_TCP_SHORT);
			return;
		}
		uint8_t doff = f[off + 12] >> 4; /* TCPH_HDRLEN */
		uint16_t nl;
		if (ref_pbuf_header_rom(n, (int16_t)-(doff * 4), &nl)) {
			if (passed) die("tcp_input passed a segment with doff*4 > l4len", idx);
			memset(th_hdr, 0, sizeof(th_hdr));
			drop(r, IXG_V_DROP_TCP_HDRLEN);
			return;
		}
		if (!passed || tot_after != nl)
			die("tcp_input head disagrees with the pbuf_header restatement", idx);
		ext_from(th_hdr, tot_after, f[off + 13] & 0x3f);
		/* no PCB: tcp_rst(ackno, seqno + tcplen, ..., dest, src) unless RST (tcp_in.c:503-506) */
		if (f[off + 13] & 0x04) {
			if (ref_th.rst_called) die("tcp_rst for a segment carrying RST", idx);
		} else if (ref_th.rst_called != 1 || ref_th.rst_seqno != th_ext.ackno ||
			   ref_th.rst_ackno != th_ext.seqno + th_ext.tcplen || ref_th.rst_local_port != th_ext.dst_port ||
			   ref_th.rst_remote_port != th_ext.src_port) {
			die("tcp_rst arguments disagree with the converted header", idx);
		}
		r->verdict = IXG_V_TCP;
		r->l4_off = (uint16_t)(off + doff * 4);
		r->l4_len = nl;
		r->tcp_flags = f[off + 13] & 0x3f;
		/* tcp_in.c:230-233: ports to host order, local = dst, remote = src */
		r->pcb_bucket = (uint16_t)ref_tcp_to_idx(raw32(f + 30), raw32(f + 26),
							 (uint16_t)((f[off + 2] << 8) | f[off + 3]),
							 (uint16_t)((f[off] << 8) | f[off + 1]));
		return;
	}
	case REF_UDP: {
		if (ref_cap.freed)
			die("udp delivered and freed", idx);
		uint32_t off = (uint32_t)ref_cap.l4_off;
		uint16_t ulen = B16z(f, L, off + 4);
		/* [UDP] mbuf_enough_space(pkt, udphdr, len) (udp.c:59) */
		if (off + (uint32_t)ulen > L) { drop(r, IXG_V_DROP_UDP_LEN); return; }
		r->verdict = IXG_V_UDP;
		r->l4_off = (uint16_t)(off + 8);
		r->l4_len = ulen;
		return;
	}
	case REF_ARP:
		r->verdict = IXG_V_ARP;
		r->l4_off = (uint16_t)ref_cap.l4_off;
		r->l4_len = (uint16_t)(L >= 14 ? L - 14 : 0);
		return;
	case REF_ICMP_REFLECT:
		memcpy(after, mbuf + IXG_MBUF_HEADER_LEN, L);
		reflected = 1;
		r->verdict = IXG_V_ICMP_ECHO;
		r->l4_off = (uint16_t)l4;
		r->l4_len = (uint16_t)(ip_len - ihl * 4);
		return;
	}
	die("unknown capture", idx);
}

int main(int argc, char **argv)
{
	/* -t SECONDS: after the run, repeat it until SECONDS have passed and
	 * print the 1-core rate (bench.py's "reference" CPU figure) */
	double tsec = 0;
	if (argc == 5 && !strcmp(argv[1], "-t")) {
		tsec = atof(argv[2]);
		argv += 2;
		argc -= 2;
	}
	if (argc != 3) {
		fprintf(stderr, "usage: ixref_rx [-t SECONDS] IN OUT\n");
		return 1;
	}
	FILE *fi = fopen(argv[1], "rb");
	if (!fi)
		die("open input", 0);
	char magic[8];
	uint32_t n, cflags, blob_len;
	uint16_t nb, dev;
	struct ixg_rx_cfg cfg;
	if (fread(magic, 1, 8, fi) != 8 || memcmp(magic, "IXGRXIN1", 8))
		die("bad magic", 0);
	if (fread(&n, 4, 1, fi) != 1 || fread(&cflags, 4, 1, fi) != 1 || fread(&nb, 2, 1, fi) != 1 ||
	    fread(&dev, 2, 1, fi) != 1 || fread(cfg.rss_key, 1, 40, fi) != 40)
		die("short header", 0);
	cfg.flags = cflags;
	cfg.nb_rx_fgs = nb;
	cfg.dev_idx = dev;
	uint16_t *len = malloc(sizeof(uint16_t) * (n + 1));
	uint32_t *off = malloc(sizeof(uint32_t) * (n + 1));
	if (fread(len, 2, n, fi) != n || fread(off, 4, n, fi) != n || fread(&blob_len, 4, 1, fi) != 1)
		die("short arrays", 0);
	uint8_t *blob = malloc(blob_len + 1);
	if (fread(blob, 1, blob_len, fi) != blob_len)
		die("short blob", 0);
	char tag[4];
	uint8_t host_mac[6] = {0};
	uint32_t host_addr = 0;
	while (fread(tag, 1, 4, fi) == 4) {
		if (!memcmp(tag, "HOST", 4)) {
			uint16_t pad;
			if (fread(host_mac, 1, 6, fi) != 6 || fread(&pad, 2, 1, fi) != 1 || fread(&host_addr, 4, 1, fi) != 1)
				die("short host block", 0);
			continue;
		}
		if (memcmp(tag, "FDIR", 4))
			die("unknown input block", 0);
		uint16_t cpu, pad;
		if (fread(&n_fdir, 4, 1, fi) != 1 || fread(&cpu, 2, 1, fi) != 1 || fread(&pad, 2, 1, fi) != 1)
			die("short fdir header", 0);
		struct ixg_fdir_filter *ff = malloc(sizeof(*ff) * (n_fdir + 1));
		if (!ff || fread(ff, sizeof(*ff), n_fdir, fi) != n_fdir)
			die("short fdir filters", 0);
		fdir = ff;
		fdir_cpu = cpu;
	}
	fclose(fi);

	if (ref_ix_init())
		die("arch_prctl(ARCH_SET_GS)", 0);
	ref_set_host(host_mac, host_addr);
	uint8_t *mbuf = aligned_alloc(64, IXG_MBUF_STRIDE);
	struct ixg_rx_rec *recs = calloc(n + 1, sizeof(*recs));
	uint32_t *cs = calloc(n + 1, sizeof(*cs));
	uint8_t *cf = calloc(n + 1, 1);
	struct ixg_tcp_ext *ext = calloc(n + 1, sizeof(*ext));
	uint8_t *hdr = calloc(n + 1, 16);
	uint8_t *refl = calloc(n + 1, 1);
	uint8_t *outb = malloc(blob_len + 1);
	for (uint32_t i = 0; i < n; i++) {
		if (len[i] > IXG_MBUF_DATA_LEN || (uint64_t)off[i] + len[i] > blob_len)
			die("frame does not fit an mbuf", i);
		one(&cfg, blob + off[i], len[i], mbuf, &recs[i], &cs[i], &cf[i], i);
		ext[i] = th_ext;
		memcpy(hdr + 16 * (size_t)i, th_hdr, 16);
		refl[i] = reflected;
		memcpy(outb + off[i], after, len[i]);
	}
	FILE *fo = fopen(argv[2], "wb");
	if (!fo)
		die("open output", 0);
	fwrite("IXGRXOUT", 1, 8, fo);
	fwrite(&n, 4, 1, fo);
	fwrite(recs, sizeof(*recs), n, fo);
	fwrite(cs, 4, n, fo);
	fwrite(cf, 1, n, fo);
	fwrite("TCPX", 1, 4, fo);
	fwrite(ext, sizeof(*ext), n, fo);
	fwrite(hdr, 16, n, fo);
	fwrite("ICMP", 1, 4, fo);
	fwrite(refl, 1, n, fo);
	for (uint32_t i = 0; i < n; i++)
		fwrite(outb + off[i], 1, len[i], fo);
	fclose(fo);
	if (tsec > 0 && n > 0) {
		struct timespec t0, t1;
		uint64_t done = 0;
		double el = 0;
		clock_gettime(CLOCK_MONOTONIC, &t0);
		do {
			for (uint32_t i = 0; i < n; i++)
				one(&cfg, blob + off[i], len[i], mbuf, &recs[i], &cs[i], &cf[i], i);
			done += n;
			clock_gettime(CLOCK_MONOTONIC, &t1);
			el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
		} while (el < tsec);
		printf("{\"pkts\": %llu, \"seconds\": %.6f, \"ns_per_pkt\": %.3f}\n",
		       (unsigned long long)done, el, 1e9 * el / (double)done);
	}
	return 0;
}
