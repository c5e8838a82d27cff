/*
 * ixgrx_oracle.c - CPU restatement of IX's RX per-packet transform.
 *
 * TEST INFRASTRUCTURE ONLY (see ixgrx_oracle.h). Every function cites the
 * reference file:line it restates (paths relative to /root/reference).
 * Pinned against golden vectors from the reference's own code
 * (the .npz files under tests/golden/, made by tests/golden/make_golden.py through
 * oracle/ref_harness) and against the public RSS verification vectors.
 *
 * Semantics that live in NIC silicon rather than in the tree (IX offloads
 * the IP/L4 checksum verdict and the RSS hash to the 82599) are stated in
 * DESIGN.md "NIC rules"; they are the same rules the harness applies, and
 * are marked [NIC] below.
 */
#include "ixgrx_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define FOLD_U32T(u) (((u) >> 16) + ((u)&0x0000ffffUL)) /* inc/lwip/lwip/inet_chksum.h:76 */
#define SWAP_BYTES_IN_WORD(w) ((((w)&0xff) << 8) | (((w)&0xff00) >> 8)) /* :70 */

static inline uint64_t ld64(const uint8_t *p)
{
	uint64_t v;
	memcpy(&v, p, 8);
	return v; /* x86-64 and gfx950 are little-endian, as the reference assumes */
}
static inline uint32_t ld32(const uint8_t *p)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}
static inline uint16_t ld16(const uint8_t *p)
{
	uint16_t v;
	memcpy(&v, p, 2);
	return v;
}
static inline uint16_t bswap16(uint16_t x) { return (uint16_t)((x >> 8) | (x << 8)); }

/*
 * chksum_internet (inc/asm/chksum.h:40-95): an adc chain over 8-byte LE
 * words (the carry threads through the loop because `dec` keeps CF), one
 * trailing adc $0, then 4/2/1-byte tails each with add+adc $0, a 64->32 fold
 * with one end-around carry, a 32->16 fold with one end-around carry, and
 * the complement. Restated step by step, carries included.
 */
uint16_t ixgo_chksum_internet(const uint8_t *buf, int len)
{
	uint64_t sum = 0;
	unsigned cf = 0; /* xorq clears CF */
	uint32_t n8 = (uint32_t)len >> 3;

	if (n8) {
		for (uint32_t i = 0; i < n8; i++) { /* 1: adcq (%1), %0 */
			uint64_t v = ld64(buf);
			uint64_t t = sum + v;
			unsigned c1 = t < sum;
			uint64_t t2 = t + cf;
			unsigned c2 = t2 < t;
			sum = t2;
			cf = c1 | c2;
			buf += 8;
		}
		sum += cf; /* adcq $0, %0 (carry-out provably 0) */
	}
	if ((uint32_t)len & 4) { /* 2: */
		uint64_t t = sum + ld32(buf);
		sum = t + (t < sum);
		buf += 4;
	}
	if ((uint32_t)len & 2) { /* 3: movzxw */
		uint64_t t = sum + ld16(buf);
		sum = t + (t < sum);
		buf += 2;
	}
	if ((uint32_t)len & 1) { /* 4: movzxb */
		uint64_t t = sum + *buf;
		sum = t + (t < sum);
	}
	/* 5: fold 64 -> 32 (addl + adcl $0) */
	uint32_t lo = (uint32_t)sum, hi = (uint32_t)(sum >> 32);
	uint32_t s32 = hi + lo;
	s32 += (s32 < lo);
	/* fold 32 -> 16 (shrl $16; addw; adcw $0) */
	uint16_t a = (uint16_t)(s32 >> 16), b = (uint16_t)s32;
	uint16_t w = (uint16_t)(a + b);
	w = (uint16_t)(w + (w < b));
	return (uint16_t)~w;
}

/*
 * lwip_standard_chksum, LWIP_CHKSUM_ALGORITHM 2 (dp/lwip/inet_chksum.c:158-198):
 * 16-bit adds into a u32, odd start address handled by byte-swapping.
 */
uint16_t ixgo_standard_chksum(const void *dataptr, int len)
{
	const uint8_t *pb = (const uint8_t *)dataptr;
	uint16_t t = 0;
	uint32_t sum = 0;
	int odd = ((uintptr_t)pb & 1);

	if (odd && len > 0) {
		((uint8_t *)&t)[1] = *pb++;
		len--;
	}
	const uint8_t *ps = pb;
	while (len > 1) {
		sum += ld16(ps);
		ps += 2;
		len -= 2;
	}
	if (len > 0)
		((uint8_t *)&t)[0] = *ps;
	sum += t;
	sum = FOLD_U32T(sum);
	sum = FOLD_U32T(sum);
	if (odd)
		sum = SWAP_BYTES_IN_WORD(sum);
	return (uint16_t)sum;
}

/*
 * inet_cksum_pseudo_partial_base (inet_chksum.c:398-440) over a single
 * PBUF_ROM pbuf {payload = seg, len = seg_len} -- the shape tcp_input_tmp
 * builds (dp/lwip/misc.c:61-62) -- with chksum_len = seg_len.
 */
static uint16_t pseudo_partial_base(const uint8_t *seg, uint16_t seg_len, uint8_t proto,
				    uint16_t proto_len, uint32_t acc)
{
	uint16_t chksum_len = seg_len;
	uint8_t swapped = 0;

	if (chksum_len > 0) { /* for (q = p; q && chksum_len > 0; q = q->next), one pbuf */
		uint16_t chklen = seg_len;
		if (chklen > chksum_len)
			chklen = chksum_len;
		acc += ixgo_standard_chksum(seg, chklen);
		acc = FOLD_U32T(acc);
		if (seg_len % 2 != 0) {
			swapped = 1 - swapped;
			acc = SWAP_BYTES_IN_WORD(acc);
		}
	}
	if (swapped)
		acc = SWAP_BYTES_IN_WORD(acc);
	acc += (uint32_t)bswap16((uint16_t)proto); /* htons on LE */
	acc += (uint32_t)bswap16(proto_len);
	acc = FOLD_U32T(acc);
	acc = FOLD_U32T(acc);
	return (uint16_t)~(acc & 0xffffUL);
}

/* inet_chksum_pseudo_partial (inet_chksum.c:454-472) */
uint16_t ixgo_pseudo_partial(const uint8_t *seg, uint16_t seg_len, uint8_t proto,
			     uint16_t proto_len, uint32_t src_raw, uint32_t dst_raw)
{
	uint32_t acc = (src_raw & 0xffffUL);
	acc += ((src_raw >> 16) & 0xffffUL);
	acc += (dst_raw & 0xffffUL);
	acc += ((dst_raw >> 16) & 0xffffUL);
	acc = FOLD_U32T(acc);
	acc = FOLD_U32T(acc);
	return pseudo_partial_base(seg, seg_len, proto, proto_len, acc);
}

/* ip6_chksum_pseudo_partial (inet_chksum.c:488-509) */
uint16_t ixgo_pseudo6_partial(const uint8_t *seg, uint16_t seg_len, uint8_t proto,
			      uint16_t proto_len, const uint8_t src[16], const uint8_t dst[16])
{
	uint32_t acc = 0;
	for (int k = 0; k < 4; k++) {
		uint32_t a = ld32(src + 4 * k);
		acc += (a & 0xffffUL);
		acc += ((a >> 16) & 0xffffUL);
		a = ld32(dst + 4 * k);
		acc += (a & 0xffffUL);
		acc += ((a >> 16) & 0xffffUL);
	}
	acc = FOLD_U32T(acc);
	acc = FOLD_U32T(acc);
	return pseudo_partial_base(seg, seg_len, proto, proto_len, acc);
}

/*
 * compute_toeplitz_hash (dp/net/tcp_api.c:581-604), bit-serial, generalised
 * from the fixed 12-byte input to n bytes (n = 36 for the IPv6 extension;
 * key bytes used: 4 + n).
 */
uint32_t ixgo_toeplitz(const uint8_t *key, const uint8_t *input, int n)
{
	uint32_t result = 0;
	uint32_t key_part = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) |
			    ((uint32_t)key[2] << 8) | key[3]; /* htonl(((u32 *)key)[0]) */
	for (int i = 0; i < n; i++) {
		for (int j = 128; j; j >>= 1) {
			if (input[i] & j)
				result ^= key_part;
			key_part <<= 1;
			if (key[i + 4] & j)
				key_part |= 1;
		}
	}
	return result;
}

/* crc32q (inc/ix/hash.h:35-39): CRC-32C, reflected poly 0x82F63B78, no
 * pre/post inversion, 8 operand bytes consumed least significant first. */
uint32_t ixgo_crc32c_u64(uint32_t crc, uint64_t val)
{
	for (int k = 0; k < 8; k++) {
		crc ^= (uint32_t)((val >> (8 * k)) & 0xff);
		for (int b = 0; b < 8; b++)
			crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
	}
	return crc;
}

/*
 * tcp_to_idx (inc/lwip/lwip/tcp_impl.h:381-387) with hash_crc32c_two/one
 * (inc/ix/hash.h:51-71). The address words are the raw network-order u32s;
 * the port word is the int expression (local_port << 16) | remote_port,
 * which sign-extends into the upper 32 bits of the crc32q operand when
 * local_port >= 0x8000.
 */
uint16_t ixgo_tcp_to_idx(uint32_t local_raw, uint32_t remote_raw, uint16_t local_port,
			 uint16_t remote_port)
{
	int idx = (int)ixgo_crc32c_u64(ixgo_crc32c_u64(IXG_PCB_HASH_SEED, (uint64_t)local_raw),
				       (uint64_t)remote_raw);
	int32_t word = (int32_t)(((uint32_t)local_port << 16) | remote_port);
	idx = (int)ixgo_crc32c_u64((uint32_t)idx, (uint64_t)(int64_t)word);
	idx &= IXG_PCB_BUCKETS - 1;
	return (uint16_t)idx;
}

/* ---- table-driven hashes (CPU-baseline fast mode) -------------------- */

/* Both hashes are GF(2)-affine in the 12 tuple bytes, so a byte table
 * T[pos][v] = {toeplitz contribution, crc contribution} reproduces them:
 * tuple byte order = Toeplitz input order (src ip, dst ip, sport, dport). */
struct hashtab {
	uint32_t toep[12][256];
	uint32_t crc[12][256];
	uint32_t crc_const;
};

/* crc stream position (0..23 = words w1 w2 w3 of tcp_to_idx) of tuple byte i */
static const int crc_pos[12] = {8, 9, 10, 11, 0, 1, 2, 3, 17, 16, 19, 18};

static uint32_t crc_stream(uint32_t seed, const uint8_t s[24])
{
	return ixgo_crc32c_u64(ixgo_crc32c_u64(ixgo_crc32c_u64(seed, ld64(s)), ld64(s + 8)), ld64(s + 16));
}

static void hashtab_build(struct hashtab *h, const uint8_t *key)
{
	uint8_t zero24[24] = {0};
	h->crc_const = crc_stream(IXG_PCB_HASH_SEED, zero24);
	for (int i = 0; i < 12; i++)
		for (int v = 0; v < 256; v++) {
			uint8_t in[12] = {0}, s[24] = {0};
			in[i] = (uint8_t)v;
			h->toep[i][v] = ixgo_toeplitz(key, in, 12);
			s[crc_pos[i]] = (uint8_t)v;
			if (i == 10 && (v & 0x80)) /* dport high byte: sign extension */
				memset(s + 20, 0xff, 4);
			h->crc[i][v] = crc_stream(0, s);
		}
}

/* ---- the per-frame transform ----------------------------------------- */

struct frame {
	const uint8_t *p;
	uint32_t len;
};
/* bytes at offsets >= L read as zero (DESIGN.md "bytes beyond L") */
static inline uint8_t B(const struct frame *f, uint32_t i) { return i < f->len ? f->p[i] : 0; }
static inline uint16_t B16(const struct frame *f, uint32_t i)
{
	return (uint16_t)((B(f, i) << 8) | B(f, i + 1));
}
static inline uint32_t Braw32(const struct frame *f, uint32_t i)
{
	return (uint32_t)B(f, i) | ((uint32_t)B(f, i + 1) << 8) | ((uint32_t)B(f, i + 2) << 16) |
	       ((uint32_t)B(f, i + 3) << 24);
}

static void set_drop(struct ixg_rx_rec *r, uint8_t v)
{
	r->verdict = v;
	r->l4_off = 0;
	r->l4_len = 0;
	r->pcb_bucket = IXG_NO_BUCKET;
	r->tcp_flags = 0;
}

/* the flow-director perfect filters of ixgo_rx_batch_fdir (ixg_rx_set_fdir) */
struct fdir_set {
	const struct ixg_fdir_filter *f;
	uint32_t n;
	uint16_t cpu_id;
};

static void rx_one(const struct ixg_rx_cfg *cfg, const struct hashtab *ht, const struct fdir_set *fd,
		   const uint8_t *frame, uint32_t L, struct ixg_rx_rec *r, uint32_t *csum, int work)
{
	struct frame fr = {frame, L}, *f = &fr;
	uint32_t rss = 0;
	uint16_t ip_res = 0xffff, l4_res = 0xffff;
	uint8_t flags = 0;
	int full = (work == IXGO_WORK_FULL);

	memset(r, 0, sizeof(*r));
	r->pcb_bucket = IXG_NO_BUCKET;

	uint16_t etype = B16(f, 12);                     /* ip.c:132 ethhdr->type */
	int v6 = (etype == 0x86DD) && (cfg->flags & IXG_F_IPV6);
	uint8_t vh = B(f, 14);
	uint32_t ihl = vh & 15, ver = vh >> 4;           /* inc/net/ip.h:84-90 LE bitfield */
	uint32_t ip_len = B16(f, 16);                    /* ip.c:82 */
	uint16_t ip_off = B16(f, 20);                    /* ip.c:78 */
	uint8_t proto = B(f, 23);
	int frag = (ip_off & 0x3FFF) != 0;               /* IP_OFFMASK | IP_MF */
	uint32_t l4 = 14 + ihl * 4;

	/* [NIC] the IPv4 header checksum is verified when the whole header is present */
	int hdr_ok = etype == 0x0800 && ver == 4 && ihl >= 5 && l4 <= L;
	if (full && hdr_ok) {
		ip_res = ixgo_chksum_internet(frame + 14, (int)(ihl * 4));
		flags |= IXG_RF_IP_CSUM_CHECKED | (ip_res == 0 ? IXG_RF_IP_CSUM_OK : 0);
	}

	/* [NIC] RSS Toeplitz over {src, dst, sport, dport}, non-fragmented IPv4
	 * TCP/UDP only (dp/drivers/common.c:116-134), ports present in the frame */
	uint8_t tup[36];
	int tup_n = 0;
	if (hdr_ok && !frag && (proto == 6 || proto == 17) && l4 + 4 <= L) {
		for (int i = 0; i < 8; i++)
			tup[i] = B(f, 26 + i);
		for (int i = 0; i < 4; i++)
			tup[8 + i] = B(f, l4 + i);
		tup_n = 12;
	} else if (v6 && L >= 58 && (B(f, 14) >> 4) == 6 && (B(f, 20) == 6 || B(f, 20) == 17)) {
		for (int i = 0; i < 32; i++)
			tup[i] = B(f, 22 + i);
		for (int i = 0; i < 4; i++)
			tup[32 + i] = B(f, 54 + i);
		tup_n = 36;
	}
	if (full && tup_n) {
		if (tup_n == 12 && ht) {
			for (int i = 0; i < 12; i++)
				rss ^= ht->toep[i][tup[i]];
		} else {
			rss = ixgo_toeplitz(cfg->rss_key, tup, tup_n);
		}
		flags |= IXG_RF_RSS;
	}
	/* fg_id = rx_fgs[rss & (nb_rx_fgs-1)].fg_id (ixgbe.c:329-335, init.c:456-462) */
	r->fg_id = (uint16_t)(cfg->dev_idx * IXG_ETH_MAX_NUM_FG + (rss & (uint32_t)(cfg->nb_rx_fgs - 1)));
	r->rss_hash = rss;
	/* [NIC] a flow-director perfect filter on the 4-tuple of an IPv4 TCP
	 * frame: FLM -> MBUF_INVALID_FG_ID (ixgbe.c:329-330) -> outbound_fg_idx()
	 * = ETH_MAX_TOTAL_FG + cpu_id (ethfg.c:504-505, ethfg.h:135-138) */
	if (fd && fd->n && hdr_ok && !frag && proto == 6 && l4 + 4 <= L) {
		const uint32_t src = Braw32(f, 26), dst = Braw32(f, 30);
		const uint16_t sp = B16(f, l4), dp = B16(f, l4 + 2);
		for (uint32_t k = 0; k < fd->n; k++)
			if (fd->f[k].src_ip == src && fd->f[k].dst_ip == dst && fd->f[k].src_port == sp &&
			    fd->f[k].dst_port == dp) {
				r->fg_id = (uint16_t)(IXG_ETH_MAX_TOTAL_FG + fd->cpu_id);
				flags |= IXG_RF_FDIR;
				break;
			}
	}

	/* [NIC] L4 checksum: TCP always, UDP when the checksum field is non-zero
	 * (RFC 768), over the IP-derived L4 length (what lwIP would pass as
	 * p->tot_len to inet_chksum_pseudo_partial) */
	int l4_checked = 0;
	if (full && hdr_ok && !frag && (proto == 6 || proto == 17) && ip_len >= ihl * 4 &&
	    14 + ip_len <= L) {
		uint32_t l4len = ip_len - ihl * 4;
		if ((proto == 6 && l4len >= 20) || (proto == 17 && l4len >= 8 && B16(f, l4 + 6) != 0)) {
			l4_res = ixgo_pseudo_partial(frame + l4, (uint16_t)l4len, proto, (uint16_t)l4len,
						     Braw32(f, 26), Braw32(f, 30));
			l4_checked = 1;
		}
	}
	uint32_t v6_plen = B16(f, 18);
	uint8_t v6_nh = B(f, 20);
	int v6_ok = v6 && L >= 54 && (B(f, 14) >> 4) == 6 && 54 + v6_plen <= L;
	if (full && v6_ok && ((v6_nh == 6 && v6_plen >= 20) || (v6_nh == 17 && v6_plen >= 8))) {
		l4_res = ixgo_pseudo6_partial(frame + 54, (uint16_t)v6_plen, v6_nh, (uint16_t)v6_plen,
					      frame + 22, frame + 38);
		l4_checked = 1; /* IPv6 UDP checksum is mandatory (RFC 8200 8.1) */
	}
	if (l4_checked)
		flags |= IXG_RF_L4_CSUM_CHECKED | (l4_res == 0 ? IXG_RF_L4_CSUM_OK : 0);
	r->flags = flags;

	/* the driver drops on the NIC verdict before eth_input (ixgbe.c:312-324,349) */
	if (!(cfg->flags & IXG_F_NO_CSUM_DROP)) {
		if ((flags & IXG_RF_IP_CSUM_CHECKED) && !(flags & IXG_RF_IP_CSUM_OK)) {
			set_drop(r, IXG_V_DROP_CSUM_IP);
			goto out;
		}
		if ((flags & IXG_RF_L4_CSUM_CHECKED) && !(flags & IXG_RF_L4_CSUM_OK)) {
			set_drop(r, IXG_V_DROP_CSUM_L4);
			goto out;
		}
	}

	/* eth_input (dp/net/ip.c:120-141) */
	if (etype == 0x0806) { /* ETHTYPE_ARP -> arp_input */
		r->verdict = IXG_V_ARP;
		r->l4_off = 14;
		r->l4_len = (uint16_t)(L >= 14 ? L - 14 : 0);
		goto out;
	}
	if (v6) {
		/* extension (DESIGN.md "IPv6"): the reference drops ethertype 0x86DD */
		if (!v6_ok) {
			set_drop(r, IXG_V_DROP_IP6);
			goto out;
		}
		l4 = 54;
		ip_len = v6_plen + 40; /* so that l4len below = payload length */
		ihl = 10;
		proto = v6_nh;
		if (proto != 6 && proto != 17) {
			set_drop(r, IXG_V_DROP_IP6);
			goto out;
		}
		goto l4_dispatch;
	}
	if (etype != 0x0800) {
		set_drop(r, IXG_V_DROP_ETHERTYPE);
		goto out;
	}
	/* ip_input (dp/net/ip.c:63-114) */
	if (!(14 + 20 <= L)) { set_drop(r, IXG_V_DROP_IP_SHORT); goto out; }  /* :68 */
	if (ver != 4) { set_drop(r, IXG_V_DROP_IP_VERSION); goto out; }       /* :71 */
	if (ihl < 5) { set_drop(r, IXG_V_DROP_IP_IHL); goto out; }            /* :74 */
	if (frag) { set_drop(r, IXG_V_DROP_IP_FRAG); goto out; }              /* :78 */
	if (ip_len < ihl * 4) { set_drop(r, IXG_V_DROP_IP_LEN); goto out; }   /* :85 */
	if (!(14 + ip_len <= L)) { set_drop(r, IXG_V_DROP_IP_TRUNC); goto out; } /* :87 */

l4_dispatch:;
	uint32_t l4len = ip_len - ihl * 4; /* ip.c:90 pktlen -= hdrlen */
	if (proto == 6) {
		/* tcp_input_tmp: pbuf len = (u16)(ip_len - ihl*4) (misc.c:61) */
		uint16_t plen = (uint16_t)l4len;
		if (plen < 20) { set_drop(r, IXG_V_DROP_TCP_SHORT); goto out; } /* tcp_in.c:189 */
		uint8_t doff = B(f, l4 + 12) >> 4;        /* TCPH_HDRLEN tcp_impl.h:195 */
		int inc = -(int)(doff * 4);                /* pbuf_header(p, -(hdrlen*4)) tcp_in.c:222 */
		if (inc != 0 && (uint16_t)(-inc) > plen) { /* pbuf.c:457-465,498-507 */
			set_drop(r, IXG_V_DROP_TCP_HDRLEN);
			goto out;
		}
		r->verdict = v6 ? IXG_V_TCP6 : IXG_V_TCP;
		r->l4_off = (uint16_t)(l4 + doff * 4);
		r->l4_len = (uint16_t)(plen - doff * 4);
		r->tcp_flags = B(f, l4 + 13) & 0x3F; /* TCPH_FLAGS, TCP_FLAGS = 0x3f (tcp_in.c:240) */
		if (!v6) /* idx = tcp_to_idx(dst, src, dest, src) after ntohs (tcp_in.c:230-233) */
			r->pcb_bucket = ht ? (uint16_t)0 : ixgo_tcp_to_idx(Braw32(f, 30), Braw32(f, 26),
									 B16(f, l4 + 2), B16(f, l4));
		if (!v6 && ht) {
			uint32_t c = ht->crc_const;
			uint8_t t12[12];
			for (int i = 0; i < 8; i++)
				t12[i] = B(f, 26 + i);
			for (int i = 0; i < 4; i++)
				t12[8 + i] = B(f, l4 + i);
			for (int i = 0; i < 12; i++)
				c ^= ht->crc[i][t12[i]];
			r->pcb_bucket = (uint16_t)(c & (IXG_PCB_BUCKETS - 1));
		}
		goto out;
	}
	if (proto == 17) {
		/* udp_input (dp/net/udp.c:53-89) */
		uint16_t ulen = B16(f, l4 + 4);
		if (!(l4 + ulen <= L)) { set_drop(r, IXG_V_DROP_UDP_LEN); goto out; } /* :59 */
		r->verdict = v6 ? IXG_V_UDP6 : IXG_V_UDP;
		r->l4_off = (uint16_t)(l4 + 8); /* data = mbuf_nextd(udphdr) :55 */
		r->l4_len = ulen;               /* usys_udp_recv(..., len, ...) :88 */
		goto out;
	}
	if (proto == 1 && !v6) {
		/* icmp_input (dp/net/icmp.c:78-115) with len = ip_len - ihl*4 (ip.c:102-104) */
		if ((int)l4len < 8) { set_drop(r, IXG_V_DROP_ICMP_SHORT); goto out; } /* :80 */
		uint16_t res = ixgo_chksum_internet(frame + l4, (int)l4len);
		if (full)
			l4_res = res;
		if (res) { set_drop(r, IXG_V_DROP_ICMP_CSUM); goto out; } /* :82 */
		if (B(f, l4) != 8) { set_drop(r, IXG_V_DROP_ICMP_TYPE); goto out; } /* :88-108 */
		r->verdict = IXG_V_ICMP_ECHO;
		r->l4_off = (uint16_t)l4;
		r->l4_len = (uint16_t)l4len;
		goto out;
	}
	set_drop(r, v6 ? IXG_V_DROP_IP6 : IXG_V_DROP_IP_PROTO); /* ip.c:106-107 */
out:
	if (csum)
		*csum = (uint32_t)ip_res | ((uint32_t)l4_res << 16);
}

/* aux residual for ICMP is defined by reaching icmp's checksum step even
 * when a NIC drop wins the verdict; recompute it here so the residual word
 * does not depend on IXG_F_NO_CSUM_DROP */
static void fix_icmp_residual(const uint8_t *frame, uint32_t L, uint32_t *csum)
{
	struct frame fr = {frame, L}, *f = &fr;
	if (B16(f, 12) != 0x0800 || L < 34)
		return;
	uint32_t ver = B(f, 14) >> 4, ihl = B(f, 14) & 15, ip_len = B16(f, 16);
	if (ver != 4 || ihl < 5 || (B16(f, 20) & 0x3FFF) || ip_len < ihl * 4 || 14 + ip_len > L ||
	    B(f, 23) != 1)
		return;
	uint32_t l4len = ip_len - ihl * 4;
	if (l4len < 8)
		return;
	uint16_t res = ixgo_chksum_internet(frame + 14 + ihl * 4, (int)l4len);
	*csum = (*csum & 0xffffu) | ((uint32_t)res << 16);
}

void ixgo_rx_one(const struct ixg_rx_cfg *cfg, const uint8_t *frame, uint32_t len,
		 struct ixg_rx_rec *rec, uint32_t *csum, int hash_mode, int work)
{
	static struct hashtab *ht_cache;
	static uint8_t ht_key[IXG_RSS_KEY_LEN];
	struct hashtab *ht = NULL;
	if (hash_mode == IXGO_HASH_TABLE) {
		if (!ht_cache) {
			ht_cache = (struct hashtab *)malloc(sizeof(*ht_cache));
			hashtab_build(ht_cache, cfg->rss_key);
			memcpy(ht_key, cfg->rss_key, IXG_RSS_KEY_LEN);
		} else if (memcmp(ht_key, cfg->rss_key, IXG_RSS_KEY_LEN)) {
			hashtab_build(ht_cache, cfg->rss_key);
			memcpy(ht_key, cfg->rss_key, IXG_RSS_KEY_LEN);
		}
		ht = ht_cache;
	}
	rx_one(cfg, ht, NULL, frame, len, rec, csum, work);
	if (csum && work == IXGO_WORK_FULL)
		fix_icmp_residual(frame, len, csum);
}

/* ---- batches ---------------------------------------------------------- */

struct job {
	const struct ixg_rx_cfg *cfg;
	const struct hashtab *ht;
	const uint8_t *base;
	const uint64_t *off;
	const uint16_t *len;
	void *const *mbufs;
	uint32_t stride, lo, hi;
	struct ixg_rx_rec *out;
	uint32_t *csum;
	int work;
	const struct fdir_set *fd;
};

static void *run_job(void *arg)
{
	struct job *j = (struct job *)arg;
	for (uint32_t i = j->lo; i < j->hi; i++) {
		const uint8_t *fr;
		uint32_t L;
		if (j->mbufs) {
			const uint8_t *m = (const uint8_t *)j->mbufs[i];
			size_t l;
			memcpy(&l, m, sizeof(l)); /* struct mbuf.len @0 (inc/ix/mbuf.h:73-74) */
			fr = m + IXG_MBUF_HEADER_LEN;
			L = (uint32_t)l;
		} else {
			fr = j->base + (j->off ? j->off[i] : (uint64_t)i * j->stride);
			L = j->len[i];
		}
		uint32_t *c = j->csum ? &j->csum[i] : NULL;
		rx_one(j->cfg, j->ht, j->fd, fr, L, &j->out[i], c, j->work);
		if (c && j->work == IXGO_WORK_FULL)
			fix_icmp_residual(fr, L, c);
	}
	return NULL;
}

static int run_batch(struct job *proto, uint32_t n, int threads, int hash_mode)
{
	struct hashtab *ht = NULL;
	if (hash_mode == IXGO_HASH_TABLE) {
		ht = (struct hashtab *)malloc(sizeof(*ht));
		if (!ht)
			return -12;
		hashtab_build(ht, proto->cfg->rss_key);
	}
	proto->ht = ht;
	if (threads <= 1) {
		proto->lo = 0;
		proto->hi = n;
		run_job(proto);
	} else {
		pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(*tid));
		struct job *jobs = (struct job *)calloc((size_t)threads, sizeof(*jobs));
		for (int t = 0; t < threads; t++) {
			jobs[t] = *proto;
			jobs[t].lo = (uint32_t)((uint64_t)n * t / threads);
			jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
			pthread_create(&tid[t], NULL, run_job, &jobs[t]);
		}
		for (int t = 0; t < threads; t++)
			pthread_join(tid[t], NULL);
		free(tid);
		free(jobs);
	}
	free(ht);
	return 0;
}

int ixgo_rx_batch(const struct ixg_rx_cfg *cfg, const uint8_t *base, const uint64_t *off,
		  const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out,
		  uint32_t *csum, int threads, int hash_mode, int work)
{
	struct job j = {cfg, NULL, base, off, len, NULL, stride, 0, 0, out, csum, work, NULL};
	return run_batch(&j, n, threads, hash_mode);
}

int ixgo_rx_batch_fdir(const struct ixg_rx_cfg *cfg, const uint8_t *base, const uint64_t *off,
		       const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out,
		       uint32_t *csum, int threads, int hash_mode, int work, const struct ixg_fdir_filter *filters,
		       uint32_t nf, uint16_t cpu_id)
{
	struct fdir_set fd = {filters, nf, cpu_id};
	struct job j = {cfg, NULL, base, off, len, NULL, stride, 0, 0, out, csum, work, &fd};
	return run_batch(&j, n, threads, hash_mode);
}

int ixgo_rx_batch_mbufs(const struct ixg_rx_cfg *cfg, void *const *mbufs, uint32_t n,
			struct ixg_rx_rec *out, int threads, int hash_mode, int work)
{
	struct job j = {cfg, NULL, NULL, NULL, NULL, mbufs, 0, 0, 0, out, NULL, work, NULL};
	return run_batch(&j, n, threads, hash_mode);
}

/* ---- PCB demux: tcp_input after the head ---------------- */

/* tcp_input_find_list (dp/net/tcp_in.c:122-143) over the list
 * ent[s..e) in list order: remote_port == tcphdr->src, local_port ==
 * tcphdr->dest (host order after tcp_in.c:230-231), remote_ip == current
 * source, local_ip == current destination (IP_PCB_IPVER_INPUT_MATCH is 1
 * without LWIP_IPV6, lwip/ip.h:99). */
static const struct ixg_pcb_key *find_list(const struct ixg_pcb_key *ent, uint32_t s, uint32_t e,
					   uint16_t src_port, uint16_t dst_port, uint32_t src_raw,
					   uint32_t dst_raw)
{
	for (uint32_t k = s; k < e; k++) {
		const struct ixg_pcb_key *pcb = &ent[k];
		if (pcb->remote_port == src_port && pcb->local_port == dst_port &&
		    pcb->remote_ip == src_raw && pcb->local_ip == dst_raw)
			return pcb;
	}
	return NULL;
}

void ixgo_demux_one(const struct ixg_demux_tables *t, uint32_t fg_base, const uint8_t *frame, uint32_t len,
		    const struct ixg_rx_rec *rec, struct ixg_demux_rec *out)
{
	memset(out, 0, sizeof(*out));
	out->kind = IXG_D_NONE;
	if (rec->verdict != IXG_V_TCP) /* only tcp_input_tmp's segments reach tcp_input (ip.c:93-96) */
		return;
	struct frame f = {frame, len};
	uint32_t ihl = B(&f, 14) & 15u, l4 = 14 + 4 * ihl;
	uint32_t src = Braw32(&f, 26), dst = Braw32(&f, 30);
	uint16_t sport = B16(&f, l4), dport = B16(&f, l4 + 2); /* ntohs, tcp_in.c:230-231 */
	/* cur_fg = fgs[pkt->fg_id] (ip.c:125): a local flow group, or for a frame
	 * the flow director steered, the CPU's outbound group ETH_MAX_TOTAL_FG +
	 * cpu_id (ethfg.c:502-505), stored after the local ones */
	uint32_t fg;
	if (rec->fg_id >= IXG_ETH_MAX_TOTAL_FG)
		fg = rec->fg_id - IXG_ETH_MAX_TOTAL_FG < t->n_out ? t->nfg + (rec->fg_id - IXG_ETH_MAX_TOTAL_FG) : ~0u;
	else
		fg = (uint32_t)rec->fg_id - fg_base < t->nfg ? (uint32_t)rec->fg_id - fg_base : ~0u;
	if (fg != ~0u) {
		/* active_tbl[idx] with idx = tcp_to_idx (tcp_in.c:233,249) */
		uint32_t a = fg * IXG_PCB_BUCKETS + rec->pcb_bucket;
		const struct ixg_pcb_key *pcb =
			find_list(t->active, t->active_start[a], t->active_start[a + 1], sport, dport, src, dst);
		if (pcb) {
			out->kind = IXG_D_ACTIVE; /* tcp_in.c:250-256 */
			out->id = pcb->id;
			return;
		}
		pcb = find_list(t->tw, t->tw_start[fg], t->tw_start[fg + 1], sport, dport, src, dst);
		if (pcb) {
			out->kind = IXG_D_TIMEWAIT; /* tcp_in.c:260-269 */
			out->id = pcb->id;
			return;
		}
	}
	/* tcp_in.c:273-304, SO_REUSE 0 (opt.h:1579), LWIP_IPV6 0 (opt.h:2016):
	 * hlist_for_each (inc/ix/list.h:731-732) assigns lpcb on every
	 * iteration, so a walk that never breaks leaves lpcb = the last entry */
	const struct ixg_listen_key *lpcb = NULL;
	for (uint32_t k = 0; k < t->n_listen; k++) {
		lpcb = &t->listen[k];
		if (lpcb->local_port == dport) {
			if (lpcb->local_ip == dst)
				break; /* exact match (:290-292) */
			else if (lpcb->local_ip == 0)
				break; /* ANY match (:293-300) */
		}
	}
	if (lpcb) {
		out->kind = IXG_D_LISTEN; /* tcp_in.c:317-323 */
		out->id = lpcb->id;
		return;
	}
	/* no PCB: tcp_rst unless the segment is itself a RST (tcp_in.c:500-510) */
	out->kind = (rec->tcp_flags & 0x04) ? IXG_D_DROP : IXG_D_RESET;
}

int ixgo_demux_batch(const struct ixg_demux_tables *t, uint32_t fg_base, const uint8_t *base, const uint64_t *off,
		     const uint16_t *len, uint32_t stride, uint32_t n, const struct ixg_rx_rec *rec,
		     struct ixg_demux_rec *out)
{
	for (uint32_t i = 0; i < n; i++) {
		uint64_t o = off ? off[i] : (uint64_t)i * stride;
		ixgo_demux_one(t, fg_base, base + o, len[i], &rec[i], &out[i]);
	}
	return 0;
}

/* ---- ICMP echo reflect (dp/net/icmp.c:44-71,88-91) -------------------------- */

/* For every frame whose record is IXG_V_ICMP_ECHO, what icmp_input's
 * ICMP_ECHO case leaves in the mbuf: hdr->type = ICMP_ECHOREPLY (:89), then
 * icmp_reflect (:44-71): Ethernet dhost = shost, shost = CFG.mac; IP dst =
 * src, src = hton32(CFG.host_addr) (the IP checksum is not recomputed: the
 * frame leaves with ol_flags 0); hdr->chksum = 0 then chksum_internet over
 * the ICMP length (the record's l4_len, ip_input's len). Returns the number
 * of frames rewritten. */
uint32_t ixgo_icmp_reflect_batch(uint8_t *base, const uint64_t *off, uint32_t stride, const struct ixg_rx_rec *rec,
				 uint32_t n, const uint8_t mac[6], uint32_t host_addr)
{
	uint32_t k = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (rec[i].verdict != IXG_V_ICMP_ECHO)
			continue;
		uint8_t *f = base + (off ? off[i] : (uint64_t)i * stride);
		uint8_t *h = f + rec[i].l4_off;
		h[0] = 0; /* ICMP_ECHOREPLY */
		memmove(f, f + 6, 6);
		memcpy(f + 6, mac, 6);
		memmove(f + 30, f + 26, 4);
		const uint32_t be = __builtin_bswap32(host_addr);
		memcpy(f + 26, &be, 4);
		h[2] = h[3] = 0;
		const uint16_t c = ixgo_chksum_internet(h, rec[i].l4_len);
		memcpy(h + 2, &c, 2);
		k++;
	}
	return k;
}

/* ---- TX: header build + checksums ------------------------ */

/* ---- the rest of the tcp_input head (tcp_in.c:230-241) --------------------- */

int ixgo_tcp_ext_batch(uint8_t *base, const uint64_t *off, uint32_t stride, const struct ixg_rx_rec *rec,
		       uint32_t n, uint32_t flags, struct ixg_tcp_ext *ext)
{
	for (uint32_t i = 0; i < n; i++) {
		struct ixg_tcp_ext *e = &ext[i];
		memset(e, 0, sizeof(*e));
		const uint8_t v = rec[i].verdict;
		if (v != IXG_V_TCP && v != IXG_V_TCP6)
			continue;
		uint8_t *f = base + (off ? off[i] : (uint64_t)i * stride);
		/* p->payload = the TCP header: after ip_input's ihl*4 (ip.c:95-98,
		 * tcp_input_tmp misc.c:61-62), or the extension's fixed 40 */
		uint8_t *t = f + (v == IXG_V_TCP ? 14u + 4u * (f[14] & 15u) : 54u);
		e->src_port = bswap16(ld16(t));     /* :230 */
		e->dst_port = bswap16(ld16(t + 2)); /* :231 */
		e->seqno = __builtin_bswap32(ld32(t + 4)); /* :236 */
		e->ackno = __builtin_bswap32(ld32(t + 8)); /* :237 */
		e->wnd = bswap16(ld16(t + 14));     /* :238 */
		/* :240-241: p->tot_len after the doff strip is the record's l4_len;
		 * TCP_FIN | TCP_SYN = 0x03 */
		e->tcplen = (uint16_t)(rec[i].l4_len + ((rec[i].tcp_flags & 0x03u) ? 1u : 0u));
		if (flags & IXG_TCPX_INPLACE) {
			/* the same fields written back in host order (:230-238) */
			memcpy(t, &e->src_port, 2);
			memcpy(t + 2, &e->dst_port, 2);
			memcpy(t + 4, &e->seqno, 4);
			memcpy(t + 8, &e->ackno, 4);
			memcpy(t + 14, &e->wnd, 2);
		}
	}
	return 0;
}

/*
 * in_pseudo + inet_chksum_pseudo (dp/lwip/inet_chksum.c:324-357): the seed
 * lwIP leaves in the TCP checksum field for the NIC:
 * in_pseudo(src, dst, hton32(proto + tot_len)) -- a 32-bit add/adc/adc $0
 * chain, one 16-bit fold, and a conditional subtract of 0xffff.
 */
uint16_t ixgo_pseudo_seed(uint32_t src_raw, uint32_t dst_raw, uint8_t proto, uint16_t tot_len)
{
	uint32_t c = __builtin_bswap32((uint32_t)proto + tot_len);
	uint64_t s = (uint64_t)src_raw + dst_raw + c; /* addl; adcl; adcl $0 */
	uint32_t sum = (uint32_t)s + (uint32_t)(s >> 32);
	sum = (sum & 0xffff) + (sum >> 16);
	if (sum > 0xffff)
		sum -= 0xffff;
	return (uint16_t)sum;
}

static void put16be(uint8_t *p, uint16_t v)
{
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}

/*
 * One TX frame (include/ixgrx.h struct ixg_tx_seg). Returns the frame length,
 * 0 for an invalid segment (proto not 6/17, a TCP segment shorter than its
 * 20-byte header, a datagram longer than 65535 bytes).
 *  - Ethernet: ip_send_one (dp/net/ip.c:198-213): dhost = dmac, shost =
 *    src_mac, type 0x0800.
 *  - TCP, tcp_output_packet (dp/net/tcp_api.c:791-812): vhl 0x45, tos/ttl
 *    from the pcb, len 20 + seg_len, id 0, off 0, proto 6, checksum 0,
 *    src/dst raw; the segment copied after it. The TCP checksum field
 *    (segment bytes 16..17) holds lwIP's seed inet_chksum_pseudo
 *    (inet_chksum.c:353-357). IXG_TX_OFFLOAD stops there (what the NIC is
 *    handed, tcp_api.c:815-817); otherwise [NIC] the IP checksum is
 *    chksum_internet of the header and the TCP checksum is the one's
 *    complement of the sum over the pseudo header and the segment, i.e.
 *    lwIP's inet_chksum_pseudo_partial with chksum_len = seg_len over the
 *    segment with the field zeroed.
 *  - UDP, udp_output (dp/net/udp.c:114-128) with ip_setup_header
 *    (dp/net/net.h:65-78): tos 0, ttl 64, proto 17, len 28 + seg_len, IP
 *    checksum by chksum_internet in software, UDP header {sport, dport,
 *    len 8 + seg_len, checksum 0}, then the payload.
 */
uint32_t ixgo_tx_one(const uint8_t *seg, const struct ixg_tx_seg *d, const uint8_t src_mac[6],
		     const uint8_t dmac[6], uint32_t flags, uint8_t *out)
{
	const int tcp = d->proto == 6, udp = d->proto == 17;
	const uint32_t l4 = (uint32_t)d->seg_len + (udp ? 8u : 0u);
	if ((!tcp && !udp) || (tcp && d->seg_len < 20) || 20u + l4 > 0xffffu)
		return 0;
	memcpy(out, dmac, 6);
	memcpy(out + 6, src_mac, 6);
	out[12] = 0x08;
	out[13] = 0x00;
	uint8_t *ip = out + 14;
	ip[0] = 0x45;
	ip[1] = tcp ? d->tos : 0;
	put16be(ip + 2, (uint16_t)(20u + l4));
	put16be(ip + 4, 0);
	put16be(ip + 6, 0);
	ip[8] = tcp ? d->ttl : 64;
	ip[9] = d->proto;
	ip[10] = ip[11] = 0;
	memcpy(ip + 12, &d->src_ip, 4);
	memcpy(ip + 16, &d->dst_ip, 4);
	uint8_t *l4p = ip + 20;
	if (udp) {
		put16be(l4p, d->src_port);
		put16be(l4p + 2, d->dst_port);
		put16be(l4p + 4, (uint16_t)l4);
		l4p[6] = l4p[7] = 0;
		memcpy(l4p + 8, seg, d->seg_len);
		uint16_t c = ixgo_chksum_internet(ip, 20);
		memcpy(ip + 10, &c, 2);
		return 14u + 20u + l4;
	}
	memcpy(l4p, seg, d->seg_len);
	if (flags & IXG_TX_OFFLOAD) {
		uint16_t s = ixgo_pseudo_seed(d->src_ip, d->dst_ip, 6, d->seg_len);
		memcpy(l4p + 16, &s, 2);
	} else {
		l4p[16] = l4p[17] = 0;
		uint16_t c = ixgo_pseudo_partial(l4p, d->seg_len, 6, d->seg_len, d->src_ip, d->dst_ip);
		memcpy(l4p + 16, &c, 2);
		uint16_t ic = ixgo_chksum_internet(ip, 20);
		memcpy(ip + 10, &ic, 2);
	}
	return 14u + 20u + l4;
}

int ixgo_tx_batch(const uint8_t *seg_buf, const struct ixg_tx_seg *segs, uint32_t n, const uint8_t src_mac[6],
		  const uint8_t *dmacs, uint32_t n_dmac, uint32_t flags, uint8_t *out, uint16_t *out_len)
{
	for (uint32_t i = 0; i < n; i++) {
		const struct ixg_tx_seg *d = &segs[i];
		if (d->dmac_idx >= n_dmac || (d->seg_off & 3) || (d->out_off & 15)) {
			out_len[i] = 0;
			continue;
		}
		out_len[i] = (uint16_t)ixgo_tx_one(seg_buf + d->seg_off, d, src_mac, dmacs + 6u * d->dmac_idx, flags,
						   out + d->out_off);
	}
	return 0;
}

/* ---- event records ---------------------------------------- */

/*
 * The usys descriptors of a batch, dense and in frame order (include/ixgrx.h
 * ixg_ev_batch_dev):
 *  - udp_input (dp/net/udp.c:81-88): the ip_tuple written over the frame
 *    start (IXG_EV_UDP_TUPLE), then usys_udp_recv(iomap(data), udp->len,
 *    iomap(id)) = BSYS_DESC_3ARG (inc/ix/syscall.h:121-123,360-365);
 *  - recv_a_pbuf (dp/net/tcp_api.c:133-147) for a segment delivered in order
 *    as one pbuf: usys_tcp_recv(handle, cookie, iomap(payload), len) =
 *    BSYS_DESC_4ARG (:124-126,416-420), handle = tcpapi_to_handle
 *    (:125-131): pcb mempool index | fg_id << 48.
 * iomap(p) = p + iomap_offset (inc/ix/mempool.h:259-263), here
 * iomap_base + frame offset + x. Returns the number of descriptors.
 */
uint32_t ixgo_ev_batch(uint8_t *base, const uint64_t *off, uint32_t stride, const struct ixg_rx_rec *rec,
		       const struct ixg_demux_rec *dmx, const struct ixg_ev_pcb *pcbs, uint32_t n_pcbs, uint32_t n,
		       uint64_t iomap_base, uint32_t flags, struct ixg_bsys_desc *ev, uint32_t *frame_idx)
{
	uint32_t k = 0;
	for (uint32_t i = 0; i < n; i++) {
		const struct ixg_rx_rec *r = &rec[i];
		const uint64_t o = off ? off[i] : (uint64_t)i * stride;
		const uint64_t fio = iomap_base + o;
		struct ixg_bsys_desc d;
		if (r->verdict == IXG_V_UDP) {
			d.sysnr = IXG_USYS_UDP_RECV;
			d.arga = fio + r->l4_off;
			d.argb = r->l4_len;
			d.argc = fio;
			d.argd = 0;
			if (flags & IXG_EV_UDP_TUPLE) {
				uint8_t *f = base + o;
				const uint8_t *u = f + r->l4_off - 8;
				uint32_t src = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
				uint32_t dst = ((uint32_t)f[30] << 24) | ((uint32_t)f[31] << 16) | ((uint32_t)f[32] << 8) | f[33];
				uint16_t sp = (uint16_t)((u[0] << 8) | u[1]), dp = (uint16_t)((u[2] << 8) | u[3]);
				memcpy(f, &src, 4); /* id->src_ip = ntoh32(iphdr->src_addr.addr) */
				memcpy(f + 4, &dst, 4);
				memcpy(f + 8, &sp, 2); /* id->src_port = ntoh16(udphdr->src_port) */
				memcpy(f + 10, &dp, 2);
			}
		} else if (r->verdict == IXG_V_TCP && dmx && dmx[i].kind == IXG_D_ACTIVE && r->l4_len > 0 &&
			   dmx[i].id < n_pcbs) {
			const struct ixg_ev_pcb *pc = &pcbs[dmx[i].id];
			d.sysnr = IXG_USYS_TCP_RECV;
			d.arga = (pc->pcb_idx & 0xffffffffffffull) | ((uint64_t)r->fg_id << 48);
			d.argb = pc->cookie;
			d.argc = fio + r->l4_off;
			d.argd = r->l4_len;
		} else {
			continue;
		}
		ev[k] = d;
		if (frame_idx)
			frame_idx[k] = i;
		k++;
	}
	return k;
}
