/*
 * harness_tx.c - drive the reference's TX frame builds over a TX case file.
 *
 * TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ixref_tx; used by
 * tests/golden/make_golden.py to produce tests/golden/tx.npz).
 *
 * For each struct ixg_tx_seg (include/ixgrx.h):
 *   - proto 6: [LWIP] the segment's checksum field is set to the seed lwIP's
 *     tcp_output_segment stores for the NIC (lwIP's tcp_out.c is not in the
 *     tree; the seed itself is the reference's inet_chksum_pseudo,
 *     ref_pseudo_seed), then the reference's tcp_output_packet + ip_send_one
 *     build the frame (ref_tcp_frame): the OFFLOAD frame. [NIC] The FULL
 *     frame adds what the NIC computes on PKT_TX_IP_CKSUM | PKT_TX_TCP_CKSUM:
 *     the reference's chksum_internet over the IP header and the reference's
 *     inet_chksum_pseudo_partial over the segment with its field zeroed.
 *   - proto 17: [UDP] ref_udp_frame (udp_output restated over the
 *     reference's ip_setup_header / chksum_internet / ip_send_one); OFFLOAD
 *     and FULL frames are the same.
 *   - anything else, or a TCP segment shorter than 20 bytes: length 0.
 *
 * Input (LE): "IXGTXIN\0", u32 n, u8 src_mac[6], u32 n_dmac,
 *   u8 dmac[n_dmac][6], struct ixg_tx_seg segs[n], u32 buf_len, buf.
 * Output (LE): "IXGTXOT\0", u32 n, then per segment u16 len_offload, bytes,
 *   u16 len_full, bytes.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ixgrx.h"
#include "ref_capture.h"

static void die(const char *m)
{
	fprintf(stderr, "ixref_tx: %s\n", m);
	exit(2);
}

static void *rd(FILE *f, size_t bytes)
{
	void *p = malloc(bytes ? bytes : 1);
	if (!p || (bytes && fread(p, 1, bytes, f) != bytes))
		die("short input");
	return p;
}

static void put(FILE *f, const void *p, size_t n)
{
	if (n && fwrite(p, 1, n, f) != n)
		die("write");
}

int main(int argc, char **argv)
{
	if (argc != 3)
		die("usage: ixref_tx IN OUT");
	FILE *fi = fopen(argv[1], "rb"), *fo = fopen(argv[2], "wb");
	if (!fi || !fo)
		die("open");
	char magic[8];
	if (fread(magic, 1, 8, fi) != 8 || memcmp(magic, "IXGTXIN", 8))
		die("magic");
	uint32_t n, n_dmac, buf_len;
	uint8_t src_mac[6];
	if (fread(&n, 4, 1, fi) != 1 || fread(src_mac, 1, 6, fi) != 6 || fread(&n_dmac, 4, 1, fi) != 1)
		die("header");
	uint8_t *dmac = rd(fi, (size_t)n_dmac * 6);
	struct ixg_tx_seg *segs = rd(fi, (size_t)n * sizeof(*segs));
	if (fread(&buf_len, 4, 1, fi) != 1)
		die("buf_len");
	uint8_t *buf = rd(fi, buf_len);
	if (ref_ix_init())
		die("arch_prctl");
	put(fo, "IXGTXOT", 8);
	put(fo, &n, 4);
	static uint8_t seg[65536], fr[2][65600];
	for (uint32_t i = 0; i < n; i++) {
		const struct ixg_tx_seg *d = &segs[i];
		uint32_t len[2] = {0, 0};
		if (d->dmac_idx >= n_dmac || d->seg_off + d->seg_len > buf_len)
			die("segment out of range");
		ref_tx_set_macs(src_mac, dmac + 6u * d->dmac_idx);
		memcpy(seg, buf + d->seg_off, d->seg_len);
		if (d->proto == 6 && d->seg_len >= 20) {
			uint16_t s = ref_pseudo_seed(d->src_ip, d->dst_ip, 6, d->seg_len);
			memcpy(seg + 16, &s, 2);
			len[0] = ref_tcp_frame(d->src_ip, d->dst_ip, d->tos, d->ttl, seg, d->seg_len, fr[0]);
			len[1] = len[0];
			memcpy(fr[1], fr[0], len[0]);
			if (len[1]) {
				uint8_t *ip = fr[1] + 14, *tcp = fr[1] + 34;
				tcp[16] = tcp[17] = 0;
				uint16_t c = ref_pseudo_partial(tcp, d->seg_len, 6, d->seg_len, d->src_ip, d->dst_ip);
				memcpy(tcp + 16, &c, 2);
				uint16_t ic = ref_chksum_internet(ip, 20);
				memcpy(ip + 10, &ic, 2);
			}
		} else if (d->proto == 17) {
			len[0] = ref_udp_frame(d->src_ip, d->dst_ip, d->src_port, d->dst_port, seg, d->seg_len, fr[0]);
			len[1] = len[0];
			memcpy(fr[1], fr[0], len[0]);
		}
		for (int k = 0; k < 2; k++) {
			uint16_t l = (uint16_t)len[k];
			put(fo, &l, 2);
			put(fo, fr[k], l);
		}
	}
	fclose(fo);
	return 0;
}
