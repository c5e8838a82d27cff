/*
 * harness_ev.c - drive the reference's usys encoders over an event case file.
 *
 * TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ixref_ev; used by
 * tests/golden/make_golden_ev.py to produce tests/golden/ev.npz).
 *
 * For each frame, in order, with its RX record (from the reference's
 * eth_input, the tests/golden fixtures) and demux record:
 *   - IXG_V_UDP: [UDP] udp_input's tail (dp/net/udp.c:81-88, unbuildable
 *     here, restated): the ip_tuple written over the frame start, then the
 *     reference's usys_udp_recv(iomap(data), ntoh16(udp->len), iomap(id));
 *   - IXG_V_TCP, demux ACTIVE, payload > 0: [TCP] recv_a_pbuf
 *     (dp/net/tcp_api.c:133-147) for the segment as one pbuf: the
 *     reference's usys_tcp_recv(handle, cookie, iomap(payload), len), with
 *     tcpapi_to_handle's value restated (:125-131: pcb index | fg_id << 48).
 * iomap through the reference's mempool_pagemem_to_iomap with
 * iomap_offset = iomap_base - (frame buffer address).
 *
 * Input (LE): "IXGEVIN\0", u32 n, u32 n_pcbs, u64 iomap_base, u32 has_dmx,
 *   u32 blob_len, blob, u64 off[n], struct ixg_rx_rec rec[n],
 *   [struct ixg_demux_rec dmx[n]], struct ixg_ev_pcb pcbs[n_pcbs].
 * Output (LE): "IXGEVOT\0", u32 k, struct ixg_bsys_desc ev[k], u32 idx[k],
 *   u32 blob_len, blob (after the tuple writes).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ixgrx.h"
#include "ref_capture.h"

static void die(const char *m)
{
	fprintf(stderr, "ixref_ev: %s\n", m);
	exit(2);
}

static void *rd(FILE *f, size_t bytes)
{
	void *p = malloc(bytes ? bytes : 1);
	if (!p || (bytes && fread(p, 1, bytes, f) != bytes))
		die("short input");
	return p;
}

int main(int argc, char **argv)
{
	if (argc != 3)
		die("usage: ixref_ev IN OUT");
	FILE *fi = fopen(argv[1], "rb"), *fo = fopen(argv[2], "wb");
	if (!fi || !fo)
		die("open");
	char magic[8];
	uint32_t n, n_pcbs, has_dmx, blob_len;
	uint64_t iomap_base;
	if (fread(magic, 1, 8, fi) != 8 || memcmp(magic, "IXGEVIN", 8) || fread(&n, 4, 1, fi) != 1 ||
	    fread(&n_pcbs, 4, 1, fi) != 1 || fread(&iomap_base, 8, 1, fi) != 1 || fread(&has_dmx, 4, 1, fi) != 1 ||
	    fread(&blob_len, 4, 1, fi) != 1)
		die("header");
	uint8_t *blob = rd(fi, blob_len);
	uint64_t *off = rd(fi, (size_t)n * 8);
	struct ixg_rx_rec *rec = rd(fi, (size_t)n * sizeof(*rec));
	struct ixg_demux_rec *dmx = has_dmx ? rd(fi, (size_t)n * sizeof(*dmx)) : NULL;
	struct ixg_ev_pcb *pcbs = rd(fi, (size_t)n_pcbs * sizeof(*pcbs));
	if (ref_ix_init())
		die("arch_prctl");
	ref_ev_set_iomap(iomap_base - (uint64_t)(uintptr_t)blob);
	uint64_t (*ev)[5] = malloc((size_t)(n ? n : 1) * 40);
	uint32_t *idx = malloc((size_t)(n ? n : 1) * 4), k = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *f = blob + off[i];
		const struct ixg_rx_rec *r = &rec[i];
		if (r->verdict == IXG_V_UDP) {
			uint8_t *u = f + r->l4_off - 8;
			/* udp.c:81-85 */
			uint32_t s = ((uint32_t)f[26] << 24) | ((uint32_t)f[27] << 16) | ((uint32_t)f[28] << 8) | f[29];
			uint32_t d = ((uint32_t)f[30] << 24) | ((uint32_t)f[31] << 16) | ((uint32_t)f[32] << 8) | f[33];
			uint16_t sp = (uint16_t)((u[0] << 8) | u[1]), dp = (uint16_t)((u[2] << 8) | u[3]);
			uint16_t len = (uint16_t)((u[4] << 8) | u[5]);
			memcpy(f, &s, 4);
			memcpy(f + 4, &d, 4);
			memcpy(f + 8, &sp, 2);
			memcpy(f + 10, &dp, 2);
			ref_ev_udp((void *)(uintptr_t)ref_iomap(u + 8), len, (void *)(uintptr_t)ref_iomap(f), ev[k]);
		} else if (r->verdict == IXG_V_TCP && dmx && dmx[i].kind == IXG_D_ACTIVE && r->l4_len > 0 &&
			   dmx[i].id < n_pcbs) {
			const struct ixg_ev_pcb *pc = &pcbs[dmx[i].id];
			uint64_t handle = (pc->pcb_idx & 0xffffffffffffull) | ((uint64_t)r->fg_id << 48);
			ref_ev_tcp(handle, pc->cookie, (void *)(uintptr_t)ref_iomap(f + r->l4_off), r->l4_len, ev[k]);
		} else {
			continue;
		}
		idx[k++] = i;
	}
	fwrite("IXGEVOT", 1, 8, fo);
	fwrite(&k, 4, 1, fo);
	fwrite(ev, 40, k, fo);
	fwrite(idx, 4, k, fo);
	fwrite(&blob_len, 4, 1, fo);
	fwrite(blob, 1, blob_len, fo);
	fclose(fo);
	return 0;
}
