/*
 * harness_demux.c - drive the reference's PCB lookup over a demux case file.
 *
 * TEST INFRASTRUCTURE ONLY (builds oracle/_ref/ixref_demux; used by
 * tests/golden/make_golden.py to produce tests/golden/demux*.npz).
 *
 * For each frame whose RX record (produced by oracle/_ref/ixref_rx from the
 * reference's eth_input) is IXG_V_TCP, the frame's 4-tuple is looked up as
 * tcp_input does (dp/net/tcp_in.c:233-323, 500-510):
 *   - the active list fgs[fg]->active_tbl[pcb_bucket] and the flow group's
 *     tw_pcbs list run through the reference's own tcp_input_find_list
 *     (ref_tcpin.c), over hlists built in the file's list order;
 *   - [LISTEN] the listen walk is inline in tcp_input (:273-304) and cannot
 *     be called on its own; it is restated here, including the hlist loop
 *     variable keeping the last entry when no `break` runs (list.h:731-732);
 *   - [RST] the no-PCB outcome (:500-510) is restated: RST unless the
 *     segment carries TCP_RST.
 *
 * Groups: fgs[pkt->fg_id] (dp/net/ip.c:125) is restated as an index into the
 * file's lists: a local flow group fg_id - fg_base < nfg, or an outbound
 * group ETH_MAX_TOTAL_FG + cpu (cpu < n_out; the flow director's frames,
 * ethfg.c:502-505) at index nfg + cpu.
 *
 * Input (LE): "IXGDMXI2", u32 n, u32 fg_base, u32 nfg, u32 n_out, u32 n_listen,
 *   u32 n_active, u32 n_tw, u32 active_start[(nfg+n_out)*512+1],
 *   struct ixg_pcb_key active[n_active], u32 tw_start[nfg+n_out+1],
 *   struct ixg_pcb_key tw[n_tw], struct ixg_listen_key listen[n_listen],
 *   u16 len[n], u32 off[n], u32 blob_len, blob, struct ixg_rx_rec rec[n].
 * Output (LE): "IXGDMXOT", u32 n, struct ixg_demux_rec[n].
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ixgrx.h"
#include "ref_capture.h"

static void die(const char *m)
{
	fprintf(stderr, "ixref_demux: %s\n", m);
	exit(2);
}

static void *rd(FILE *f, size_t bytes)
{
	void *p = malloc(bytes ? bytes : 1);
	if (!p || (bytes && fread(p, 1, bytes, f) != bytes))
		die("short input");
	return p;
}

static uint32_t raw32(const uint8_t *p)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}

static struct ref_pcb *to_ref(const struct ixg_pcb_key *k, uint32_t s, uint32_t e)
{
	static struct ref_pcb buf[4096];
	if (e - s > 4096)
		die("list too long");
	for (uint32_t j = s; j < e; j++) {
		buf[j - s].remote_ip = k[j].remote_ip;
		buf[j - s].local_ip = k[j].local_ip;
		buf[j - s].remote_port = k[j].remote_port;
		buf[j - s].local_port = k[j].local_port;
	}
	return buf;
}

int main(int argc, char **argv)
{
	if (argc != 3) {
		fprintf(stderr, "usage: ixref_demux IN OUT\n");
		return 2;
	}
	FILE *fi = fopen(argv[1], "rb");
	if (!fi)
		die("open input");
	char magic[8];
	uint32_t h[7];
	if (fread(magic, 1, 8, fi) != 8 || memcmp(magic, "IXGDMXI2", 8) || fread(h, 4, 7, fi) != 7)
		die("bad header");
	uint32_t n = h[0], fg_base = h[1], nfg = h[2], nout = h[3], nl = h[4], na = h[5], ntw = h[6];
	const size_t ng = (size_t)nfg + nout;
	uint32_t *astart = rd(fi, (ng * IXG_PCB_BUCKETS + 1) * 4);
	struct ixg_pcb_key *act = rd(fi, (size_t)na * sizeof(*act));
	uint32_t *twstart = rd(fi, (ng + 1) * 4);
	struct ixg_pcb_key *tw = rd(fi, (size_t)ntw * sizeof(*tw));
	struct ixg_listen_key *lis = rd(fi, (size_t)nl * sizeof(*lis));
	uint16_t *len = rd(fi, (size_t)n * 2);
	uint32_t *off = rd(fi, (size_t)n * 4);
	uint32_t blen;
	if (fread(&blen, 4, 1, fi) != 1)
		die("short input");
	uint8_t *blob = rd(fi, blen);
	struct ixg_rx_rec *rec = rd(fi, (size_t)n * sizeof(*rec));
	fclose(fi);

	struct ixg_demux_rec *out = calloc(n ? n : 1, sizeof(*out));
	for (uint32_t i = 0; i < n; i++) {
		const struct ixg_rx_rec *r = &rec[i];
		out[i].kind = IXG_D_NONE;
		if (r->verdict != IXG_V_TCP)
			continue;
		const uint8_t *f = blob + off[i];
		uint32_t L = len[i], ihl = f[14] & 15, l4 = 14 + 4 * ihl;
		if (l4 + 4 > L)
			die("TCP record on a frame without ports");
		uint32_t src = raw32(f + 26), dst = raw32(f + 30);
		uint16_t sport = (uint16_t)((f[l4] << 8) | f[l4 + 1]), dport = (uint16_t)((f[l4 + 2] << 8) | f[l4 + 3]);
		uint32_t fg = r->fg_id >= IXG_ETH_MAX_TOTAL_FG ? nfg + (r->fg_id - IXG_ETH_MAX_TOTAL_FG)
							    : (uint32_t)r->fg_id - fg_base;
		if (r->fg_id >= IXG_ETH_MAX_TOTAL_FG ? r->fg_id - IXG_ETH_MAX_TOTAL_FG < nout : fg < nfg) {
			uint32_t a = fg * IXG_PCB_BUCKETS + r->pcb_bucket;
			uint32_t s = astart[a], e = astart[a + 1];
			int k = ref_find_list(to_ref(act, s, e), (int)(e - s), src, dst, sport, dport);
			if (k >= 0) {
				out[i].kind = IXG_D_ACTIVE;
				out[i].id = act[s + k].id;
				continue;
			}
			s = twstart[fg];
			e = twstart[fg + 1];
			k = ref_find_list(to_ref(tw, s, e), (int)(e - s), src, dst, sport, dport);
			if (k >= 0) {
				out[i].kind = IXG_D_TIMEWAIT;
				out[i].id = tw[s + k].id;
				continue;
			}
		}
		/* [LISTEN] tcp_in.c:273-304 */
		const struct ixg_listen_key *lp = NULL;
		for (uint32_t k = 0; k < nl; k++) {
			lp = &lis[k];
			if (lp->local_port == dport && (lp->local_ip == dst || lp->local_ip == 0))
				break;
		}
		if (lp) {
			out[i].kind = IXG_D_LISTEN;
			out[i].id = lp->id;
			continue;
		}
		/* [RST] tcp_in.c:500-510 */
		out[i].kind = (r->tcp_flags & 0x04) ? IXG_D_DROP : IXG_D_RESET;
	}
	FILE *fo = fopen(argv[2], "wb");
	if (!fo)
		die("open output");
	fwrite("IXGDMXOT", 1, 8, fo);
	fwrite(&n, 4, 1, fo);
	fwrite(out, sizeof(*out), n, fo);
	fclose(fo);
	return 0;
}
