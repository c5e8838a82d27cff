/*
 * ix_echo_pipeline.c - the §8(f) rows chained through the C ABI, device
 * resident: an echoserver's replies are built by the TX kernel (what
 * tcp_output_packet + ip_send_one + the NIC's checksum offload do), then
 * received back as a loopback batch: RX + PCB demux in one pass (eth_input ..
 * tcp_input's lookup), the rest of the tcp_input head (seqno, ackno, wnd,
 * tcplen in host order), then the usys descriptors libix consumes
 * (recv_a_pbuf's usys_tcp_recv).
 *
 * Every connection i is ESTABLISHED on the receiving side; its PCB is placed
 * in the flow group and bucket its packets hash to, read off the RX records
 * (IX computes the same at connect time). Checks: every frame is a TCP frame
 * with both checksums verified, every segment demuxes to its own PCB, its
 * seqno/ackno/wnd/tcplen/ports are the ones the segment was built with, and
 * one USYS_TCP_RECV per segment carries that PCB's handle and cookie.
 *
 * build: gcc -O2 -Iinclude -I/opt/rocm/include examples/ix_echo_pipeline.c \
 *            -Lix_amd -lixgrx -L/opt/rocm/lib -lamdhip64 -o ix_echo_pipeline
 * run:   ./ix_echo_pipeline   (needs a GPU; exits 2 with a message without one)
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ixgrx.h"

#define N 4096u          /* connections, one reply segment each */
#define SEG 26u          /* 20-byte TCP header + 6 bytes of echo payload */
#define SLOT 64u         /* frame slots: 16-aligned, 60-byte frames */

static int fail(const char *what, int rc)
{
	fprintf(stderr, "%s: %d (%s)\n", what, rc, ixg_strerror(rc));
	return 2;
}

#define HIP(x)                                                         \
	do {                                                           \
		if ((x) != hipSuccess) {                               \
			fprintf(stderr, "%s failed\n", #x);            \
			return 1;                                      \
		}                                                      \
	} while (0)

static uint32_t rnd(uint64_t *s)
{
	*s ^= *s << 13;
	*s ^= *s >> 7;
	*s ^= *s << 17;
	return (uint32_t)*s;
}

int main(void)
{
	static const uint8_t ms_key[40] = {
		0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
		0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
		0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
	struct ixg_rx_cfg cfg;
	memset(&cfg, 0, sizeof(cfg));
	memcpy(cfg.rss_key, ms_key, 40);
	cfg.nb_rx_fgs = 128;
	void *ctx = NULL;
	int rc = ixg_rx_init(&cfg, 0, &ctx);
	if (rc)
		return fail("ixg_rx_init", rc);

	/* ---- the replies: TCP segments as lwIP hands them to tcp_output_packet */
	static uint8_t seg_buf[N * 28 + IXG_TAIL_PAD];
	static struct ixg_tx_seg segs[N];
	uint64_t s = 0x9e3779b97f4a7c15ull;
	for (uint32_t i = 0; i < N; i++) {
		uint8_t *t = seg_buf + 28u * i;
		uint16_t sport = (uint16_t)(1 + rnd(&s) % 65535), dport = 7; /* echo */
		t[0] = (uint8_t)(dport >> 8); /* the server's reply: from port 7 */
		t[1] = (uint8_t)dport;
		t[2] = (uint8_t)(sport >> 8);
		t[3] = (uint8_t)sport;
		for (int k = 4; k < 12; k++)
			t[k] = (uint8_t)rnd(&s); /* seq, ack */
		t[12] = 5 << 4;                  /* doff 5 */
		t[13] = 0x18;                    /* PSH|ACK */
		t[14] = 0x10;                    /* window */
		t[15] = 0x00;
		t[16] = t[17] = t[18] = t[19] = 0;
		for (int k = 20; k < (int)SEG; k++)
			t[k] = (uint8_t)('a' + k);
		segs[i].seg_off = 28u * i;
		segs[i].out_off = (uint64_t)SLOT * i;
		segs[i].src_ip = 0x0100000a;             /* 10.0.0.1, raw */
		segs[i].dst_ip = rnd(&s);                /* the clients */
		segs[i].seg_len = SEG;
		segs[i].proto = 6;
		segs[i].ttl = 64;
		segs[i].dmac_idx = (uint16_t)(i & 3);
	}
	const uint8_t smac[6] = {2, 0, 0, 0, 0, 1};
	uint8_t dmacs[4 * 6];
	for (int k = 0; k < 24; k++)
		dmacs[k] = (uint8_t)(0x10 + k);
	if ((rc = ixg_tx_set_macs(ctx, smac, dmacs, 4)))
		return fail("ixg_tx_set_macs", rc);

	void *d_seg, *d_segs, *d_frames, *d_len, *d_rec, *d_dmx, *d_pcbs, *d_ev, *d_idx, *d_cnt, *d_ext;
	HIP(hipMalloc(&d_seg, sizeof(seg_buf)));
	HIP(hipMalloc(&d_segs, sizeof(segs)));
	HIP(hipMalloc(&d_frames, (size_t)N * SLOT + IXG_TAIL_PAD));
	HIP(hipMalloc(&d_len, N * sizeof(uint16_t)));
	HIP(hipMalloc(&d_rec, N * sizeof(struct ixg_rx_rec)));
	HIP(hipMalloc(&d_dmx, N * sizeof(struct ixg_demux_rec)));
	HIP(hipMalloc(&d_pcbs, N * sizeof(struct ixg_ev_pcb)));
	HIP(hipMalloc(&d_ev, N * sizeof(struct ixg_bsys_desc)));
	HIP(hipMalloc(&d_idx, N * sizeof(uint32_t)));
	HIP(hipMalloc(&d_cnt, sizeof(uint32_t)));
	HIP(hipMalloc(&d_ext, N * sizeof(struct ixg_tcp_ext)));
	HIP(hipMemset(d_frames, 0, (size_t)N * SLOT + IXG_TAIL_PAD));
	HIP(hipMemcpy(d_seg, seg_buf, sizeof(seg_buf), hipMemcpyHostToDevice));
	HIP(hipMemcpy(d_segs, segs, sizeof(segs), hipMemcpyHostToDevice));

	/* ---- TX: frames as they go on the wire (checksums computed) */
	if ((rc = ixg_tx_batch_dev(ctx, d_seg, d_segs, N, d_frames, d_len, 0, NULL)))
		return fail("ixg_tx_batch_dev", rc);

	/* ---- RX of the same frames (loopback): records, to place the PCBs */
	struct ixg_rx_frames fr = {d_frames, NULL, d_len, SLOT, 0};
	if ((rc = ixg_rx_batch_dev(ctx, &fr, N, d_rec, NULL, NULL)))
		return fail("ixg_rx_batch_dev", rc);
	static struct ixg_rx_rec rec[N];
	HIP(hipMemcpy(rec, d_rec, sizeof(rec), hipMemcpyDeviceToHost));
	unsigned tcp_ok = 0;
	for (uint32_t i = 0; i < N; i++)
		tcp_ok += rec[i].verdict == IXG_V_TCP && (rec[i].flags & 0x0f) == 0x0f && rec[i].l4_len == SEG - 20;

	/* ---- the receiver's PCB lists: connection i = (remote = the frame's
	 * source, local = its destination), in the bucket its records name */
	const uint32_t nfg = cfg.nb_rx_fgs, rows = nfg * IXG_PCB_BUCKETS;
	uint32_t *start = calloc(rows + 1, sizeof(uint32_t)), *fill = calloc(rows, sizeof(uint32_t));
	struct ixg_pcb_key *act = calloc(N, sizeof(*act));
	uint32_t tw_start[129] = {0};
	if (!start || !fill || !act)
		return 1;
	for (uint32_t i = 0; i < N; i++)
		start[(rec[i].fg_id % 512u) * IXG_PCB_BUCKETS + rec[i].pcb_bucket + 1]++;
	for (uint32_t r = 0; r < rows; r++)
		start[r + 1] += start[r];
	for (uint32_t i = 0; i < N; i++) {
		const uint32_t row = (rec[i].fg_id % 512u) * IXG_PCB_BUCKETS + rec[i].pcb_bucket;
		struct ixg_pcb_key *k = &act[start[row] + fill[row]++];
		k->remote_ip = segs[i].src_ip;
		k->local_ip = segs[i].dst_ip;
		k->remote_port = 7;
		k->local_port = (uint16_t)((seg_buf[28u * i + 2] << 8) | seg_buf[28u * i + 3]);
		k->id = i;
	}
	struct ixg_demux_tables tabs = {nfg, 0, start, act, tw_start, NULL, NULL};
	if ((rc = ixg_demux_load(ctx, &tabs)))
		return fail("ixg_demux_load", rc);

	/* ---- RX + demux in one pass, then the usys descriptors */
	if ((rc = ixg_rx_demux_batch_dev(ctx, &fr, N, d_rec, d_dmx, NULL)))
		return fail("ixg_rx_demux_batch_dev", rc);
	/* the rest of the tcp_input head: what tcp_process reads from its context */
	if ((rc = ixg_tcp_ext_batch_dev(ctx, &fr, d_rec, N, d_ext, 0, NULL)))
		return fail("ixg_tcp_ext_batch_dev", rc);
	static struct ixg_ev_pcb pcbs[N];
	for (uint32_t i = 0; i < N; i++) {
		pcbs[i].pcb_idx = 1000u + i;           /* its pcb mempool index */
		pcbs[i].cookie = 0xc0c0000000000000ull | i;
	}
	HIP(hipMemcpy(d_pcbs, pcbs, sizeof(pcbs), hipMemcpyHostToDevice));
	const uint64_t iomap = 0x7f0000000000ull;
	if ((rc = ixg_ev_batch_dev(ctx, &fr, d_rec, d_dmx, d_pcbs, N, N, iomap, 0, d_ev, d_idx, d_cnt, NULL)))
		return fail("ixg_ev_batch_dev", rc);
	HIP(hipDeviceSynchronize());

	static struct ixg_demux_rec dmx[N];
	static struct ixg_bsys_desc ev[N];
	static uint32_t idx[N];
	uint32_t cnt = 0;
	HIP(hipMemcpy(dmx, d_dmx, sizeof(dmx), hipMemcpyDeviceToHost));
	HIP(hipMemcpy(&cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
	HIP(hipMemcpy(ev, d_ev, sizeof(ev), hipMemcpyDeviceToHost));
	HIP(hipMemcpy(idx, d_idx, sizeof(idx), hipMemcpyDeviceToHost));
	static struct ixg_tcp_ext ext[N];
	HIP(hipMemcpy(ext, d_ext, sizeof(ext), hipMemcpyDeviceToHost));
	unsigned own = 0, good_ev = 0, head_ok = 0;
	for (uint32_t i = 0; i < N; i++) {
		own += dmx[i].kind == IXG_D_ACTIVE && dmx[i].id == i;
		const uint8_t *t = seg_buf + 28u * i;
		const uint32_t seq = (uint32_t)t[4] << 24 | (uint32_t)t[5] << 16 | (uint32_t)t[6] << 8 | t[7];
		const uint32_t ack = (uint32_t)t[8] << 24 | (uint32_t)t[9] << 16 | (uint32_t)t[10] << 8 | t[11];
		head_ok += ext[i].seqno == seq && ext[i].ackno == ack && ext[i].wnd == 0x1000 &&
			   ext[i].tcplen == SEG - 20 && ext[i].src_port == 7 &&
			   ext[i].dst_port == ((uint32_t)t[2] << 8 | t[3]);
	}
	for (uint32_t k = 0; k < cnt && k < N; k++) {
		const uint32_t i = idx[k];
		const uint64_t handle = ((uint64_t)rec[i].fg_id << 48) | (1000u + i);
		good_ev += ev[k].sysnr == IXG_USYS_TCP_RECV && ev[k].arga == handle && ev[k].argb == pcbs[i].cookie &&
			   ev[k].argc == iomap + (uint64_t)SLOT * i + 54 && ev[k].argd == SEG - 20;
	}
	printf("tx=%u rx_tcp_csum_ok=%u demux_own_pcb=%u tcp_head=%u usys_tcp_recv=%u/%u\n", N, tcp_ok, own, head_ok,
	       good_ev, cnt);
	ixg_rx_fini(ctx);
	return (tcp_ok == N && own == N && head_ok == N && good_ev == N && cnt == N) ? 0 : 1;
}
