/*
 * harness_bench.c - dp/ix's own RX path timed on host cores (bench.py's
 * cpu_baseline, kind "reference").
 *
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY (builds oracle/_ref/ixref_bench from
 * the reference's own objects; see oracle/Makefile). Nothing here is shipped
 * or called by the product path.
 *
 * What one packet costs on an IX core, as eth_process_recv runs it
 * (dp/core/ethqueue.c:117-149): the reference's eth_input (dp/net/ip.c:120-141)
 * -> ip_input (:63-114) -> tcp_input_tmp (dp/lwip/misc.c:57-67) -> the head of
 * tcp_input (dp/net/tcp_in.c:157-241): the length check, pbuf_header's doff
 * strip (the reference's dp/lwip/pbuf.c), the ports to host order and
 * tcp_to_idx (inc/lwip/lwip/tcp_impl.h:381-387). In the timed loop the mbufs
 * are pre-filled IX mbufs (2112-B elements: len at +0, data at +64,
 * inc/ix/mbuf.h:73-90) in an arena far larger than the caches, walked in
 * order; nothing is copied or zeroed per packet. The pbuf comes from the
 * stack rather than the per-CPU pbuf mempool, and the walk stops before the
 * PCB lookup (the GPU path's scope ends there too), so this is a lower bound
 * on IX's per-packet cost.
 *
 * Modes:
 *   ix    the above: IX with the NIC's checksum offload and RSS (the real
 *         deployment: ixgbe.c:312-335 takes the verdicts from the descriptor)
 *   full  + what the NIC does, in software, with the reference's functions:
 *         chksum_internet over the IP header (inc/asm/chksum.h:40-95),
 *         inet_chksum_pseudo_partial over the segment (dp/lwip/inet_chksum.c),
 *         compute_toeplitz_hash (dp/net/tcp_api.c:581-604) and the fg mask -
 *         the same work the GPU kernels do per frame
 *
 * P worker processes (one per core, each with its own %gs per-CPU block and
 * its own arena: IX's per-CPU model) run for SECONDS after a common start.
 *
 * usage: ixref_bench MODE PROCS SECONDS MBUFS_PER_PROC IN
 *   IN: the harness frame file (harness_main.c's "IXGRXIN1" format)
 * prints one JSON line: {"mode", "procs", "pkts", "seconds", "mpps",
 *   "ns_per_pkt_core", "checksum"}
 */
#define _GNU_SOURCE
#include <sched.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "../../include/ixgrx.h"
#include "ref_capture.h"

/* set in ref_ix.c's tcp_input_tmp: when non-NULL it runs instead of the
 * capture (frame start, L4 header, tcp_input_tmp's pbuf length) */
extern void (*ref_tcp_hook)(const uint8_t *frame, const uint8_t *tcphdr, uint16_t len);
void ref_eth_input_raw(void *mbuf);

static int full_mode;
static uint8_t rss_key[40];
static uint32_t fg_mask = 127;
static volatile uint64_t sink;
static uint64_t acc;

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

/* the tcp_input head (tcp_in.c:189, 221-233) over the reference's pbuf_header
 * and tcp_to_idx; in full mode also the NIC's work in the reference's code */
static void tcp_head(const uint8_t *f, const uint8_t *th, uint16_t len)
{
	uint16_t nl = 0;
	uint32_t h = len;
	if (len >= 20 && !ref_pbuf_header_rom(len, (int16_t)-((th[12] >> 4) * 4), &nl)) {
		uint16_t sport = (uint16_t)((th[0] << 8) | th[1]), dport = (uint16_t)((th[2] << 8) | th[3]);
		h = (uint32_t)ref_tcp_to_idx(raw32(f + 30), raw32(f + 26), dport, sport) ^ ((uint32_t)nl << 16) ^ th[13];
	}
	if (full_mode) {
		const uint8_t *ip = f + 14;
		const int ihl = (ip[0] & 15) * 4;
		h ^= ref_chksum_internet(ip, ihl);
		h ^= (uint32_t)ref_pseudo_partial(th, len, 6, len, raw32(f + 26), raw32(f + 30)) << 9;
		h ^= ref_toeplitz(rss_key, raw32(f + 26), raw32(f + 30), raw16(th), raw16(th + 2)) & fg_mask;
	}
	acc += h;
}

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void die(const char *m)
{
	fprintf(stderr, "ixref_bench: %s\n", m);
	exit(2);
}

int main(int argc, char **argv)
{
	if (argc != 6)
		die("usage: ixref_bench ix|full PROCS SECONDS MBUFS_PER_PROC IN");
	full_mode = !strcmp(argv[1], "full");
	const int procs = atoi(argv[2]);
	const double secs = atof(argv[3]);
	const uint32_t m = (uint32_t)atoi(argv[4]);
	if (procs < 1 || m < 1 || secs <= 0)
		die("bad arguments");
	FILE *fi = fopen(argv[5], "rb");
	if (!fi)
		die("open input");
	char magic[8];
	uint32_t n, cflags, blob_len;
	uint16_t nb, dev;
	if (fread(magic, 1, 8, fi) != 8 || memcmp(magic, "IXGRXIN1", 8) || fread(&n, 4, 1, fi) != 1 ||
	    fread(&cflags, 4, 1, fi) != 1 || fread(&nb, 2, 1, fi) != 1 || fread(&dev, 2, 1, fi) != 1 ||
	    fread(rss_key, 1, 40, fi) != 40 || n == 0)
		die("bad header");
	fg_mask = (uint32_t)nb - 1u;
	uint16_t *len = malloc(sizeof(uint16_t) * n);
	uint32_t *off = malloc(sizeof(uint32_t) * n);
	if (!len || !off || fread(len, 2, n, fi) != n || fread(off, 4, n, fi) != n || fread(&blob_len, 4, 1, fi) != 1)
		die("short arrays");
	uint8_t *blob = malloc(blob_len + 1);
	if (!blob || fread(blob, 1, blob_len, fi) != blob_len)
		die("short blob");
	fclose(fi);
	for (uint32_t i = 0; i < n; i++)
		if (len[i] > IXG_MBUF_DATA_LEN || (uint64_t)off[i] + len[i] > blob_len)
			die("frame does not fit an mbuf");

	cpu_set_t allowed;
	CPU_ZERO(&allowed);
	sched_getaffinity(0, sizeof(allowed), &allowed);
	int go[2], res[2];
	if (pipe(go) || pipe(res))
		die("pipe");
	for (int w = 0; w < procs; w++) {
		pid_t pid = fork();
		if (pid < 0)
			die("fork");
		if (pid)
			continue;
		/* worker w: the w-th CPU this process may use */
		int seen = 0;
		for (int c = 0; c < CPU_SETSIZE; c++)
			if (CPU_ISSET(c, &allowed) && seen++ == w) {
				cpu_set_t one;
				CPU_ZERO(&one);
				CPU_SET(c, &one);
				sched_setaffinity(0, sizeof(one), &one);
				break;
			}
		if (ref_ix_init())
			die("arch_prctl(ARCH_SET_GS)");
		ref_tcp_hook = tcp_head;
		uint8_t *arena = aligned_alloc(64, (size_t)m * IXG_MBUF_STRIDE);
		if (!arena)
			die("arena");
		memset(arena, 0, (size_t)m * IXG_MBUF_STRIDE);
		for (uint32_t k = 0; k < m; k++) {
			const uint32_t i = (k + (uint32_t)w * 7919u) % n;
			uint8_t *mb = arena + (size_t)k * IXG_MBUF_STRIDE;
			size_t l = len[i];
			memcpy(mb, &l, sizeof(l));
			memcpy(mb + IXG_MBUF_HEADER_LEN, blob + off[i], l);
		}
		for (uint32_t k = 0; k < m; k++) /* warm pass */
			ref_eth_input_raw(arena + (size_t)k * IXG_MBUF_STRIDE);
		char c;
		if (read(go[0], &c, 1) != 1)
			_exit(3);
		uint64_t done = 0;
		const double t0 = now();
		double el = 0;
		do {
			for (uint32_t k = 0; k < m; k++)
				ref_eth_input_raw(arena + (size_t)k * IXG_MBUF_STRIDE);
			done += m;
			el = now() - t0;
		} while (el < secs);
		sink = acc;
		double out[3] = {(double)done, el, (double)(acc & 0xffffffffu)};
		if (write(res[1], out, sizeof(out)) != (ssize_t)sizeof(out))
			_exit(4);
		_exit(0);
	}
	usleep(200000 + 20000 * procs); /* arenas built and warmed (workers block on the pipe) */
	char startbuf[4096];
	memset(startbuf, 1, sizeof(startbuf));
	if (write(go[1], startbuf, (size_t)procs) != procs)
		die("start");
	double pkts = 0, tmax = 0, ck = 0;
	for (int w = 0; w < procs; w++) {
		double out[3];
		if (read(res[0], out, sizeof(out)) != (ssize_t)sizeof(out))
			die("worker result");
		pkts += out[0];
		tmax = out[1] > tmax ? out[1] : tmax;
		ck += out[2];
	}
	int bad = 0;
	for (int w = 0; w < procs; w++) {
		int st;
		wait(&st);
		bad |= !WIFEXITED(st) || WEXITSTATUS(st);
	}
	if (bad)
		die("a worker failed");
	printf("{\"mode\": \"%s\", \"procs\": %d, \"pkts\": %.0f, \"seconds\": %.4f, \"mpps\": %.3f, "
	       "\"ns_per_pkt_core\": %.2f, \"mbufs_per_proc\": %u, \"checksum\": %.0f}\n",
	       full_mode ? "full" : "ix", procs, pkts, tmax, pkts / tmax / 1e6, 1e9 * tmax * procs / pkts, m, ck);
	return 0;
}
