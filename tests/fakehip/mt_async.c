/*
 * mt_async.c - TEST INFRASTRUCTURE ONLY. Many IX CPUs at once on the C host
 * library over the fake HIP runtime (fakehip.c), built three ways by the
 * Makefile (plain, ASan/UBSan, ThreadSanitizer) and run by
 * tests/test_hostpath_mt.py.
 *
 * Each thread is one IX CPU with its own context (the per-CPU model of
 * dp/core/ethqueue.c:117-149): it builds an arena of IX mbufs, optionally
 * registers it (zero copy), and drives ixg_rx_submit_mbufs / ixg_rx_poll in
 * 1..64-frame iterations, as examples/ix_async_loop.c does on the GPU, so
 * launch_open -> ixg_stage_launch -> ixg_launch_ds -> ixgrx_launch run on
 * all threads concurrently. Every returned (mbuf, record) pair is checked
 * against the oracle's record of that mbuf, in submission order. Some threads
 * also make synchronous ixg_rx_batch_mbufs calls and re-install flow-director
 * filters with batches in flight (ixg_rx_set_fdir quiesces the ring), and one
 * makes launches fail now and then (the retry path of a zero-copy batch).
 *
 * usage: mt_async THREADS FRAMES_PER_THREAD ROUNDS [zc=0|1] [fail=0|1]
 * exit 0 and "ok ..." on stdout when every record matched.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ixgrx.h"
#include "../../oracle/ixgrx_oracle.h"

void fakehip_set_cfg(const struct ixg_rx_cfg *cfg);
void fakehip_fail_launches(int k);

static const uint8_t rss_key[40] = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
				    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
				    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};

static struct ixg_rx_cfg g_cfg;
static uint32_t g_frames, g_rounds;
static int g_zc, g_fail;

struct worker {
	int id;
	pthread_t th;
	uint64_t checked, launches_failed;
	int rc;
	char msg[200];
};

static uint32_t rnd(uint64_t *s)
{
	*s ^= *s << 13;
	*s ^= *s >> 7;
	*s ^= *s << 17;
	return (uint32_t)(*s >> 11);
}

static void put16(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}

static uint32_t sum16(const uint8_t *p, size_t n)
{
	uint32_t s = 0;
	for (size_t i = 0; i + 1 < n; i += 2)
		s += ((uint32_t)p[i] << 8) | p[i + 1];
	if (n & 1)
		s += (uint32_t)p[n - 1] << 8;
	return s;
}

static uint16_t fold(uint32_t s)
{
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	return (uint16_t)s;
}

/* one frame: IPv4 TCP or UDP of a random size with valid checksums (some
 * broken), the Ethernet pad past ip_len filled with garbage, now and then
 * an ARP or a truncated frame */
static size_t make_frame(uint8_t *f, uint64_t *s)
{
	const uint32_t kind = rnd(s) % 16;
	static const uint16_t sizes[] = {60, 60, 60, 64, 90, 128, 590, 1514};
	size_t L = sizes[rnd(s) % 8];
	for (size_t i = 0; i < L; i++)
		f[i] = (uint8_t)rnd(s);
	f[12] = 0x08;
	f[13] = kind == 0 ? 0x06 : 0x00; /* ARP now and then */
	if (kind == 0)
		return L;
	const int udp = kind < 5;
	const size_t ihl = kind == 5 ? 6 : 5, l4 = 14 + 4 * ihl;
	size_t ip_len = L - 14 - (L == 60 ? 6 : rnd(s) % 4);
	if (ip_len < 4 * ihl + 20)
		ip_len = 4 * ihl + 20;
	f[14] = (uint8_t)(0x40 | ihl);
	put16(f + 16, (uint32_t)ip_len);
	f[20] = 0x40;
	f[21] = 0;
	f[23] = udp ? 17 : 6;
	put16(f + 24, 0);
	put16(f + 24, (uint16_t)~fold(sum16(f + 14, 4 * ihl)));
	const size_t l4len = ip_len - 4 * ihl;
	if (udp) {
		put16(f + l4 + 4, (uint32_t)l4len);
		put16(f + l4 + 6, 0);
	} else {
		f[l4 + 12] = 0x50;
		put16(f + l4 + 16, 0);
	}
	uint32_t ps = sum16(f + 26, 8) + f[23] + (uint32_t)l4len + sum16(f + l4, l4len);
	uint16_t ck = (uint16_t)~fold(ps);
	if (udp && ck == 0)
		ck = 0xffff;
	put16(f + l4 + (udp ? 6 : 16), ck);
	if (kind == 15)
		f[l4 + 1] ^= 1; /* a bad L4 checksum */
	if (kind == 14)
		L = 14 + ip_len - 2; /* truncated: ip_len past the frame */
	return L;
}

static void fail(struct worker *w, const char *m, uint64_t i)
{
	if (!w->rc) {
		w->rc = 1;
		snprintf(w->msg, sizeof(w->msg), "thread %d: %s (item %llu)", w->id, m, (unsigned long long)i);
	}
}

static void *work(void *arg)
{
	struct worker *w = (struct worker *)arg;
	uint64_t seed = 0x9e3779b97f4a7c15ull * (uint64_t)(w->id + 1);
	const uint32_t n = g_frames;
	const size_t bytes = (size_t)n * IXG_MBUF_STRIDE + IXG_TAIL_PAD + 4096;
	uint8_t *arena = (uint8_t *)aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095);
	void **ptrs = (void **)malloc((size_t)n * sizeof(void *));
	struct ixg_rx_rec *exp = (struct ixg_rx_rec *)malloc((size_t)n * sizeof(*exp));
	struct ixg_rx_rec *got = (struct ixg_rx_rec *)malloc((size_t)n * sizeof(*got));
	void **gm = (void **)malloc((size_t)n * sizeof(void *));
	if (!arena || !ptrs || !exp || !got || !gm) {
		fail(w, "out of memory", 0);
		return NULL;
	}
	memset(arena, 0, bytes);
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *mb = arena + (size_t)i * IXG_MBUF_STRIDE;
		size_t l = make_frame(mb + IXG_MBUF_HEADER_LEN, &seed);
		memcpy(mb, &l, sizeof(l));
		ptrs[i] = mb;
	}
	ixgo_rx_batch_mbufs(&g_cfg, ptrs, n, exp, 1, IXGO_HASH_TABLE, IXGO_WORK_FULL);
	void *ctx = NULL;
	int rc = ixg_rx_init(&g_cfg, 0, &ctx);
	struct ixg_rx_async_cfg ac = {IXG_ASYNC_DEF_FRAMES, IXG_ASYNC_DEF_BYTES, 0, 2, IXG_ASYNC_DIRECT};
	ac.batch_frames = 64u + rnd(&seed) % 2000u;
	ac.batch_bytes = 4096u + rnd(&seed) % (1u << 18);
	ac.depth = 1u + rnd(&seed) % 4u;
	if (!rc)
		rc = ixg_rx_async_init(ctx, &ac);
	if (!rc && g_zc)
		rc = ixg_rx_register_memory(ctx, arena, bytes);
	if (rc) {
		fail(w, ixg_strerror(rc), 0);
		return NULL;
	}
	for (uint32_t round = 0; round < g_rounds && !w->rc; round++) {
		uint32_t sub = 0, ret = 0;
		while (ret < n && !w->rc) {
			if (sub < n) {
				uint32_t k = 1u + rnd(&seed) % 64u;
				if (k > n - sub)
					k = n - sub;
				if (g_fail && w->id == 0 && rnd(&seed) % 64u == 0)
					fakehip_fail_launches(1);
				const int acc = ixg_rx_submit_mbufs(ctx, ptrs + sub, k);
				if (acc == -EIO) {
					w->launches_failed++; /* reported once; the frames stay accepted */
				} else if (acc < 0) {
					fail(w, ixg_strerror(acc), sub);
					break;
				} else {
					sub += (uint32_t)acc;
				}
			}
			if (w->id % 4 == 1 && rnd(&seed) % 256u == 0) {
				/* the connect path re-installs filters with batches in flight */
				const struct ixg_fdir_filter flt = {0x0a000001u + (uint32_t)w->id, 0x0a000002u, 40000, 80};
				const int r2 = ixg_rx_set_fdir(ctx, &flt, 1, (uint16_t)w->id);
				if (r2 == -EIO)
					w->launches_failed++;
				else if (r2) {
					fail(w, "set_fdir", ret);
					break;
				}
			}
			const int r = ixg_rx_poll(ctx, gm + ret, got + ret, n - ret, sub == n || rnd(&seed) % 8u == 0);
			if (r == -EIO) {
				w->launches_failed++;
				continue;
			}
			if (r < 0) {
				fail(w, ixg_strerror(r), ret);
				break;
			}
			ret += (uint32_t)r;
		}
		if (ixg_rx_async_pending(ctx) != 0)
			fail(w, "frames pending after the round", ret);
		for (uint32_t i = 0; i < n && !w->rc; i++) {
			if (gm[i] != ptrs[i])
				fail(w, "mbuf order", i);
			else if (memcmp(&got[i], &exp[i], sizeof(exp[i])))
				fail(w, "record differs from the oracle", i);
		}
		w->checked += n;
		if (w->id % 4 == 2 && !w->rc) {
			/* the synchronous pipelined path from the same thread */
			memset(got, 0, (size_t)n * sizeof(*got));
			const int r3 = ixg_rx_batch_mbufs(ctx, ptrs, n, got);
			if (r3 == -EIO)
				w->launches_failed++;
			else if (r3 || memcmp(got, exp, (size_t)n * sizeof(*got)))
				fail(w, "ixg_rx_batch_mbufs", 0);
		}
	}
	if (g_zc && !w->rc && ixg_rx_unregister_memory(ctx, arena))
		fail(w, "unregister", 0);
	ixg_rx_fini(ctx);
	free(arena);
	free(ptrs);
	free(exp);
	free(got);
	free(gm);
	return NULL;
}

int main(int argc, char **argv)
{
	if (argc < 4) {
		fprintf(stderr, "usage: %s THREADS FRAMES ROUNDS [zc=0|1] [fail=0|1]\n", argv[0]);
		return 2;
	}
	const int t = atoi(argv[1]);
	g_frames = (uint32_t)atoi(argv[2]);
	g_rounds = (uint32_t)atoi(argv[3]);
	for (int i = 4; i < argc; i++) {
		if (!strncmp(argv[i], "zc=", 3))
			g_zc = atoi(argv[i] + 3);
		else if (!strncmp(argv[i], "fail=", 5))
			g_fail = atoi(argv[i] + 5);
	}
	if (t < 1 || t > 64 || g_frames < 1)
		return 2;
	memset(&g_cfg, 0, sizeof(g_cfg));
	memcpy(g_cfg.rss_key, rss_key, 40);
	g_cfg.nb_rx_fgs = 128;
	fakehip_set_cfg(&g_cfg);
	struct worker *ws = (struct worker *)calloc((size_t)t, sizeof(*ws));
	for (int i = 0; i < t; i++) {
		ws[i].id = i;
		pthread_create(&ws[i].th, NULL, work, &ws[i]);
	}
	int bad = 0;
	uint64_t checked = 0, failed = 0;
	for (int i = 0; i < t; i++) {
		pthread_join(ws[i].th, NULL);
		if (ws[i].rc) {
			fprintf(stderr, "%s\n", ws[i].msg);
			bad = 1;
		}
		checked += ws[i].checked;
		failed += ws[i].launches_failed;
	}
	free(ws);
	if (bad)
		return 1;
	printf("ok threads=%d records=%llu failed_launches_reported=%llu\n", t, (unsigned long long)checked,
	       (unsigned long long)failed);
	return 0;
}
