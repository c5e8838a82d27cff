/*
 * ixgrx_async.c - the asynchronous, aggregating host path.
 *
 * IX's run loop hands at most eth_rx_max_batch (64) frames per sys_bpoll
 * iteration to eth_input (dp/core/ethqueue.c:71,117-149) and then moves on to
 * timers and TX (dp/core/syscall.c:187-196). A GPU round trip per 64 frames
 * would stall that loop for tens of microseconds. Here a context accumulates
 * the frames of many iterations into one staged batch and launches it when
 * it is full or its oldest frame has waited long enough; records come back
 * in submission order on a later poll. The loop never waits on the GPU.
 *
 * Polling reads each in-flight batch's completion word, written by a one-lane
 * kernel enqueued after the batch (ixgrx_stamp): a poll that finds nothing
 * makes no runtime call. (hipEventQuery per poll took the runtime's locks;
 * with 16 threads polling every 64 frames the threads slept on them: 17 ns
 * per frame in poll and loop gaps up to 31 ms) Runtime calls
 * are made only to launch a batch and to wait for one.
 *
 * A context owns a ring of `depth` batches (pinned staging, device image,
 * a stream, a completion word and its own defer state each):
 *
 *   FREE -> OPEN (frames gathered by submit) -> INFLIGHT (H2D + kernels +
 *   D2H enqueued) -> DONE (event complete, records being polled) -> FREE
 *
 * Batches open, launch and retire in ring order, so records are returned in
 * the order the frames were submitted.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/prctl.h>

#include "ixgrx_ctx.h"

enum { AS_FREE = 0, AS_OPEN, AS_INFLIGHT, AS_DONE };

struct ixg_abatch {
	int state;
	struct ixg_dstate ds;
	hipStream_t stream;
	uint32_t *h_done;    /* completion word (coherent pinned host memory):
	                        the stream's last operation stores `seq` to it */
	uint32_t seq;        /* launches of this batch slot */
	uint64_t t_open;     /* ns: when its first frame was gathered */
	uint32_t nabs;       /* frames read in place (registered memory) */
	uint32_t n, taken;   /* frames held, frames already returned by poll */
	size_t span;         /* gathered bytes (ixg_gather_mbufs) */
	size_t hi;           /* the furthest gathered frame's end (ixg_stage_finish) */
	size_t link;         /* bytes of the in-place frames (host-link reads) */
	uint8_t *h_buf, *d_buf;
	uint64_t *h_off;
	uint16_t *h_len;
	void **mbufs;
	struct ixg_rx_rec *h_rec, *d_rec;
	/* IXG_ASYNC_ICMP_REFLECT: the echo-request candidates (pinned) */
	uint32_t nic;
	uint32_t *h_ic_idx;
	uint64_t *h_ic_addr;
	int dead;            /* its reflect ran but the batch could not be completed
	                        (ixg_stage_launch -EPIPE): never launched again */
	/* where its frames' time goes (ixg_rx_async_stats' worst batch): ns */
	uint64_t t_launch, t_seen, t_gpu, wait_ns;
	uint64_t gap_max;    /* TSC ticks: longest interval outside the library while pending */
	uint64_t naps, nap_max; /* poll(wait)'s naps on it, the longest (ns) */
};

struct ixg_async {
	struct ixg_rx_async_cfg cfg;
	struct ixg_rx_async_stats st; /* the *_ns fields in TSC ticks until read */
	uint64_t tsc0, ns0;           /* calibration: a TSC reading and the clock with it */
	uint32_t head;       /* oldest batch not yet fully polled */
	uint32_t tail;       /* next batch to open */
	uint32_t count;      /* batches in the ring that are not FREE */
	int err;             /* a launch that failed after submit had accepted
	                        frames: reported (and cleared) by the next
	                        submit / poll / flush; the batch stays OPEN */
	size_t bytes_cap;    /* gathered-bytes capacity of a batch */
	uint64_t t_exit;     /* TSC: the last return from submit / poll (0: none yet) */
	/* the device's wall clock -> CLOCK_MONOTONIC ns: ns = ticks * gclk_mul + gclk_off
	 * (gclk_mul 0: unknown) */
	double gclk_mul, gclk_off;
	struct ixg_abatch b[IXG_ASYNC_MAX_DEPTH];
};

static uint64_t now_ns(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

/* the stats' clock: the TSC (a few ns per reading; converted to ns against
 * CLOCK_MONOTONIC over the context's lifetime when the stats are read) */
static inline uint64_t tsc(void)
{
#if defined(__x86_64__)
	return __builtin_ia32_rdtsc();
#else
	return now_ns();
#endif
}

static void batch_free(struct ixg_abatch *b)
{
	if (b->stream)
		hipStreamSynchronize(b->stream);
	ixg_dstate_free(&b->ds);
	hipHostFree(b->h_buf);
	hipHostFree(b->h_done);
	hipHostFree(b->h_rec);
	hipHostFree(b->h_ic_idx);
	hipHostFree(b->h_ic_addr);
	hipFree(b->d_buf);
	hipFree(b->d_rec);
	free(b->h_off);
	free(b->h_len);
	free(b->mbufs);
	if (b->stream)
		hipStreamDestroy(b->stream);
	memset(b, 0, sizeof(*b));
}

void ixg_async_free(struct ixg_ctx *c)
{
	struct ixg_async *a = c->async;
	if (!a)
		return;
	for (uint32_t k = 0; k < IXG_ASYNC_MAX_DEPTH; k++)
		batch_free(&a->b[k]);
	free(a);
	c->async = NULL;
}

static int batch_alloc(struct ixg_async *a, struct ixg_abatch *b)
{
	const uint32_t nf = a->cfg.batch_frames;
	const size_t bcap = IXG_STAGE_BYTES(a->bytes_cap, nf);
	HIPCHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
	/* the completion word and the stamp's device clock (ixgrx_stamp) */
	HIPCHK(hipHostMalloc((void **)&b->h_done, 4 * sizeof(uint32_t), hipHostMallocCoherent));
	memset(b->h_done, 0, 4 * sizeof(uint32_t));
	HIPCHK(hipMalloc((void **)&b->ds.d_present, IXG_PRESENT_WORDS * sizeof(uint32_t)));
	HIPCHK(hipMemset(b->ds.d_present, 0, IXG_PRESENT_WORDS * sizeof(uint32_t)));
	const int rc = ixg_dstate_reserve(&b->ds, ((size_t)nf + 63u) / 64u);
	if (rc)
		return rc;
	HIPCHK(hipHostMalloc((void **)&b->h_buf, bcap, hipHostMallocDefault));
	HIPCHK(hipHostMalloc((void **)&b->h_rec, (size_t)nf * sizeof(struct ixg_rx_rec), hipHostMallocDefault));
	if (!(a->cfg.flags & IXG_ASYNC_DIRECT)) {
		HIPCHK(hipMalloc((void **)&b->d_buf, bcap));
		HIPCHK(hipMalloc((void **)&b->d_rec, (size_t)nf * sizeof(struct ixg_rx_rec)));
	}
	if (a->cfg.flags & IXG_ASYNC_ICMP_REFLECT) {
		HIPCHK(hipHostMalloc((void **)&b->h_ic_idx, (size_t)nf * sizeof(uint32_t), hipHostMallocDefault));
		HIPCHK(hipHostMalloc((void **)&b->h_ic_addr, (size_t)nf * sizeof(uint64_t), hipHostMallocDefault));
	}
	b->h_off = (uint64_t *)malloc((size_t)nf * sizeof(uint64_t));
	b->h_len = (uint16_t *)malloc((size_t)nf * sizeof(uint16_t));
	b->mbufs = (void **)malloc((size_t)nf * sizeof(void *));
	if (!b->h_off || !b->h_len || !b->mbufs)
		return -ENOMEM;
	memset(b->h_buf, 0, bcap);
	return 0;
}

/* The device wall clock (the stamp's, wall_clock64) against CLOCK_MONOTONIC:
 * a stamp on batch 0's stream between two host clock readings, three times,
 * the tightest bracket kept. Its rate comes from the device attribute. On
 * failure the split reports no device time (gclk_mul 0). */
static void clock_calibrate(struct ixg_ctx *c, struct ixg_async *a)
{
	int khz = 0;
	if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0)
		return;
	struct ixg_abatch *b = &a->b[0];
	uint64_t best = ~0ull;
	double off = 0;
	const double mul = 1e6 / (double)khz;
	int ok = 1;
	for (int k = 0; k < 3 && ok; k++) {
		b->h_done[0] = 0;
		const uint64_t t0 = now_ns();
		ok = ixgrx_stamp(b->h_done, 0x7fffffffu, b->stream) == 0 && hipStreamSynchronize(b->stream) == hipSuccess;
		const uint64_t t1 = now_ns();
		const uint64_t g = (uint64_t)b->h_done[2] | ((uint64_t)b->h_done[3] << 32);
		ok = ok && __atomic_load_n(b->h_done, __ATOMIC_ACQUIRE) == 0x7fffffffu && g != 0;
		if (ok && t1 - t0 < best) {
			best = t1 - t0;
			off = (double)(t0 + (t1 - t0) / 2) - (double)g * mul;
		}
	}
	memset(b->h_done, 0, 4 * sizeof(uint32_t)); /* (the batch's first launch stores 1) */
	if (ok) {
		a->gclk_mul = mul;
		a->gclk_off = off;
	}
}

/* time outside the library: on entry to submit / poll, the interval since the
 * last return, charged to every pending batch */
static void entry_gap(struct ixg_async *a)
{
	if (!a->t_exit || !a->count)
		return;
	const uint64_t g = tsc() - a->t_exit;
	for (uint32_t k = 0, i = a->head; k < a->count; k++, i = (i + 1) % a->cfg.depth)
		if (g > a->b[i].gap_max)
			a->b[i].gap_max = g;
}

/* a batch's last frame was returned at t (ns): the window's worst batch so far? */
static void batch_returned(struct ixg_async *a, const struct ixg_abatch *b, uint64_t t)
{
	const uint64_t tot = t - b->t_open;
	if (tot <= a->st.worst_total_ns)
		return;
	a->st.worst_total_ns = tot;
	a->st.worst_open_ns = b->t_launch - b->t_open;
	uint64_t gpu = 0, vis = b->t_seen - b->t_launch;
	if (b->t_gpu >= b->t_launch && b->t_gpu <= b->t_seen) {
		gpu = b->t_gpu - b->t_launch;
		vis = b->t_seen - b->t_gpu;
	}
	a->st.worst_gpu_ns = gpu;
	a->st.worst_visible_ns = vis;
	a->st.worst_returned_ns = t - b->t_seen;
	a->st.worst_wait_ns = b->wait_ns;
	a->st.worst_outside_ns = b->gap_max; /* (ticks: converted when read) */
	a->st.worst_naps = b->naps;
	a->st.worst_nap_max_ns = b->nap_max;
}

/* the library saw batch b's completion word (its stamp's device clock: when
 * the stamp ran, in CLOCK_MONOTONIC ns; 0 when unknown) */
static void batch_seen(const struct ixg_async *a, struct ixg_abatch *b)
{
	b->t_seen = now_ns();
	b->t_gpu = 0;
	if (a->gclk_mul > 0) {
		const uint64_t g = (uint64_t)b->h_done[2] | ((uint64_t)b->h_done[3] << 32);
		const double t = (double)g * a->gclk_mul + a->gclk_off;
		b->t_gpu = t > 0 ? (uint64_t)t : 0;
	}
}

int ixg_rx_async_init(void *vctx, const struct ixg_rx_async_cfg *cfg)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return -EINVAL;
	struct ixg_rx_async_cfg k = {IXG_ASYNC_DEF_FRAMES, IXG_ASYNC_DEF_BYTES, IXG_ASYNC_DEF_WAIT_US,
				     IXG_ASYNC_DEF_DEPTH, IXG_ASYNC_DEF_FLAGS};
	if (cfg)
		k = *cfg;
	if (k.batch_frames == 0 || k.batch_frames > (1u << 20) || k.batch_bytes < 4096u ||
	    k.batch_bytes > (256u << 20) || k.depth < 1 || k.depth > IXG_ASYNC_MAX_DEPTH ||
	    (k.flags & ~(uint32_t)(IXG_ASYNC_DIRECT | IXG_ASYNC_ICMP_REFLECT)))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (c->async) {
		/* re-configuring: only with nothing submitted and not yet polled */
		if (c->async->count)
			return -EBUSY;
		ixg_async_free(c);
	}
	struct ixg_async *a = (struct ixg_async *)calloc(1, sizeof(*a));
	if (!a)
		return -ENOMEM;
	a->cfg = k;
	a->tsc0 = tsc();
	a->ns0 = now_ns();
	/* a batch can always take one more frame of the largest size */
	a->bytes_cap = (size_t)k.batch_bytes + IXG_MBUF_DATA_LEN;
	c->async = a;
	for (uint32_t i = 0; i < k.depth; i++) {
		int rc = batch_alloc(a, &a->b[i]);
		if (rc) {
			ixg_async_free(c);
			return rc;
		}
	}
	clock_calibrate(c, a);
	return 0;
}

/* launch the OPEN batch (if any): one H2D image, the kernels, the records
 * back (or, IXG_ASYNC_DIRECT, kernels reading and writing pinned memory) */
static int launch_open(struct ixg_ctx *c, struct ixg_async *a)
{
	if (!a->count)
		return 0;
	const uint32_t last = (a->tail + a->cfg.depth - 1) % a->cfg.depth;
	struct ixg_abatch *b = &a->b[last];
	if (b->state != AS_OPEN)
		return 0;
	if (b->dead)
		return -EIO;
	HIPCHK(hipSetDevice(c->device));
	struct ixg_stage st;
	if (b->nabs)
		ixg_stage_finish_abs(b->h_buf, b->span, b->hi, b->h_off, b->h_len, b->n, &st);
	else
		ixg_stage_finish(b->h_buf, b->span, b->hi, b->h_off, b->h_len, b->n, &st);
	const int direct = (a->cfg.flags & IXG_ASYNC_DIRECT) != 0;
	const uint64_t t0 = tsc();
	const struct ixg_icmp_items ic = {b->nic, b->h_ic_idx, b->h_ic_addr};
	int rc = ixg_stage_launch(c, &b->ds, &st, b->h_buf, b->d_buf, b->n, b->d_rec, b->h_rec, direct, &ic,
				  b->h_done, b->seq + 1u, b->stream);
	if (rc == 0)
		b->seq++;
	const uint64_t dt = tsc() - t0;
	a->st.launch_ns += dt;
	if (dt > a->st.launch_max_ns)
		a->st.launch_max_ns = dt;
	if (rc == -EPIPE) {
		b->dead = 1;
		return -EIO;
	}
	if (rc)
		return rc;
	b->state = AS_INFLIGHT;
	b->t_launch = now_ns();
	a->st.batches++;
	a->st.image_bytes += st.h2d;
	a->st.inplace_bytes += b->link;
	a->st.frames_launched += b->n;
	if (b->n < a->cfg.batch_frames && b->span + b->link < a->cfg.batch_bytes)
		a->st.batches_by_time++;
	return 0;
}

/* the batch frames go into: the OPEN one, or a FREE one opened now; NULL
 * when every batch of the ring is in flight or not yet polled */
static struct ixg_abatch *open_batch(struct ixg_async *a, uint64_t t)
{
	if (a->count) {
		struct ixg_abatch *b = &a->b[(a->tail + a->cfg.depth - 1) % a->cfg.depth];
		if (b->state == AS_OPEN)
			return b;
	}
	if (a->count == a->cfg.depth)
		return NULL;
	struct ixg_abatch *b = &a->b[a->tail];
	b->state = AS_OPEN;
	b->t_open = t;
	b->n = b->taken = 0;
	b->nabs = b->nic = 0;
	b->span = b->hi = b->link = 0;
	b->dead = 0;
	b->wait_ns = b->gap_max = b->naps = b->nap_max = 0;
	a->tail = (a->tail + 1) % a->cfg.depth;
	a->count++;
	return b;
}

/* batch_bytes counts the bytes the kernels read over the host link: the
 * staged ones and the in-place frames' (a zero-copy batch of 1514-B frames
 * that counted only its ~10 staged bytes per frame closed at 16384 frames,
 * 25 MB of link reads, and queued its frames for 12 ms at 16 threads) */
/* IXG_ASYNC_ICMP_REFLECT: frames k0..k0+n-1 of batch b that may be echo
 * requests (IPv4, protocol 1; the parse decides) and whose mbufs lie in a
 * registered region become the batch's reflect candidates (a frame outside
 * every region is left to the host's icmp_reflect: its record has no
 * IXG_RF_REPLY) */
static void icmp_candidates(const struct ixg_ctx *c, struct ixg_abatch *b, uint32_t k0, uint32_t n)
{
	for (uint32_t k = k0; k < k0 + n; k++) {
		const uint8_t *mb = (const uint8_t *)b->mbufs[k];
		const uint8_t *f = mb + IXG_MBUF_HEADER_LEN;
		if (b->h_len[k] < 34 || f[12] != 0x08 || f[13] != 0x00 || (f[14] >> 4) != 4 || f[23] != 1)
			continue;
		const uintptr_t a = (uintptr_t)mb;
		for (uint32_t r = 0; r < c->nreg; r++)
			if (a >= c->reg[r].lo && a + IXG_MBUF_STRIDE <= c->reg[r].hi) {
				b->h_ic_idx[b->nic] = k;
				b->h_ic_addr[b->nic] = (uint64_t)(a + IXG_MBUF_HEADER_LEN) + (uint64_t)c->reg[r].delta;
				b->nic++;
				break;
			}
	}
}

static int due(const struct ixg_async *a, const struct ixg_abatch *b, uint64_t t)
{
	return b->n >= a->cfg.batch_frames || b->span + b->link >= a->cfg.batch_bytes ||
	       t - b->t_open >= (uint64_t)a->cfg.max_wait_us * 1000u;
}

int ixg_rx_submit_mbufs(void *vctx, void *const *mbufs, uint32_t n)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && !mbufs))
		return -EINVAL;
	if (!c->async) {
		int rc = ixg_rx_async_init(c, NULL);
		if (rc)
			return rc;
	}
	if (ixg_check_mbufs(mbufs, n))
		return -EINVAL;
	struct ixg_async *a = c->async;
	if (a->err) {
		const int e = a->err;
		a->err = 0;
		return e;
	}
	entry_gap(a);
	const uint64_t t = now_ns();
	uint32_t done = 0;
	a->st.submit_calls++;
	while (done < n) {
		struct ixg_abatch *b = open_batch(a, t);
		if (!b)
			break; /* back-pressure: the caller polls, then submits the rest */
		/* frames that fit the batch's count and byte limits (the last one
		 * may pass the byte limit: bytes_cap leaves room for it) */
		uint32_t m = 0;
		const uint64_t g0 = tsc();
		while (done + m < n && b->n + m < a->cfg.batch_frames && b->span + b->link < a->cfg.batch_bytes) {
			/* at most as many frames as can still start below batch_bytes
			 * (each stages or reads at most IXG_MBUF_DATA_LEN - 12 bytes) */
			const size_t room = (a->cfg.batch_bytes - b->span - b->link) / (IXG_MBUF_DATA_LEN - 12u) + 1u;
			uint32_t step = n - done - m < 16u ? n - done - m : 16u;
			if (step > room)
				step = (uint32_t)room;
			const uint32_t take = a->cfg.batch_frames - b->n - m < step ? a->cfg.batch_frames - b->n - m : step;
			if (c->nreg && (a->cfg.flags & IXG_ASYNC_DIRECT))
				b->span = ixg_gather_mbufs_zc(c, b->h_buf, b->span, mbufs + done + m, take, n - done - m,
							      b->h_off + b->n + m, b->h_len + b->n + m, &b->hi, &b->nabs,
							      &b->link);
			else
				b->span = ixg_gather_mbufs(b->h_buf, b->span, mbufs + done + m, take, n - done - m,
							   b->h_off + b->n + m, b->h_len + b->n + m, &b->hi);
			memcpy(b->mbufs + b->n + m, mbufs + done + m, (size_t)take * sizeof(void *));
			if ((a->cfg.flags & IXG_ASYNC_ICMP_REFLECT) && c->nreg)
				icmp_candidates(c, b, b->n + m, take);
			m += take;
		}
		a->st.gather_ns += tsc() - g0;
		b->n += m;
		done += m;
		if (due(a, b, t)) {
			int rc = launch_open(c, a);
			if (rc) {
				/* the accepted frames stay in the OPEN batch (owned by the
				 * library until poll returns them; a later flush, submit or
				 * poll launches it again): report the count now and the
				 * error on the next call */
				a->err = rc;
				break;
			}
		}
	}
	a->st.frames_submitted += done;
	a->st.frames_refused += n - done;
	a->t_exit = tsc();
	return (int)done;
}

int ixg_rx_flush(void *vctx)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return -EINVAL;
	if (!c->async)
		return 0;
	struct ixg_async *a = c->async;
	if (a->err) {
		const int e = a->err;
		a->err = 0;
		return e;
	}
	return launch_open(c, a);
}

int ixg_async_quiesce(struct ixg_ctx *c)
{
	struct ixg_async *a = c->async;
	if (!a || !a->count)
		return 0;
	/* the OPEN batch goes now, with the state its frames were submitted under;
	 * once it is launched, an earlier failed launch of it is not reported
	 * again (its frames are in flight) */
	int rc = launch_open(c, a);
	if (rc)
		return rc;
	a->err = 0;
	for (uint32_t k = 0, i = a->head; k < a->count; k++, i = (i + 1) % a->cfg.depth)
		if (a->b[i].state == AS_INFLIGHT) {
			HIPCHK(hipSetDevice(c->device));
			HIPCHK(hipStreamSynchronize(a->b[i].stream));
		}
	return 0;
}

/* Block until batch b's completion word holds its sequence number: a short
 * spin, then naps that give the CPU away. On the GPU box (a cgroup quota of
 * 16 CPUs) 16 threads that spin while their rings are full, plus the HIP
 * runtime's own threads, got the whole process throttled for ~10 ms at a
 * time (cpu.stat nr_throttled 29 in 3 s). The wait makes no
 * runtime call while the batch is on time (a query per wait from 16 threads
 * is the lock traffic the completion word removed): after
 * IXG_WAIT_QUERY_NS one stream query reports a failed stream early, and
 * past IXG_WAIT_RUNTIME_NS the runtime's own wait decides, so a batch whose
 * kernels failed returns -EIO instead of waiting forever. */
#ifndef IXG_WAIT_NAP_NS
#define IXG_WAIT_NAP_NS 10000L
#endif
/* the naps' timer slack while waiting (the default 50 us would make a 10 us
 * nap ~60 us; the caller's slack is restored after the wait) */
#ifndef IXG_WAIT_SLACK_NS
#define IXG_WAIT_SLACK_NS 2000L
#endif
#ifndef IXG_WAIT_SPIN
#define IXG_WAIT_SPIN 256u
#endif
#define IXG_WAIT_QUERY_NS 1000000ull
#define IXG_WAIT_RUNTIME_NS 200000000ull
/* the caller's timer slack, saved when the naps set the wait's own */
struct slack_save {
	int changed;       /* PR_SET_TIMERSLACK was called: restore `saved` */
	unsigned long saved;
};
static int wait_word(struct ixg_ctx *c, struct ixg_abatch *b, uint64_t t0, struct slack_save *sv)
{
	int queried = 0;
	for (uint32_t k = 0;; k++) {
		if (__atomic_load_n(b->h_done, __ATOMIC_ACQUIRE) == b->seq)
			return 0;
		if (k < IXG_WAIT_SPIN) {
#if defined(__x86_64__)
			__builtin_ia32_pause();
#endif
			continue;
		}
		const uint64_t dt = now_ns() - t0;
		if (!queried && dt > IXG_WAIT_QUERY_NS) {
			queried = 1;
			HIPCHK(hipSetDevice(c->device));
			const hipError_t e = hipStreamQuery(b->stream);
			if (e != hipSuccess && e != hipErrorNotReady)
				return -EIO;
			continue;
		}
		if (dt > IXG_WAIT_RUNTIME_NS)
			return 1;
		if (!sv->changed && IXG_WAIT_SLACK_NS > 0) {
			const int cur = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
			/* a saved 0 could not be restored (PR_SET_TIMERSLACK 0 means
			 * "the default"), and a slack already at the wait's needs no change */
			if (cur > 0 && (unsigned long)cur != (unsigned long)IXG_WAIT_SLACK_NS &&
			    prctl(PR_SET_TIMERSLACK, (unsigned long)IXG_WAIT_SLACK_NS, 0, 0, 0) == 0) {
				sv->saved = (unsigned long)cur;
				sv->changed = 1;
			}
		}
		const struct timespec nap = {0, IXG_WAIT_NAP_NS};
		const uint64_t n0 = now_ns();
		nanosleep(&nap, NULL);
		const uint64_t dn = now_ns() - n0;
		b->naps++;
		if (dn > b->nap_max)
			b->nap_max = dn;
		if (dn > c->async->st.nap_max_ns)
			c->async->st.nap_max_ns = dn;
	}
}

static int wait_done(struct ixg_ctx *c, struct ixg_abatch *b)
{
	struct slack_save sv = {0, 0};
	const int rc = wait_word(c, b, now_ns(), &sv);
	if (sv.changed)
		prctl(PR_SET_TIMERSLACK, sv.saved, 0, 0, 0);
	if (rc <= 0)
		return rc;
	HIPCHK(hipSetDevice(c->device));
	if (hipStreamSynchronize(b->stream) != hipSuccess || __atomic_load_n(b->h_done, __ATOMIC_ACQUIRE) != b->seq)
		return -EIO;
	return 0;
}

int ixg_rx_poll(void *vctx, void **mbufs, struct ixg_rx_rec *recs, uint32_t max, int wait)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (max && (!mbufs || !recs)))
		return -EINVAL;
	struct ixg_async *a = c->async;
	if (a && a->err) {
		const int e = a->err;
		a->err = 0;
		return e;
	}
	if (!a)
		return 0;
	a->st.poll_calls++;
	entry_gap(a);
	if (!a->count || !max) {
		a->t_exit = tsc();
		return 0;
	}
	/* an OPEN batch whose oldest frame has waited long enough goes now */
	{
		const struct ixg_abatch *o = &a->b[(a->tail + a->cfg.depth - 1) % a->cfg.depth];
		if (o->state == AS_OPEN && (wait || due(a, o, now_ns()))) {
			int rc = launch_open(c, a);
			if (rc)
				return rc;
		}
	}
	const uint64_t p0 = tsc(); /* (after the launch: launch_ns has it) */
	uint32_t got = 0;
	while (a->count && got < max) {
		struct ixg_abatch *b = &a->b[a->head];
		if (b->state == AS_INFLIGHT) {
			if (__atomic_load_n(b->h_done, __ATOMIC_ACQUIRE) != b->seq) {
				if (!wait || got)
					break;
				const uint64_t w0 = tsc(), n0 = now_ns();
				const int rc = wait_done(c, b);
				a->st.wait_ns += tsc() - w0;
				b->wait_ns += now_ns() - n0;
				if (rc)
					return rc;
			}
			batch_seen(a, b);
			b->state = AS_DONE;
		}
		if (b->state != AS_DONE)
			break; /* the OPEN batch: nothing launched behind it */
		const uint32_t k = b->n - b->taken < max - got ? b->n - b->taken : max - got;
		memcpy(mbufs + got, b->mbufs + b->taken, (size_t)k * sizeof(void *));
		memcpy(recs + got, b->h_rec + b->taken, (size_t)k * sizeof(struct ixg_rx_rec));
		b->taken += k;
		got += k;
		if (b->taken == b->n) {
			batch_returned(a, b, now_ns());
			b->state = AS_FREE;
			a->head = (a->head + 1) % a->cfg.depth;
			a->count--;
		}
	}
	a->st.frames_returned += got;
	a->t_exit = tsc();
	a->st.poll_ns += a->t_exit - p0;
	return (int)got;
}

int ixg_rx_async_stats(void *vctx, struct ixg_rx_async_stats *out, int reset)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return -EINVAL;
	struct ixg_async *a = c->async;
	if (out) {
		memset(out, 0, sizeof(*out));
		if (a) {
			*out = a->st;
			/* ticks -> ns at the rate measured over the context's life */
			const uint64_t dt = tsc() - a->tsc0, dn = now_ns() - a->ns0;
			const double r = dt ? (double)dn / (double)dt : 1.0;
			out->gather_ns = (uint64_t)((double)a->st.gather_ns * r);
			out->launch_ns = (uint64_t)((double)a->st.launch_ns * r);
			/* (poll_ns includes wait_ns) */
			out->poll_ns = (uint64_t)((double)(a->st.poll_ns - a->st.wait_ns) * r);
			out->wait_ns = (uint64_t)((double)a->st.wait_ns * r);
		out->launch_max_ns = (uint64_t)((double)a->st.launch_max_ns * r);
			out->worst_outside_ns = (uint64_t)((double)a->st.worst_outside_ns * r);
		}
	}
	if (reset && a)
		memset(&a->st, 0, sizeof(a->st));
	return 0;
}

int ixg_rx_async_pending(void *vctx)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return -EINVAL;
	const struct ixg_async *a = c->async;
	if (!a)
		return 0;
	uint64_t n = 0;
	for (uint32_t k = 0, i = a->head; k < a->count; k++, i = (i + 1) % a->cfg.depth)
		n += a->b[i].n - a->b[i].taken;
	return n > 0x7fffffffu ? 0x7fffffff : (int)n;
}
