/*
 * ix_async_loop.c - IX's run-to-completion loop driving libixgrx's
 * asynchronous host path, one context per CPU.
 *
 * Each thread plays one IX CPU: per iteration of sys_bpoll
 * (dp/core/syscall.c:134-222) it takes up to eth_rx_max_batch (64) frames off
 * its RX queue (dp/core/ethqueue.c:71,117-149), hands them to
 * ixg_rx_submit_mbufs, polls finished records without waiting and runs the
 * eth_input callees on them through ixg_rx_dispatch, then moves on (timers,
 * TX). Frames come from an arena of IX mbufs (2112-B elements, len @0, data
 * @+64) built per thread from a frames file.
 *
 * Modes (one JSON line on stdout):
 *   loop   T threads for S seconds: aggregate Mpkt/s, submit->poll latency
 *          per iteration (p50/p99/max, us), host-link bytes per frame
 *   sync   one thread, ixg_rx_batch_mbufs of N frames per call, repeated:
 *          latency per call (us) and Mpkt/s
 *   async1 one thread, one batch of N frames at a time: submit, flush,
 *          poll(wait): the round trip of one batch through the async path
 *
 * build: gcc -O2 -Iinclude examples/ix_async_loop.c -Lix_amd -lixgrx -lpthread -o ix_async_loop
 * usage: ix_async_loop FRAMES_FILE MODE [key=value ...]
 *   threads=T seconds=S batch=64 n=N arena=FRAMES_PER_THREAD device=D
 *   cfg_frames= cfg_bytes= cfg_wait_us= cfg_depth= direct=0|1 dump=FILE
 *   register=1: register each thread's mbuf arena (ixg_rx_register_memory)
 *   so the kernels read the frames in place (zero copy)
 *   pages=huge|4k: the mbuf arenas on 2 MB pages as IX's mempools are
 *   (dp/core/mempool.c:198-243: hugetlbfs pages if the host has them
 *   reserved, else transparent huge pages; the default), or on 4 KB pages
 *   idle=wait|spin: an iteration whose frames the full ring refused either
 *   waits in ixg_rx_poll for the oldest batch (wait, the default: the CPU
 *   has no RX work until a batch returns, and gives its time away) or polls
 *   again at once (spin). On a CPU quota (the GPU box: 16 CPUs per 100 ms),
 *   16 spinning threads plus the HIP runtime's own got the process throttled
 *   for ~10 ms at a time.
 *   pin=K: thread i runs on the K*i-th CPU of the process's allowed set (as
 *   IX pins one thread per dedicated core, dp/core/cpu.c); 0 (the default):
 *   the scheduler places the threads
 *   pinset=K: thread i may run on the K CPUs from the K*i-th of the lower
 *   half of the allowed set and on their SMT siblings in the upper half
 *   (K = 8 on the GPU box: one core complex, its L3, per thread), and the
 *   scheduler picks among them
 * FRAMES_FILE: u32 count, u16 lengths[count], then the frames back to back.
 * dump=FILE (loop mode): thread 0's first `count` records, in submission
 * order, for the caller's parity check against the oracle.
 */
#define _GNU_SOURCE
#include <execinfo.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <ucontext.h>
#include <signal.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ixgrx.h"

#define MBUF_STRIDE IXG_MBUF_STRIDE

static double now_s(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* A fault anywhere in the process (the library, the HIP runtime, a
 * profiler's interception) prints the fault address, the stack and the
 * process's mappings, so every frame can be resolved to a library and an
 * offset afterwards (a SIGSEGV under rocprofv3 whose runtime
 * frames could not be attributed). Only async-signal-safe calls. */
static void fault_dump(int sig, siginfo_t *si, void *uc)
{
	char b[160];
	const void *pc = NULL;
#if defined(__x86_64__)
	if (uc)
		pc = (const void *)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
#endif
	int n = snprintf(b, sizeof(b), "\n*** ix_async_loop: signal %d at address %p, pc %p, thread %d; stack:\n", sig,
			 si ? si->si_addr : NULL, pc, (int)gettid());
	if (write(2, b, (size_t)n) < 0)
		_exit(128 + sig);
	void *fr[64];
	backtrace_symbols_fd(fr, backtrace(fr, 64), 2);
	if (write(2, "/proc/self/maps:\n", 17) < 0)
		_exit(128 + sig);
	const int fd = open("/proc/self/maps", O_RDONLY);
	if (fd >= 0) {
		char m[4096];
		ssize_t k;
		while ((k = read(fd, m, sizeof(m))) > 0)
			if (write(2, m, (size_t)k) < 0)
				break;
		close(fd);
	}
	signal(sig, SIG_DFL);
	raise(sig);
}

static void install_fault_dump(void)
{
	void *fr[4];
	backtrace(fr, 4); /* loads the unwinder now, not inside the handler */
	struct sigaction sa;
	memset(&sa, 0, sizeof(sa));
	sa.sa_sigaction = fault_dump;
	sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
	sigaction(SIGSEGV, &sa, NULL);
	sigaction(SIGBUS, &sa, NULL);
}

/* ---- options ------------------------------------------------------------- */
static struct {
	const char *frames, *mode, *dump;
	int threads, batch, device, direct, reg, spin, small_pages;
	double seconds;
	uint32_t n, arena;
	struct ixg_rx_async_cfg acfg;
	int pin, pinset;
} opt = {NULL, "loop", NULL, 1, 64, 0, 0, 0, 0, 0, 2.0, 64, 1u << 16,
	 {IXG_ASYNC_DEF_FRAMES, IXG_ASYNC_DEF_BYTES, IXG_ASYNC_DEF_WAIT_US, IXG_ASYNC_DEF_DEPTH, IXG_ASYNC_DEF_FLAGS}, 0, 0};

/* thread i -> the (pin * i)-th CPU the process may run on, or (pinset) the
 * (pinset * i)-th block of pinset CPUs of the allowed set's lower half with
 * their upper-half siblings; 0 or -errno */
static int pin_thread(pthread_t th, int i)
{
	cpu_set_t all, one;
	if (sched_getaffinity(0, sizeof(all), &all))
		return -1;
	if (opt.pinset) {
		int list[CPU_SETSIZE], n = 0;
		for (int cpu = 0; cpu < CPU_SETSIZE; cpu++)
			if (CPU_ISSET(cpu, &all))
				list[n++] = cpu;
		const int half = n / 2 ? n / 2 : 1, b = (opt.pinset * i) % half;
		CPU_ZERO(&one);
		for (int k = 0; k < opt.pinset && b + k < half; k++) {
			CPU_SET(list[b + k], &one);
			if (half + b + k < n)
				CPU_SET(list[half + b + k], &one);
		}
		return -pthread_setaffinity_np(th, sizeof(one), &one);
	}
	const int n = CPU_COUNT(&all), want = (opt.pin * i) % (n ? n : 1);
	for (int cpu = 0, k = 0; cpu < CPU_SETSIZE; cpu++) {
		if (!CPU_ISSET(cpu, &all))
			continue;
		if (k++ == want) {
			CPU_ZERO(&one);
			CPU_SET(cpu, &one);
			return -pthread_setaffinity_np(th, sizeof(one), &one);
		}
	}
	return -1;
}

static const uint8_t rss_key[40] = {0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
				    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
				    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};

/* ---- the frames pool ----------------------------------------------------- */
static uint32_t pool_n;
static uint16_t *pool_len;
static uint8_t **pool_frame;
static uint64_t pool_bytes;

static int load_pool(const char *path)
{
	FILE *f = fopen(path, "rb");
	if (!f)
		return -1;
	if (fread(&pool_n, 4, 1, f) != 1 || pool_n == 0)
		return -1;
	pool_len = malloc(pool_n * sizeof(uint16_t));
	pool_frame = malloc(pool_n * sizeof(uint8_t *));
	if (!pool_len || !pool_frame || fread(pool_len, 2, pool_n, f) != pool_n)
		return -1;
	for (uint32_t i = 0; i < pool_n; i++) {
		if (pool_len[i] > IXG_MBUF_DATA_LEN)
			return -1;
		pool_frame[i] = malloc(pool_len[i] ? pool_len[i] : 1);
		if (!pool_frame[i] || fread(pool_frame[i], 1, pool_len[i], f) != pool_len[i])
			return -1;
		pool_bytes += pool_len[i];
	}
	fclose(f);
	return 0;
}

/* an arena of n IX mbufs holding the pool tiled: len = size_t at +0, data at
 * +64 (inc/ix/mbuf.h:73-90) */
#define HUGE_PAGE (2u << 20)
static const char *arena_pages = "4k"; /* what the arenas got: hugetlb, thp or 4k */

/* (+ the tail bytes the kernels may read past the last frame) */
static size_t arena_bytes(uint32_t n)
{
	return ((size_t)n * MBUF_STRIDE + IXG_TAIL_PAD + HUGE_PAGE - 1) & ~((size_t)HUGE_PAGE - 1);
}

static uint8_t *arena_alloc(size_t sz)
{
	if (opt.small_pages)
		return aligned_alloc(4096, sz);
	void *a = mmap(NULL, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_HUGETLB, -1, 0);
	if (a != MAP_FAILED) {
		arena_pages = "hugetlb";
		return a;
	}
	/* no reserved huge pages: 2 MB-aligned, transparent huge pages asked for */
	a = mmap(NULL, sz + HUGE_PAGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
	if (a == MAP_FAILED)
		return NULL;
	uint8_t *b = (uint8_t *)(((uintptr_t)a + HUGE_PAGE - 1) & ~(uintptr_t)(HUGE_PAGE - 1));
	if (madvise(b, sz, MADV_HUGEPAGE) == 0)
		arena_pages = "thp";
	return b;
}

static void **make_arena(uint32_t n, uint8_t **mem)
{
	uint8_t *a = arena_alloc(arena_bytes(n));
	void **p = malloc((size_t)n * sizeof(void *));
	if (!a || !p)
		return NULL;
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *mb = a + (size_t)i * MBUF_STRIDE;
		const uint32_t k = i % pool_n;
		size_t l = pool_len[k];
		memset(mb, 0, 64);
		memcpy(mb, &l, sizeof(l));
		memcpy(mb + 64, pool_frame[k], l);
		p[i] = mb;
	}
	*mem = a;
	return p;
}

/* ---- the eth_input callees (counting stand-ins) -------------------------- */
struct stats {
	uint64_t tcp, udp, icmp, arp, drop;
};
static void on_tcp(void *u, void *m, const struct ixg_rx_rec *r) { (void)m; (void)r; ((struct stats *)u)->tcp++; }
static void on_udp(void *u, void *m, const struct ixg_rx_rec *r) { (void)m; (void)r; ((struct stats *)u)->udp++; }
static void on_icmp(void *u, void *m, const struct ixg_rx_rec *r) { (void)m; (void)r; ((struct stats *)u)->icmp++; }
static void on_arp(void *u, void *m, const struct ixg_rx_rec *r) { (void)m; (void)r; ((struct stats *)u)->arp++; }
static void on_drop(void *u, void *m, const struct ixg_rx_rec *r) { (void)m; (void)r; ((struct stats *)u)->drop++; }
static const struct ixg_rx_ops ops = {on_tcp, on_udp, on_icmp, on_arp, on_drop};

static int new_ctx(void **ctx)
{
	struct ixg_rx_cfg cfg;
	memset(&cfg, 0, sizeof(cfg));
	memcpy(cfg.rss_key, rss_key, 40);
	cfg.nb_rx_fgs = 128;
	return ixg_rx_init(&cfg, opt.device, ctx);
}

static int cmp_d(const void *a, const void *b)
{
	const double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

static double pct(double *v, size_t n, double q)
{
	if (!n)
		return 0;
	size_t k = (size_t)(q * (double)(n - 1) + 0.5);
	return v[k];
}

/* ---- loop mode: one thread = one IX CPU --------------------------------- */
struct worker {
	int id, rc;
	pthread_t th;
	void *ctx;
	void **ptrs;
	uint8_t *mem;
	uint64_t frames_done, iters;
	double t_end;
	struct stats st;
	double *lat;
	size_t nlat, cap_lat;
	struct ixg_rx_rec *dump;
	uint32_t ndump;
	/* where the thread's time went: the library's counters, the callees, the
	 * longest gap between two passes of the loop (the thread not running,
	 * or stuck in a call), the scheduler's context switches */
	struct ixg_rx_async_stats ast;
	double t_dispatch, max_gap;
	long nvcsw, nivcsw;
};

static pthread_barrier_t bar;
static double t_start;

#define POLL_MAX 8192u

static void *work(void *arg)
{
	struct worker *w = arg;
	void **pm = malloc(POLL_MAX * sizeof(void *));
	struct ixg_rx_rec *pr = malloc(POLL_MAX * sizeof(*pr));
	/* the iterations in flight: frame sequence number their last frame has,
	 * and when they were submitted */
	const size_t qcap = 1u << 20;
	uint64_t *q_seq = malloc(qcap * sizeof(uint64_t));
	double *q_t = malloc(qcap * sizeof(double));
	size_t qh = 0, qt = 0;
	w->cap_lat = 1u << 22;
	w->lat = malloc(w->cap_lat * sizeof(double));
	if (!pm || !pr || !q_seq || !q_t || !w->lat) {
		w->rc = -12;
		pthread_barrier_wait(&bar);
		return NULL;
	}
	pthread_barrier_wait(&bar);
	const uint32_t n = opt.arena;
	uint64_t sub = 0, got = 0; /* frames submitted / polled */
	uint32_t pos = 0;
	ixg_rx_async_stats(w->ctx, NULL, 1);
	struct rusage ru0;
	getrusage(RUSAGE_THREAD, &ru0);
	double t_prev = now_s();
	int last_acc = 1;
	for (;;) {
		const double t = now_s();
		if (t - t_prev > w->max_gap)
			w->max_gap = t - t_prev;
		t_prev = t;
		const int more = t < w->t_end;
		if (more) {
			/* one sys_bpoll iteration: up to `batch` frames off the RX queue */
			uint32_t k = (uint32_t)opt.batch;
			if (pos + k > n)
				k = n - pos;
			int acc = ixg_rx_submit_mbufs(w->ctx, w->ptrs + pos, k);
			if (acc < 0) {
				w->rc = acc;
				break;
			}
			last_acc = acc;
			if (acc > 0) {
				sub += (uint64_t)acc;
				pos = (pos + (uint32_t)acc) % n;
				if (qt - qh < qcap) {
					q_seq[qt % qcap] = sub;
					q_t[qt % qcap] = t;
					qt++;
				}
				w->iters++;
			}
		} else if (got == sub) {
			break;
		}
		/* frames refused by a full ring: nothing to do for RX until the
		 * oldest batch returns */
		const int idle = more && last_acc == 0 && !opt.spin;
		int r = ixg_rx_poll(w->ctx, pm, pr, POLL_MAX, more && !idle ? 0 : 1);
		if (r < 0) {
			w->rc = r;
			break;
		}
		if (r > 0) {
			const double d0 = now_s();
			ixg_rx_dispatch(pm, pr, (uint32_t)r, &ops, &w->st);
			w->t_dispatch += now_s() - d0;
			if (w->dump && w->ndump < pool_n) {
				uint32_t c = (uint32_t)r < pool_n - w->ndump ? (uint32_t)r : pool_n - w->ndump;
				memcpy(w->dump + w->ndump, pr, c * sizeof(*pr));
				w->ndump += c;
			}
			got += (uint64_t)r;
			const double t2 = now_s();
			while (qh < qt && q_seq[qh % qcap] <= got) {
				if (w->nlat < w->cap_lat)
					w->lat[w->nlat++] = (t2 - q_t[qh % qcap]) * 1e6;
				qh++;
			}
		}
	}
	w->frames_done = got;
	ixg_rx_async_stats(w->ctx, &w->ast, 0);
	struct rusage ru1;
	getrusage(RUSAGE_THREAD, &ru1);
	w->nvcsw = ru1.ru_nvcsw - ru0.ru_nvcsw;
	w->nivcsw = ru1.ru_nivcsw - ru0.ru_nivcsw;
	free(pm);
	free(pr);
	free(q_seq);
	free(q_t);
	return NULL;
}

static int run_loop(void)
{
	struct worker *ws = calloc((size_t)opt.threads, sizeof(*ws));
	if (!ws)
		return 1;
	pthread_barrier_init(&bar, NULL, (unsigned)opt.threads + 1);
	for (int i = 0; i < opt.threads; i++) {
		struct worker *w = &ws[i];
		w->id = i;
		if ((w->rc = new_ctx(&w->ctx)) || (w->rc = ixg_rx_async_init(w->ctx, &opt.acfg))) {
			fprintf(stderr, "context %d: %s\n", i, ixg_strerror(w->rc));
			return 2;
		}
		w->ptrs = make_arena(opt.arena, &w->mem);
		if (!w->ptrs)
			return 1;
		if (opt.reg && (w->rc = ixg_rx_register_memory(w->ctx, w->mem, arena_bytes(opt.arena)))) {
			fprintf(stderr, "register %d: %s\n", i, ixg_strerror(w->rc));
			return 2;
		}
		if (i == 0 && opt.dump)
			w->dump = malloc(pool_n * sizeof(struct ixg_rx_rec));
	}
	/* warm-up: one batch through every context (allocations, code objects) */
	for (int i = 0; i < opt.threads; i++) {
		void *pm[64];
		struct ixg_rx_rec pr[64];
		ixg_rx_submit_mbufs(ws[i].ctx, ws[i].ptrs, 64);
		while (ixg_rx_async_pending(ws[i].ctx) > 0)
			ixg_rx_poll(ws[i].ctx, pm, pr, 64, 1);
	}
	t_start = now_s();
	for (int i = 0; i < opt.threads; i++) {
		ws[i].t_end = t_start + opt.seconds;
		pthread_create(&ws[i].th, NULL, work, &ws[i]);
		if ((opt.pin || opt.pinset) && pin_thread(ws[i].th, i))
			fprintf(stderr, "pin: thread %d not pinned\n", i);
	}
	pthread_barrier_wait(&bar);
	t_start = now_s();
	for (int i = 0; i < opt.threads; i++)
		pthread_join(ws[i].th, NULL);
	const double el = now_s() - t_start;
	uint64_t frames = 0, iters = 0;
	struct stats st = {0, 0, 0, 0, 0};
	size_t nl = 0;
	for (int i = 0; i < opt.threads; i++) {
		if (ws[i].rc) {
			fprintf(stderr, "thread %d: %s\n", i, ixg_strerror(ws[i].rc));
			return 3;
		}
		frames += ws[i].frames_done;
		iters += ws[i].iters;
		st.tcp += ws[i].st.tcp;
		st.udp += ws[i].st.udp;
		st.icmp += ws[i].st.icmp;
		st.arp += ws[i].st.arp;
		st.drop += ws[i].st.drop;
		nl += ws[i].nlat;
	}
	/* the per-thread breakdown, summed over threads (ns per frame of each
	 * part of a thread's time; the rest is the loop itself and waiting) */
	double g_ns = 0, l_ns = 0, p_ns = 0, w_ns = 0, d_s = 0, gap = 0, lmax = 0;
	uint64_t batches = 0, by_time = 0, refused = 0, offered = 0, img = 0, inpl = 0, launched = 0;
	long vcs = 0, ivcs = 0;
	/* the worst batch of all threads, and where its time went */
	const struct ixg_rx_async_stats *wb = &ws[0].ast;
	int wth = 0;
	double nap_max = 0;
	for (int i = 0; i < opt.threads; i++) {
		if (ws[i].ast.worst_total_ns > wb->worst_total_ns) {
			wb = &ws[i].ast;
			wth = i;
		}
		if ((double)ws[i].ast.nap_max_ns > nap_max)
			nap_max = (double)ws[i].ast.nap_max_ns;
	}
	for (int i = 0; i < opt.threads; i++) {
		const struct ixg_rx_async_stats *a = &ws[i].ast;
		g_ns += (double)a->gather_ns;
		l_ns += (double)a->launch_ns;
		p_ns += (double)a->poll_ns;
		w_ns += (double)a->wait_ns;
		d_s += ws[i].t_dispatch;
		batches += a->batches;
		img += a->image_bytes;
		inpl += a->inplace_bytes;
		launched += a->frames_launched;
		by_time += a->batches_by_time;
		refused += a->frames_refused;
		offered += a->frames_refused + a->frames_submitted;
		vcs += ws[i].nvcsw;
		ivcs += ws[i].nivcsw;
		if (ws[i].max_gap > gap)
			gap = ws[i].max_gap;
		if ((double)a->launch_max_ns > lmax)
			lmax = (double)a->launch_max_ns;
	}
	const double fr = frames ? (double)frames : 1.0;
	double *lat = malloc((nl ? nl : 1) * sizeof(double));
	size_t o = 0;
	for (int i = 0; i < opt.threads; i++) {
		memcpy(lat + o, ws[i].lat, ws[i].nlat * sizeof(double));
		o += ws[i].nlat;
	}
	qsort(lat, nl, sizeof(double), cmp_d);
	/* bytes per frame of the staged images the library launched (frame bytes
	 * past the MAC addresses up to the IP total length, 4-aligned, offsets
	 * and lengths unless the run is of fixed stride / one length; zero copy:
	 * offsets and lengths only, the frames are read in place) */
	const double staged_b = launched ? (double)img / (double)launched : 0.0;
	const double inplace_b = launched ? (double)inpl / (double)launched : 0.0;
	printf("{\"mode\": \"loop\", \"threads\": %d, \"seconds\": %.3f, \"frames\": %llu, \"mpps\": %.2f, "
	       "\"iterations\": %llu, \"frames_per_iteration\": %.1f, \"batch\": %d, "
	       "\"latency_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f, \"n\": %zu}, "
	       "\"staged_bytes_per_frame\": %.1f, \"inplace_bytes_per_frame\": %.1f, \"record_bytes_per_frame\": 16, "
	       "\"cfg\": {\"batch_frames\": %u, \"batch_bytes\": %u, \"max_wait_us\": %u, \"depth\": %u, \"direct\": %d, "
	       "\"zero_copy\": %d, \"arena_pages\": \"%s\", \"pin\": %d, \"pinset\": %d}, "
	       "\"verdicts\": {\"tcp\": %llu, \"udp\": %llu, \"icmp\": %llu, \"arp\": %llu, \"drop\": %llu}, "
	       "\"breakdown\": {\"thread_ns_per_frame\": %.2f, \"gather_ns_per_frame\": %.2f, \"launch_us_per_batch\": %.2f, "
	       "\"poll_ns_per_frame\": %.2f, \"wait_ns_per_frame\": %.2f, \"dispatch_ns_per_frame\": %.2f, "
	       "\"frames_per_batch\": %.0f, \"batches_by_time\": %.3f, \"refused_share\": %.3f, "
	       "\"max_loop_gap_us\": %.1f, \"max_launch_us\": %.1f, \"context_switches\": {\"voluntary\": %ld, \"involuntary\": %ld}}, "
	       "\"worst_batch_us\": {\"thread\": %d, \"total\": %.1f, \"open\": %.1f, \"gpu\": %.1f, \"visible\": %.1f, "
	       "\"returned\": %.1f, \"wait\": %.1f, \"outside\": %.1f, \"thread_max_loop_gap\": %.1f, \"naps\": %llu, "
	       "\"nap_max\": %.1f, \"all_threads_nap_max\": %.1f}}\n",
	       opt.threads, el, (unsigned long long)frames, frames / el / 1e6, (unsigned long long)iters,
	       iters ? (double)frames / (double)iters : 0.0, opt.batch, pct(lat, nl, 0.5), pct(lat, nl, 0.99),
	       nl ? lat[nl - 1] : 0.0, nl, staged_b, inplace_b, opt.acfg.batch_frames, opt.acfg.batch_bytes, opt.acfg.max_wait_us,
	       opt.acfg.depth, (opt.acfg.flags & IXG_ASYNC_DIRECT) ? 1 : 0, opt.reg, arena_pages, opt.pin, opt.pinset, (unsigned long long)st.tcp,
	       (unsigned long long)st.udp, (unsigned long long)st.icmp, (unsigned long long)st.arp,
	       (unsigned long long)st.drop, el * opt.threads * 1e9 / fr, g_ns / fr,
	       batches ? l_ns / (double)batches / 1e3 : 0.0, p_ns / fr, w_ns / fr, d_s * 1e9 / fr,
	       batches ? fr / (double)batches : 0.0, batches ? (double)by_time / (double)batches : 0.0,
	       offered ? (double)refused / (double)offered : 0.0, gap * 1e6, lmax / 1e3, vcs, ivcs, wth,
	       wb->worst_total_ns / 1e3, wb->worst_open_ns / 1e3, wb->worst_gpu_ns / 1e3, wb->worst_visible_ns / 1e3,
	       wb->worst_returned_ns / 1e3, wb->worst_wait_ns / 1e3, wb->worst_outside_ns / 1e3, ws[wth].max_gap * 1e6,
	       (unsigned long long)wb->worst_naps, wb->worst_nap_max_ns / 1e3, nap_max / 1e3);
	if (opt.dump) {
		FILE *f = fopen(opt.dump, "wb");
		if (!f || fwrite(ws[0].dump, sizeof(struct ixg_rx_rec), ws[0].ndump, f) != ws[0].ndump)
			return 4;
		fclose(f);
	}
	for (int i = 0; i < opt.threads; i++) {
		ixg_rx_fini(ws[i].ctx);
		if (opt.small_pages)
			free(ws[i].mem); /* (the mapped arenas go with the process) */
		free(ws[i].ptrs);
		free(ws[i].lat);
		free(ws[i].dump);
	}
	free(ws);
	free(lat);
	return 0;
}

/* ---- sync / async1 modes: the latency of one batch of n frames ---------- */
static int run_latency(int async)
{
	void *ctx;
	int rc = new_ctx(&ctx);
	if (rc || (async && (rc = ixg_rx_async_init(ctx, &opt.acfg)))) {
		fprintf(stderr, "%s\n", ixg_strerror(rc));
		return 2;
	}
	const uint32_t n = opt.n;
	uint8_t *mem;
	void **ptrs = make_arena(n, &mem);
	struct ixg_rx_rec *recs = malloc((size_t)n * sizeof(*recs));
	void **pm = malloc((size_t)n * sizeof(void *));
	if (!ptrs || !recs || !pm)
		return 1;
	size_t cap = 200000, nl = 0;
	double *lat = malloc(cap * sizeof(double));
	double t0 = 0, tot = 0;
	for (int it = -3; nl < cap; it++) {
		const double a = now_s();
		if (async) {
			uint32_t i = 0, got = 0;
			while (i < n) {
				int acc = ixg_rx_submit_mbufs(ctx, ptrs + i, n - i);
				if (acc < 0)
					return 3;
				i += (uint32_t)acc;
				if (i < n) { /* ring full: take what is ready */
					int r = ixg_rx_poll(ctx, pm + got, recs + got, n - got, 1);
					if (r < 0)
						return 3;
					got += (uint32_t)r;
				}
			}
			ixg_rx_flush(ctx);
			while (got < n) {
				int r = ixg_rx_poll(ctx, pm + got, recs + got, n - got, 1);
				if (r < 0)
					return 3;
				got += (uint32_t)r;
			}
		} else if ((rc = ixg_rx_batch_mbufs(ctx, ptrs, n, recs)) != 0) {
			fprintf(stderr, "%s\n", ixg_strerror(rc));
			return 3;
		}
		const double b = now_s();
		if (it < 0)
			continue; /* warm-up calls */
		if (nl == 0)
			t0 = a;
		lat[nl++] = (b - a) * 1e6;
		tot += b - a;
		if (b - t0 > opt.seconds)
			break;
	}
	qsort(lat, nl, sizeof(double), cmp_d);
	double mean = 0;
	for (size_t i = 0; i < nl; i++)
		mean += lat[i];
	mean /= (double)(nl ? nl : 1);
	printf("{\"mode\": \"%s\", \"n\": %u, \"calls\": %zu, \"latency_us\": {\"mean\": %.1f, \"p50\": %.1f, "
	       "\"p99\": %.1f, \"min\": %.1f}, \"mpps\": %.3f, \"direct\": %d}\n",
	       async ? "async1" : "sync", n, nl, mean, pct(lat, nl, 0.5), pct(lat, nl, 0.99), nl ? lat[0] : 0.0,
	       (double)n * (double)nl / tot / 1e6, (opt.acfg.flags & IXG_ASYNC_DIRECT) ? 1 : 0);
	ixg_rx_fini(ctx);
	if (opt.small_pages)
		free(mem);
	free(ptrs);
	free(recs);
	free(pm);
	free(lat);
	return 0;
}

int main(int argc, char **argv)
{
	if (argc < 3) {
		fprintf(stderr, "usage: %s FRAMES_FILE loop|sync|async1 [key=value ...]\n", argv[0]);
		return 2;
	}
	install_fault_dump();
	opt.frames = argv[1];
	opt.mode = argv[2];
	for (int i = 3; i < argc; i++) {
		char *eq = strchr(argv[i], '=');
		if (!eq)
			return 2;
		*eq = 0;
		const char *k = argv[i], *v = eq + 1;
		if (!strcmp(k, "threads")) opt.threads = atoi(v);
		else if (!strcmp(k, "seconds")) opt.seconds = atof(v);
		else if (!strcmp(k, "batch")) opt.batch = atoi(v);
		else if (!strcmp(k, "n")) opt.n = (uint32_t)atoi(v);
		else if (!strcmp(k, "arena")) opt.arena = (uint32_t)atoi(v);
		else if (!strcmp(k, "device")) opt.device = atoi(v);
		else if (!strcmp(k, "dump")) opt.dump = v;
		else if (!strcmp(k, "cfg_frames")) opt.acfg.batch_frames = (uint32_t)atoi(v);
		else if (!strcmp(k, "cfg_bytes")) opt.acfg.batch_bytes = (uint32_t)atoi(v);
		else if (!strcmp(k, "cfg_wait_us")) opt.acfg.max_wait_us = (uint32_t)atoi(v);
		else if (!strcmp(k, "cfg_depth")) opt.acfg.depth = (uint32_t)atoi(v);
		else if (!strcmp(k, "direct")) opt.acfg.flags = atoi(v) ? IXG_ASYNC_DIRECT : 0;
		else if (!strcmp(k, "register")) opt.reg = atoi(v);
		else if (!strcmp(k, "pages")) opt.small_pages = !strcmp(v, "4k");
		else if (!strcmp(k, "idle")) opt.spin = !strcmp(v, "spin");
		else if (!strcmp(k, "pin")) opt.pin = atoi(v);
		else if (!strcmp(k, "pinset")) opt.pinset = atoi(v);
		else {
			fprintf(stderr, "unknown option %s\n", k);
			return 2;
		}
	}
	if (opt.threads < 1 || opt.batch < 1 || opt.n < 1 || opt.arena < (uint32_t)opt.batch ||
	    load_pool(opt.frames)) {
		fprintf(stderr, "bad options or frames file\n");
		return 2;
	}
	if (opt.dump && opt.arena < pool_n)
		opt.arena = pool_n;
	if (!strcmp(opt.mode, "loop"))
		return run_loop();
	if (!strcmp(opt.mode, "sync"))
		return run_latency(0);
	if (!strcmp(opt.mode, "async1"))
		return run_latency(1);
	return 2;
}
