/*
 * fakehip.c - TEST INFRASTRUCTURE ONLY. A CPU stand-in for the HIP runtime
 * and the RX kernels, linked with the C host library (ixgrx_host.c,
 * ixgrx_async.c) into tests/fakehip/libixgrx_fake.so, so the CPU test tier
 * can drive the host paths' staging, ring and ordering logic (under ASan
 * and UBSan) without a GPU. Never shipped, never used by a product path.
 *
 * "Device" memory is host memory. Every stream is a FIFO of deferred
 * operations (copies, memsets, launches, event marks) that run only when
 * someone synchronizes: hipStreamSynchronize and hipEventSynchronize run the
 * queue up to the point asked for; hipEventQuery returns hipErrorNotReady
 * the first time it is asked about pending work (and runs nothing), then
 * runs it. So a host path that read results before synchronizing, or
 * reused a staging buffer whose copy had not run yet, sees wrong records.
 * An RX "launch" runs the oracle's restatement (oracle/ixgrx_oracle.c) over
 * the launch's frames with the configuration fakehip_set_cfg installed, after
 * checking that every byte a kernel may read of each frame lies in memory
 * the device could reach (an allocation of this runtime or a registered
 * host range): a frame outside them would fault a real GPU, here it aborts.
 *
 * The runtime is thread-safe as HIP's is: one lock around every entry point
 * (contexts on several host threads call it at once; tests/fakehip/mt_async.c
 * runs 16 of them under ThreadSanitizer and under ASan/UBSan).
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ixgrx.h"
#include "../../ix_amd/csrc/ixgrx_internal.h"
#include "../../ix_amd/csrc/ixgrx_icmp.h"
#include "../../oracle/ixgrx_oracle.h"

enum { OP_COPY, OP_SET, OP_SET16, OP_RX, OP_MARK, OP_STAMP, OP_ICMP };

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static void lk(void) { pthread_mutex_lock(&g_mu); }
static void ul(void) { pthread_mutex_unlock(&g_mu); }

struct op {
	int kind;
	void *dst;
	const void *src;
	size_t n;
	int val;
	struct ixg_kparams p;
	struct ixg_iparams ip; /* OP_ICMP */
	uint64_t fdir_sum; /* OP_RX: the flow-director table when launched */
	struct fevent *ev;
	struct op *next;
};

struct fstream {
	struct op *head, *tail;
};

struct fevent {
	struct fstream *s; /* stream of the last record, NULL once it ran */
	int queried;       /* pending work was reported not ready once */
};

static struct ixg_rx_cfg g_cfg;
static unsigned long g_launches;
static int g_fail_launches;      /* the next this many RX launches fail */
static unsigned long g_fdir_stale; /* RX launches that ran after their table changed */
void fakehip_fail_launches(int k) { lk(); g_fail_launches = k; ul(); }
static int g_fail_stamps;        /* the next this many completion stamps fail to launch */
void fakehip_fail_stamps(int k) { lk(); g_fail_stamps = k; ul(); }
unsigned long fakehip_fdir_stale(void) { lk(); unsigned long v = g_fdir_stale; ul(); return v; }

/* FNV-1a over the flow-director table a launch reads (header + slots) */
static uint64_t fdir_sum(const uint32_t *t)
{
	if (!t)
		return 0;
	const size_t words = 4u * ((t[0] ? (size_t)t[0] + 1u : 0u) + 1u);
	uint64_t h = 1469598103934665603ull;
	for (size_t i = 0; i < words; i++)
		h = (h ^ t[i]) * 1099511628211ull;
	return h;
}

/* memory the device can reach: allocations and registered host ranges */
#define MAXR 4096
static struct {
	uintptr_t lo, hi;
	int registered;
} g_mem[MAXR];
static int g_nmem;
static unsigned long g_inplace; /* frames read from registered host memory */
static struct ixg_kparams g_last; /* the last RX launch's parameters */
static unsigned long g_icmp_items; /* echo-reflect items run */
static unsigned long g_stamps;     /* stamp kernels run */
unsigned long fakehip_icmp_items(void) { lk(); unsigned long v = g_icmp_items; ul(); return v; }
/* the last RX launch's layout: its stride (0: u64 offsets) and frame count */
void fakehip_last_launch(uint32_t *stride, uint32_t *n)
{
	lk();
	*stride = g_last.off ? 0u : g_last.stride;
	*n = g_last.n;
	ul();
}
/* the last launch's plan inputs: frames in host memory, every frame long
 * (the host-memory big-frame kernel), deferral in use */
void fakehip_last_plan(uint32_t *host_mem, uint32_t *long_only, uint32_t *defer)
{
	lk();
	*host_mem = g_last.host_mem;
	*long_only = g_last.long_only;
	*defer = g_last.defer != NULL;
	ul();
}
unsigned long fakehip_inplace_frames(void) { lk(); unsigned long v = g_inplace; ul(); return v; }
static void mem_add(const void *p, size_t n, int registered)
{
	if (g_nmem == MAXR)
		abort();
	g_mem[g_nmem].lo = (uintptr_t)p;
	g_mem[g_nmem].hi = (uintptr_t)p + n;
	g_mem[g_nmem].registered = registered;
	g_nmem++;
}
static void mem_del(const void *p)
{
	for (int i = 0; i < g_nmem; i++)
		if (g_mem[i].lo == (uintptr_t)p) {
			g_mem[i] = g_mem[--g_nmem];
			return;
		}
}
/* 0: unreachable, 1: an allocation, 2: registered host memory */
static int reachable(uintptr_t lo, uintptr_t hi)
{
	for (int i = 0; i < g_nmem; i++)
		if (lo >= g_mem[i].lo && hi <= g_mem[i].hi)
			return 1 + g_mem[i].registered;
	return 0;
}

void fakehip_set_cfg(const struct ixg_rx_cfg *cfg) { lk(); g_cfg = *cfg; ul(); }
unsigned long fakehip_launches(void) { lk(); unsigned long v = g_launches; ul(); return v; }
unsigned long fakehip_stamps(void) { lk(); unsigned long v = g_stamps; ul(); return v; }

static void run_op(struct op *o)
{
	switch (o->kind) {
	case OP_COPY:
		memcpy(o->dst, o->src, o->n);
		break;
	case OP_SET:
		memset(o->dst, o->val, o->n);
		break;
	case OP_SET16:
		for (size_t k = 0; k < o->n; k++)
			((uint16_t *)o->dst)[k] = (uint16_t)o->val;
		break;
	case OP_RX: {
		/* the bytes the kernels may read of frame i: its first max(L, 112)
		 * bytes and up to 16 past them (IXG_TAIL_PAD covers it) */
		for (uint32_t i = 0; i < o->p.n; i++) {
			const uint64_t off = o->p.off ? o->p.off[i] : (uint64_t)i * o->p.stride;
			const uintptr_t a = (uintptr_t)o->p.base + off;
			const uint32_t L = o->p.len[i] > 112 ? o->p.len[i] : 112;
			const int r = reachable(a, a + L + 16);
			if (!r || !reachable((uintptr_t)(o->p.out + i), (uintptr_t)(o->p.out + i + 1)))
				abort();
			g_inplace += r == 2;
		}
		/* a kernel reads the table when it runs: it must still be the one
		 * in force when the launch was made */
		if (fdir_sum(o->p.fdir) != o->fdir_sum)
			g_fdir_stale++;
		struct ixg_rx_cfg c = g_cfg;
		ixgo_rx_batch(&c, o->p.base, o->p.off, o->p.len, o->p.stride, o->p.n, o->p.out, o->p.csum, 1,
			      IXGO_HASH_TABLE, IXGO_WORK_FULL);
		g_launches++;
		break;
	}
	case OP_MARK:
		o->ev->s = NULL;
		break;
	case OP_ICMP: {
		/* the reflect kernel's items through the oracle, one frame each */
		const struct ixg_iparams *q = &o->ip;
		uint32_t host;
		memcpy(&host, q->host, 4);
		host = __builtin_bswap32(host);
		for (uint32_t j = 0; j < q->n; j++) {
			const uint64_t r = q->idx ? q->idx[j] : j;
			uint8_t *f = (uint8_t *)((uintptr_t)q->base + (q->off ? q->off[j] : (uint64_t)j * q->stride));
			const uint32_t len = 14u + q->rec[r].l4_off + q->rec[r].l4_len;
			if (!reachable((uintptr_t)f, (uintptr_t)f + len) ||
			    !reachable((uintptr_t)(q->rec + r), (uintptr_t)(q->rec + r + 1)))
				abort();
			if (ixgo_icmp_reflect_batch(f, NULL, 0, &q->rec[r], 1, q->mac, host) && q->mark)
				q->rec[r].flags |= IXG_RF_REPLY;
		}
		g_icmp_items += q->n;
		break;
	}
	case OP_STAMP:
		__atomic_store_n((uint32_t *)o->dst, (uint32_t)o->val, __ATOMIC_RELEASE);
		g_stamps++;
		break;
	}
}

/* run stream s's operations up to and including `upto` (NULL: all) */
static void drain(struct fstream *s, struct op *upto)
{
	while (s->head) {
		struct op *o = s->head;
		s->head = o->next;
		if (!s->head)
			s->tail = NULL;
		run_op(o);
		const int last = o == upto;
		free(o);
		if (last)
			return;
	}
}

static struct fstream g_null;
static struct fstream *S(hipStream_t s) { return s ? (struct fstream *)s : &g_null; }

static struct op *push(hipStream_t st, struct op *o)
{
	struct fstream *s = S(st);
	o->next = NULL;
	if (s->tail)
		s->tail->next = o;
	else
		s->head = o;
	s->tail = o;
	return o;
}

static struct op *new_op(int kind)
{
	struct op *o = (struct op *)calloc(1, sizeof(*o));
	if (!o)
		abort();
	o->kind = kind;
	return o;
}

/* ---- the runtime (every entry point under g_mu) ------------------------- */
hipError_t hipSetDevice(int d) { return d == 0 ? hipSuccess : hipErrorInvalidDevice; }
/* (no device clock here: the stats' worst-batch split reports no device time) */
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t a, int d)
{
	(void)a;
	(void)d;
	*v = 0;
	return hipErrorNotSupported;
}
hipError_t hipGetDeviceCount(int *n)
{
	*n = 1;
	return hipSuccess;
}
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600 *p, int d)
{
	(void)d;
	memset(p, 0, sizeof(*p));
	p->multiProcessorCount = 256;
	return hipSuccess;
}
static hipError_t dev_alloc(void **p, size_t n)
{
	*p = aligned_alloc(256, (n + 255) & ~(size_t)255);
	if (*p)
		mem_add(*p, n, 0);
	return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipMalloc(void **p, size_t n)
{
	lk();
	const hipError_t e = dev_alloc(p, n);
	ul();
	return e;
}
hipError_t hipHostMalloc(void **p, size_t n, unsigned int f)
{
	(void)f;
	return hipMalloc(p, n);
}
static unsigned long g_frees; /* hipFree of an allocation (a device-wide wait on HIP) */
unsigned long fakehip_frees(void) { lk(); unsigned long v = g_frees; ul(); return v; }
hipError_t hipFree(void *p)
{
	lk();
	g_frees += p != NULL;
	mem_del(p);
	ul();
	free(p);
	return hipSuccess;
}
hipError_t hipHostFree(void *p)
{
	lk();
	mem_del(p);
	ul();
	free(p);
	return hipSuccess;
}
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind k)
{
	(void)k;
	lk();
	drain(&g_null, NULL);
	memcpy(d, s, n);
	ul();
	return hipSuccess;
}
hipError_t hipMemset(void *d, int v, size_t n)
{
	lk();
	drain(&g_null, NULL);
	memset(d, v, n);
	ul();
	return hipSuccess;
}
hipError_t hipMemcpyAsync(void *d, const void *s, size_t n, hipMemcpyKind k, hipStream_t st)
{
	(void)k;
	struct op *o = new_op(OP_COPY);
	o->dst = d;
	o->src = s;
	o->n = n;
	lk();
	push(st, o);
	ul();
	return hipSuccess;
}
hipError_t hipMemsetAsync(void *d, int v, size_t n, hipStream_t st)
{
	struct op *o = new_op(OP_SET);
	o->dst = d;
	o->val = v;
	o->n = n;
	lk();
	push(st, o);
	ul();
	return hipSuccess;
}
hipError_t hipMemsetD16Async(hipDeviceptr_t d, unsigned short v, size_t n, hipStream_t st)
{
	struct op *o = new_op(OP_SET16);
	o->dst = d;
	o->val = v;
	o->n = n;
	lk();
	push(st, o);
	ul();
	return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t *s, unsigned int f)
{
	(void)f;
	*s = (hipStream_t)calloc(1, sizeof(struct fstream));
	return *s ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipStreamSynchronize(hipStream_t s)
{
	lk();
	drain(S(s), NULL);
	ul();
	return hipSuccess;
}
/* a query runs what the stream holds (as a device that finished it by now) */
hipError_t hipStreamQuery(hipStream_t s)
{
	lk();
	drain(S(s), NULL);
	ul();
	return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s)
{
	lk();
	drain(S(s), NULL);
	ul();
	if (s)
		free(s);
	return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned int f)
{
	(void)f;
	*e = (hipEvent_t)calloc(1, sizeof(struct fevent));
	return *e ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipEventDestroy(hipEvent_t e)
{
	free(e);
	return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t st)
{
	struct fevent *ev = (struct fevent *)e;
	struct op *o = new_op(OP_MARK);
	o->ev = ev;
	lk();
	ev->s = S(st);
	ev->queried = 0;
	push(st, o);
	ul();
	return hipSuccess;
}
/* run the event's stream up to its (latest) mark */
static void run_to(struct fevent *ev)
{
	struct fstream *s = ev->s;
	while (ev->s && s->head)
		drain(s, s->head);
	ev->s = NULL;
}
hipError_t hipEventSynchronize(hipEvent_t e)
{
	lk();
	run_to((struct fevent *)e);
	ul();
	return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e)
{
	struct fevent *ev = (struct fevent *)e;
	hipError_t r = hipSuccess;
	lk();
	if (ev->s) {
		if (!ev->queried) {
			ev->queried = 1;
			r = hipErrorNotReady;
		} else {
			run_to(ev);
		}
	}
	ul();
	return r;
}

hipError_t hipHostRegister(void *p, size_t n, unsigned int f)
{
	(void)f;
	lk();
	mem_add(p, n, 1);
	ul();
	return hipSuccess;
}
hipError_t hipHostUnregister(void *p)
{
	lk();
	mem_del(p);
	ul();
	return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void **d, void *h, unsigned int f)
{
	(void)f;
	*d = h;
	return hipSuccess;
}

/* ---- the kernels' launch entry points (ixgrx_internal.h) ------------------ */
int ixgrx_launch(const void *params, uint32_t ncu, void *stream)
{
	(void)ncu;
	lk();
	if (g_fail_launches > 0) {
		g_fail_launches--;
		ul();
		return -1;
	}
	struct op *o = new_op(OP_RX);
	memcpy(&o->p, params, sizeof(o->p));
	o->fdir_sum = fdir_sum(o->p.fdir);
	g_last = o->p;
	push((hipStream_t)stream, o);
	ul();
	return 0;
}
/* the completion stamp: written when the stream runs up to it (a poll that
 * reads the word before someone synchronizes sees the batch unfinished) */
int ixgrx_stamp(uint32_t *flag, uint32_t v, void *stream)
{
	lk();
	if (!reachable((uintptr_t)flag, (uintptr_t)(flag + 1)))
		abort();
	if (g_fail_stamps > 0) {
		g_fail_stamps--;
		ul();
		return -1;
	}
	struct op *o = new_op(OP_STAMP);
	o->dst = flag;
	o->val = (int)v;
	push((hipStream_t)stream, o);
	ul();
	return 0;
}
uint32_t ixgrx_kparams_size(void) { return (uint32_t)sizeof(struct ixg_kparams); }
uint32_t ixgrx_block(void) { return 256; }
int ixgrx_demux_launch(const void *p, uint32_t ncu, void *s)
{
	(void)p; (void)ncu; (void)s;
	return -1;
}
int ixgrx_tx_launch(const void *p, uint32_t ncu, void *s)
{
	(void)p; (void)ncu; (void)s;
	return -1;
}
int ixgrx_ev_launch(const void *p, uint32_t ncu, void *s)
{
	(void)p; (void)ncu; (void)s;
	return -1;
}
int ixgrx_icmp_launch(const void *p, void *s)
{
	struct op *o = new_op(OP_ICMP);
	memcpy(&o->ip, p, sizeof(o->ip));
	lk();
	push((hipStream_t)s, o);
	ul();
	return 0;
}
int ixgrx_tcpx_fusable(const void *p)
{
	(void)p;
	return 0;
}
int ixgrx_tcpx_launch(const void *p, void *s)
{
	(void)p; (void)s;
	return -1;
}
