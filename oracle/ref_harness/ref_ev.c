/*
 * ref_ev.c - the reference's usys descriptor encoders.
 *
 * TEST INFRASTRUCTURE ONLY. usys_udp_recv / usys_tcp_recv
 * (inc/ix/syscall.h:360-365,416-420, BSYS_DESC_*ARG :113-126) write into the
 * per-CPU usys array through usys_next (:350-353); mempool_pagemem_to_iomap
 * (inc/ix/mempool.h:259-263) maps a buffer address to its IOMAP address.
 * All are header inlines, compiled here unmodified; the per-CPU usys_arr is
 * this harness's (the %gs block ref_ix_init sets up).
 */
#include <ix/stddef.h>
#include <ix/mempool.h>
#include <ix/syscall.h>
#include <string.h>

#include "ref_capture.h"

DEFINE_PERCPU(struct bsys_arr *, usys_arr);

static struct {
	struct bsys_arr a;
	struct bsys_desc d[1];
} one;
static struct mempool pool;

void ref_ev_set_iomap(uint64_t iomap_offset)
{
	memset(&pool, 0, sizeof(pool));
	pool.iomap_offset = (uintptr_t)iomap_offset;
}

uint64_t ref_iomap(const void *p)
{
	return (uint64_t)(uintptr_t)mempool_pagemem_to_iomap(&pool, (void *)p);
}

static void *next_slot(void)
{
	one.a.len = 0;
	one.a.max_len = 1;
	percpu_get(usys_arr) = &one.a;
	return &one.d[0];
}

void ref_ev_udp(void *addr, size_t len, void *id, uint64_t out[5])
{
	next_slot();
	memset(&one.d[0], 0, sizeof(one.d[0]));
	usys_udp_recv(addr, len, (struct ip_tuple *)id);
	memcpy(out, &one.d[0], 40);
}

void ref_ev_tcp(uint64_t handle, unsigned long cookie, void *addr, size_t len, uint64_t out[5])
{
	next_slot();
	memset(&one.d[0], 0, sizeof(one.d[0]));
	usys_tcp_recv((hid_t)handle, cookie, addr, len);
	memcpy(out, &one.d[0], 40);
}
