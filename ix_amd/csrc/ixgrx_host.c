/*
 * ixgrx_host.c - the C host side of the RX engine: contexts, hash tables,
 * device and host batch entry points, and the eth_input-replacing dispatch.
 *
 * Plain C over the HIP runtime API; the kernels live in ixgrx_kernels.hip.
 * Semantics of every record field: include/ixgrx.h and DESIGN.md.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "ixgrx_ctx.h"
#include "ixgrx_demux.h"
#include "ixgrx_tcpx.h"
#include "ixgrx_tx.h"
#include "ixgrx_ev.h"
#include "ixgrx_icmp.h"

/* ---- hash tables -------------------------------------------------------- */

/* CRC-32C step as x86 crc32q (inc/ix/hash.h:35-39): reflected 0x82F63B78,
 * no inversion, operand bytes least significant first */
static uint32_t crc32c_u64(uint32_t crc, uint64_t v)
{
	for (int k = 0; k < 64; k++) {
		crc ^= (uint32_t)(v >> k) & 1u;
		crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
	}
	return crc;
}

static uint32_t crc_stream(uint32_t seed, const uint8_t s[24])
{
	uint64_t w[3];
	memcpy(w, s, 24);
	return crc32c_u64(crc32c_u64(crc32c_u64(seed, w[0]), w[1]), w[2]);
}

/* Toeplitz contribution of byte value v at tuple position i: the 32-bit
 * key windows starting at key bits 8i..8i+7, XORed for the set bits of v
 * (MSB first), as compute_toeplitz_hash accumulates them (tcp_api.c:593-601) */
static uint32_t toeplitz_byte(const uint8_t *key, int i, unsigned v)
{
	uint64_t k40 = ((uint64_t)key[i] << 32) | ((uint64_t)key[i + 1] << 24) |
		       ((uint64_t)key[i + 2] << 16) | ((uint64_t)key[i + 3] << 8) | key[i + 4];
	uint32_t r = 0;
	for (int j = 0; j < 8; j++)
		if (v & (0x80u >> j))
			r ^= (uint32_t)(k40 >> (8 - j));
	return r;
}

/* tuple byte i (Toeplitz order: src ip, dst ip, sport, dport; wire bytes)
 * -> byte position in tcp_to_idx's 24-byte crc32q stream: w1 = local (dst)
 * ip, w2 = remote (src) ip, w3 = (dport<<16 | sport) host order, sign-extended */
static const int k_crc_pos[12] = {8, 9, 10, 11, 0, 1, 2, 3, 17, 16, 19, 18};

int ixg_rx_hash_tables(const struct ixg_rx_cfg *cfg, uint64_t *tab, uint32_t *crc_const)
{
	if (!cfg || !tab)
		return -EINVAL;
	uint8_t s[24];
	memset(s, 0, sizeof(s));
	if (crc_const)
		*crc_const = crc_stream(IXG_PCB_HASH_SEED, s);
	for (int i = 0; i < 12; i++)
		for (unsigned v = 0; v < 256; v++) {
			memset(s, 0, sizeof(s));
			s[k_crc_pos[i]] = (uint8_t)v;
			if (i == 10 && (v & 0x80)) /* dport's high byte is the int's sign */
				memset(s + 20, 0xff, 4);
			uint64_t crc = crc_stream(0, s);
			tab[i * 256 + v] = (uint64_t)toeplitz_byte(cfg->rss_key, i, v) | (crc << 32);
		}
	return 0;
}

/* IXG_TAB6_WORDS: [i - IXG_TAB6_FIRST][v] = the Toeplitz contribution of
 * value v at tuple byte i of the 36-byte IPv6 tuple, for i = 12..35 (bytes
 * 0..11 share the IPv4 tables' key offsets) */
static void hash_table6(const struct ixg_rx_cfg *cfg, uint32_t *tab6)
{
	for (unsigned i = IXG_TAB6_FIRST; i < 36; i++)
		for (unsigned v = 0; v < 256; v++)
			tab6[(i - IXG_TAB6_FIRST) * 256 + v] = toeplitz_byte(cfg->rss_key, (int)i, v);
}

/* ---- context -------------------------------------------------------------- */

int ixg_abi_version(void) { return IXGRX_ABI_VERSION; }

const char *ixg_strerror(int err)
{
	switch (err) {
	case 0: return "ok";
	case -EINVAL: return "invalid argument";
	case -ENOMEM: return "out of memory";
	case -ENODEV: return "no such HIP device";
	case -EIO: return "HIP runtime error";
	case -ENOENT: return "no demux tables / TX MAC table loaded";
	default: return "unknown error";
	}
}

void ixg_dstate_free(struct ixg_dstate *ds)
{
	hipFree(ds->d_defer);
	hipFree(ds->d_lenc);
	hipFree(ds->d_present);
	memset(ds, 0, sizeof(*ds));
}

static void ixg_slot_free(struct ixg_slot *sl);
static int fdir_upload(struct ixg_ctx *c, const uint32_t *tab, uint32_t slots);

void ixg_rx_fini(void *vctx)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return;
	hipSetDevice(c->device);
	if (c->stream)
		hipStreamSynchronize(c->stream);
	ixg_async_free(c);
	for (uint32_t r = 0; r < c->nreg; r++)
		hipHostUnregister((void *)c->reg[r].lo);
	for (int k = 0; k < IXG_SLOTS; k++)
		ixg_slot_free(&c->slot[k]);
	hipFree(c->d_tab);
	hipFree(c->d_tab6);
	hipFree(c->d_tab32);
	hipFree(c->d_tab16);
	ixg_dstate_free(&c->ds);
	hipFree(c->d_zero);
	hipFree(c->d_dmacs);
	hipFree(c->d_bline);
	hipFree(c->d_txbuf);
	hipFree(c->d_txout);
	hipFree(c->d_txsegs);
	hipFree(c->d_txlen);
	hipFree(c->d_evbase);
	hipFree(c->d_fdir);
	hipFree(c->d_frames);
	hipFree(c->d_off);
	hipFree(c->d_len);
	hipFree(c->d_out);
	hipFree(c->d_csum);
	hipFree(c->d_astart);
	hipFree(c->d_active);
	hipFree(c->d_tw);
	hipFree(c->d_listen);
	hipFree(c->d_dmx);
	if (c->stream)
		hipStreamDestroy(c->stream);
	free(c);
}

int ixg_rx_init(const struct ixg_rx_cfg *cfg, int device, void **out)
{
	if (!cfg || !out)
		return -EINVAL;
	*out = NULL;
	if (cfg->nb_rx_fgs == 0 || cfg->nb_rx_fgs > IXG_ETH_MAX_NUM_FG ||
	    (cfg->nb_rx_fgs & (cfg->nb_rx_fgs - 1)))
		return -EINVAL;
	if ((uint32_t)cfg->dev_idx * IXG_ETH_MAX_NUM_FG + IXG_ETH_MAX_NUM_FG > 0x10000u)
		return -EINVAL;
	if (cfg->flags & ~(uint32_t)(IXG_F_NO_CSUM_DROP | IXG_F_IPV6))
		return -EINVAL;
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
		return -ENODEV;
	struct ixg_ctx *c = (struct ixg_ctx *)calloc(1, sizeof(*c));
	if (!c)
		return -ENOMEM;
	c->device = device;
	c->cfg = *cfg;
	int rc = -EIO;
	if (hipSetDevice(device) != hipSuccess)
		goto fail;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, device) != hipSuccess)
		goto fail;
	c->force_mode = IXG_MODE_AUTO;
	c->ncu = (uint32_t)prop.multiProcessorCount;
	uint64_t *tab = (uint64_t *)malloc(12 * 256 * sizeof(uint64_t));
	if (!tab) {
		rc = -ENOMEM;
		goto fail;
	}
	ixg_rx_hash_tables(cfg, tab, &c->crc_const);
	uint32_t tab32[12 * 256];
	uint16_t tab16[12 * 256];
	for (int k = 0; k < 12 * 256; k++) {
		tab32[k] = (uint32_t)tab[k];
		tab16[k] = (uint16_t)(tab[k] >> 32);
	}
	if (hipMalloc((void **)&c->d_tab, 12 * 256 * sizeof(uint64_t)) != hipSuccess ||
	    hipMemcpy(c->d_tab, tab, 12 * 256 * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess ||
	    hipMalloc((void **)&c->d_tab32, sizeof(tab32)) != hipSuccess ||
	    hipMemcpy(c->d_tab32, tab32, sizeof(tab32), hipMemcpyHostToDevice) != hipSuccess ||
	    hipMalloc((void **)&c->d_tab16, sizeof(tab16)) != hipSuccess ||
	    hipMemcpy(c->d_tab16, tab16, sizeof(tab16), hipMemcpyHostToDevice) != hipSuccess) {
		free(tab);
		goto fail;
	}
	free(tab);
	if (cfg->flags & IXG_F_IPV6) {
		uint32_t *t6 = (uint32_t *)malloc(IXG_TAB6_WORDS * sizeof(uint32_t));
		if (!t6) {
			rc = -ENOMEM;
			goto fail;
		}
		hash_table6(cfg, t6);
		if (hipMalloc((void **)&c->d_tab6, IXG_TAB6_WORDS * sizeof(uint32_t)) != hipSuccess ||
		    hipMemcpy(c->d_tab6, t6, IXG_TAB6_WORDS * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
			free(t6);
			goto fail;
		}
		free(t6);
	}
	if (hipMalloc((void **)&c->d_zero, IXG_ZERO_PAGE) != hipSuccess ||
	    hipMemset(c->d_zero, 0, IXG_ZERO_PAGE) != hipSuccess ||
	    hipMalloc((void **)&c->ds.d_present, IXG_PRESENT_WORDS * sizeof(uint32_t)) != hipSuccess ||
	    hipMemset(c->ds.d_present, 0, IXG_PRESENT_WORDS * sizeof(uint32_t)) != hipSuccess)
		goto fail;
	if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
		goto fail;
	{
		const uint32_t none[4] = {0, 0, 0, 0};
		if ((rc = fdir_upload(c, none, 0)) != 0)
			goto fail;
	}
	*out = c;
	return 0;
fail:
	ixg_rx_fini(c);
	return rc;
}

/* ---- batches --------------------------------------------------------------- */

int ixg_dstate_reserve(struct ixg_dstate *ds, size_t nchunks)
{
	if (nchunks <= ds->defer_cap)
		return 0;
	/* hipFree waits for the whole device, i.e. for every other thread's
	 * launches too: the host paths reserve their largest batch when they
	 * allocate (ixgrx_async.c batch_alloc, slot_init) */
	hipFree(ds->d_defer);
	hipFree(ds->d_lenc);
	ds->d_defer = NULL;
	ds->d_lenc = NULL;
	ds->defer_cap = 0;
	ds->lenc = 0;
	const size_t cap = nchunks + nchunks / 4 + 64;
	HIPCHK(hipMalloc((void **)&ds->d_defer, cap));
	HIPCHK(hipMalloc((void **)&ds->d_lenc, cap * 64u * sizeof(uint16_t)));
	ds->defer_cap = cap;
	return 0;
}

int ixg_launch_ds(struct ixg_ctx *c, struct ixg_dstate *ds, const uint8_t *base, const uint64_t *off,
		  const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out, uint32_t *csum,
		  struct ixg_demux_rec *dmx, uint32_t overlap, hipStream_t s)
{
	return ixg_launch_x(c, ds, base, off, len, stride, n, out, csum, dmx, NULL, 0, overlap, NULL, s);
}

int ixg_launch_x(struct ixg_ctx *c, struct ixg_dstate *ds, const uint8_t *base, const uint64_t *off,
		 const uint16_t *len, uint32_t stride, uint32_t n, struct ixg_rx_rec *out, uint32_t *csum,
		 struct ixg_demux_rec *dmx, struct ixg_tcp_ext *ext, uint32_t xflags, uint32_t overlap,
		 const struct ixg_icmp_fuse *ic, hipStream_t s)
{
	struct ixg_kparams p;
	memset(&p, 0, sizeof(p));
	p.base = base;
	p.off = off;
	p.len = len;
	p.out = out;
	p.csum = csum;
	p.tab = c->d_tab;
	p.tab6 = c->d_tab6;
	p.tab32 = c->d_tab32;
	p.tab16 = c->d_tab16;
	p.stride = stride;
	p.n = n;
	p.crc_const = c->crc_const;
	p.flags = c->cfg.flags;
	p.fg_base = (uint32_t)c->cfg.dev_idx * IXG_ETH_MAX_NUM_FG;
	p.fg_mask = (uint32_t)c->cfg.nb_rx_fgs - 1u;
	p.zero = c->d_zero;
	p.fdir = c->d_fdir;
	p.overlap = overlap & 1u;
	p.host_mem = (overlap >> 1) & 1u;
	p.long_only = (overlap & IXG_LF_LONG) ? 1u : 0u;
	if (dmx) {
		p.dmx = dmx;
		p.active_start = c->d_astart;
		p.bline = c->d_bline;
		p.active = c->d_active;
		p.tw = c->d_tw;
		p.listen = c->d_listen;
		p.nfg = c->dmx_nfg;
		p.n_out = c->dmx_nout;
		p.n_listen = c->dmx_nlisten;
	}
	size_t nchunks = ((size_t)n + 63) / 64;
	if (!c->force_general && !(overlap & IXG_LF_LONG)) {
		/* grows once per larger batch; not inside a graph capture */
		int rc = ixg_dstate_reserve(ds, nchunks);
		if (rc)
			return rc;
		p.defer = ds->d_defer;
		p.present = ds->d_present;
		if (++ds->epoch == 0)
			ds->epoch = 1;
		p.epoch = ds->epoch;
		p.force_mode = c->force_mode;
	}
	if (ic) {
		/* the echo replies: the reflect pass behind the RX kernels, marking
		 * the records it answers (replies built in the span-staged kernel
		 * from its registers measured slower: DESIGN.md 8, round 6) */
		if (ixgrx_launch(&p, c->ncu, s) != 0)
			return -EIO;
		struct ixg_iparams ip;
		memset(&ip, 0, sizeof(ip));
		ip.base = (uint8_t *)(uintptr_t)base;
		ip.off = off;
		ip.rec = out;
		ip.stride = stride;
		ip.n = n;
		memcpy(ip.mac, ic->mac, 6);
		const uint32_t be = __builtin_bswap32(ic->host_addr); /* hton32 (icmp.c:55) */
		memcpy(ip.host, &be, 4);
		ip.mark = 1;
		return ixgrx_icmp_launch(&ip, s) == 0 ? 0 : -EIO;
	}
	if (!ext)
		return ixgrx_launch(&p, c->ncu, s) == 0 ? 0 : -EIO;
	/* the tcp_input head: fused into the coalesced fixed-shape kernel, else
	 * the separate pass over the records behind the launch */
	p.ext = ext;
	p.xflags = xflags;
	if (ixgrx_tcpx_fusable(&p))
		return ixgrx_launch(&p, c->ncu, s) == 0 ? 0 : -EIO;
	p.ext = NULL;
	p.xflags = 0;
	if (ixgrx_launch(&p, c->ncu, s) != 0)
		return -EIO;
	struct ixg_xparams xp;
	memset(&xp, 0, sizeof(xp));
	xp.base = (uint8_t *)(uintptr_t)base;
	xp.off = off;
	xp.rec = out;
	xp.ext = ext;
	xp.stride = stride;
	xp.n = n;
	xp.flags = xflags;
	return ixgrx_tcpx_launch(&xp, s) == 0 ? 0 : -EIO;
}

/* the table: header {mask, fg, 0, 0} + slots (ixgrx_internal.h); the
 * device copy is grow-only, so its address (captured by HIP graphs) only
 * changes when a larger set arrives */
static int fdir_upload(struct ixg_ctx *c, const uint32_t *tab, uint32_t slots)
{
	if (slots > c->fdir_cap || !c->d_fdir) {
		hipFree(c->d_fdir);
		c->d_fdir = NULL;
		c->fdir_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_fdir, ((size_t)slots + 1) * 16));
		c->fdir_cap = slots;
	}
	HIPCHK(hipMemcpy(c->d_fdir, tab, ((size_t)slots + 1) * 16, hipMemcpyHostToDevice));
	return 0;
}

int ixg_rx_set_fdir(void *vctx, const struct ixg_fdir_filter *f, uint32_t n, uint16_t cpu_id)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && !f) || n > (1u << 24) || IXG_ETH_MAX_TOTAL_FG + (uint32_t)cpu_id > 0xfffeu)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	/* every launch of this context that may read the table finishes first:
	 * the synchronous paths' stream, the pipelined mbuf path's stages, and
	 * the asynchronous ring (its OPEN batch is launched first, so frames
	 * submitted before this call are matched against the filters they were
	 * submitted under, as frames the NIC received before the filter was
	 * installed) */
	HIPCHK(hipStreamSynchronize(c->stream));
	for (int k = 0; k < IXG_SLOTS; k++)
		if (c->slot[k].stream)
			HIPCHK(hipStreamSynchronize(c->slot[k].stream));
	{
		const int rc = ixg_async_quiesce(c);
		if (rc)
			return rc;
	}
	/* open addressing, load factor <= 1/2, linear probing; duplicates kept
	 * once (a perfect filter matches or not) */
	uint32_t slots = 16;
	while (slots < 2 * n)
		slots <<= 1;
	uint32_t *tab = (uint32_t *)calloc(((size_t)slots + 1) * 4, sizeof(uint32_t));
	if (!tab)
		return -ENOMEM;
	uint32_t *slot = tab + 4;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t ports = (uint32_t)f[i].src_port | ((uint32_t)f[i].dst_port << 16);
		uint32_t k = ixg_fdir_hash(f[i].src_ip, f[i].dst_ip, ports) & (slots - 1);
		while (slot[4 * k + 3] &&
		       !(slot[4 * k] == f[i].src_ip && slot[4 * k + 1] == f[i].dst_ip && slot[4 * k + 2] == ports))
			k = (k + 1) & (slots - 1);
		slot[4 * k] = f[i].src_ip;
		slot[4 * k + 1] = f[i].dst_ip;
		slot[4 * k + 2] = ports;
		slot[4 * k + 3] = 1;
	}
	tab[0] = n ? slots - 1 : 0;
	tab[1] = IXG_ETH_MAX_TOTAL_FG + cpu_id;
	const int rc = fdir_upload(c, tab, n ? slots : 0);
	free(tab);
	return rc;
}

/* ---- host memory the kernels read in place (the asynchronous path) ------- */

int ixg_rx_register_memory(void *vctx, void *base, size_t bytes)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !base || bytes < IXG_MBUF_STRIDE + IXG_TAIL_PAD)
		return -EINVAL;
	if (c->nreg == IXG_MAX_REGIONS)
		return -ENOMEM;
	const uintptr_t lo = (uintptr_t)base, hi = lo + bytes;
	for (uint32_t r = 0; r < c->nreg; r++)
		if (lo < c->reg[r].hi && c->reg[r].lo < hi)
			return -EINVAL; /* overlaps a registered region */
	HIPCHK(hipSetDevice(c->device));
	if (hipHostRegister(base, bytes, hipHostRegisterMapped) != hipSuccess)
		return -EIO;
	void *dev = NULL;
	if (hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
		hipHostUnregister(base);
		return -EIO;
	}
	c->reg[c->nreg].lo = lo;
	c->reg[c->nreg].hi = hi;
	c->reg[c->nreg].delta = (intptr_t)dev - (intptr_t)lo;
	c->nreg++;
	return 0;
}

int ixg_rx_unregister_memory(void *vctx, void *base)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c)
		return -EINVAL;
	for (uint32_t r = 0; r < c->nreg; r++) {
		if (c->reg[r].lo != (uintptr_t)base)
			continue;
		HIPCHK(hipSetDevice(c->device));
		/* no batch of this context may still read it */
		if (c->async && ixg_rx_async_pending(c) > 0)
			return -EBUSY;
		hipHostUnregister(base);
		c->reg[r] = c->reg[--c->nreg];
		return 0;
	}
	return -ENOENT;
}

int ixg_rx_set_split(void *vctx, uint32_t split)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	static const uint32_t mode[] = {IXG_MODE_AUTO, IXG_MODE_FAST, IXG_MODE_SHORT, IXG_MODE_LONG, IXG_MODE_AUTO};
	if (!c || split > IXG_SPLIT_GENERAL)
		return -EINVAL;
	c->force_general = split == IXG_SPLIT_GENERAL;
	c->force_mode = mode[split];
	return 0;
}

int ixg_rx_launch_info(void *vctx, uint32_t info[3])
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !info)
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipStreamSynchronize(c->stream));
	uint32_t w[IXG_PRESENT_WORDS];
	HIPCHK(hipMemcpy(w, c->ds.d_present, sizeof(w), hipMemcpyDeviceToHost));
	const int ran = c->ds.epoch != 0 && w[0] == c->ds.epoch;
	info[0] = ran ? w[3] : 0xffffffffu;
	info[1] = ran && w[6] != 0;
	info[2] = (uint32_t)ran;
	return 0;
}

static int launch(struct ixg_ctx *c, const uint8_t *base, const uint64_t *off, const uint16_t *len,
		  uint32_t stride, uint32_t n, struct ixg_rx_rec *out, uint32_t *csum, hipStream_t s)
{
	return ixg_launch_ds(c, &c->ds, base, off, len, stride, n, out, csum, NULL, 0, s);
}

int ixg_rx_batch_dev(void *vctx, const struct ixg_rx_frames *fr, uint32_t n, struct ixg_rx_rec *d_out,
		     ixg_csum_t *d_csum, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || (n && (!fr->base || !fr->len || !d_out)))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_out & 15) ||
	    ((uintptr_t)fr->len & 1) || ((uintptr_t)fr->off & 7) || ((uintptr_t)d_csum & 3))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -EIO;
	return launch(c, (const uint8_t *)fr->base, fr->off, fr->len, fr->stride, n, d_out, d_csum,
		      (hipStream_t)stream);
}

static int grow_dev(struct ixg_ctx *c, size_t bytes, size_t n)
{
	/* a cap is set only once its buffers exist: a failed allocation leaves
	 * cap 0, so the next call retries instead of launching on NULL */
	if (bytes > c->d_frames_cap) {
		hipFree(c->d_frames);
		c->d_frames = NULL;
		c->d_frames_cap = 0;
		size_t cap = bytes + bytes / 4 + 4096;
		HIPCHK(hipMalloc((void **)&c->d_frames, cap));
		c->d_frames_cap = cap;
	}
	if (n > c->d_n_cap) {
		hipFree(c->d_off);
		hipFree(c->d_len);
		hipFree(c->d_out);
		hipFree(c->d_csum);
		hipFree(c->d_dmx);
		c->d_off = NULL;
		c->d_len = NULL;
		c->d_out = NULL;
		c->d_csum = NULL;
		c->d_dmx = NULL;
		c->d_n_cap = 0;
		c->d_dmx_cap = 0;
		size_t cap = n + n / 4 + 64;
		HIPCHK(hipMalloc((void **)&c->d_off, cap * sizeof(uint64_t)));
		HIPCHK(hipMalloc((void **)&c->d_len, cap * sizeof(uint16_t)));
		HIPCHK(hipMalloc((void **)&c->d_out, cap * sizeof(struct ixg_rx_rec)));
		HIPCHK(hipMalloc((void **)&c->d_csum, cap * sizeof(uint32_t)));
		c->d_n_cap = cap;
	}
	return 0;
}

int ixg_rx_batch_host(void *vctx, const void *frames, const uint64_t *off, const uint16_t *len,
		      uint32_t stride, uint32_t n, struct ixg_rx_rec *out, ixg_csum_t *csum)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && (!frames || !len || !out)))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (((uintptr_t)frames & 3) || (!off && (stride & 3)))
		return -EINVAL;
	uint64_t end = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint64_t o = off ? off[i] : (uint64_t)i * stride;
		if (o & 3)
			return -EINVAL;
		if (o + len[i] > end)
			end = o + len[i];
	}
	/* the caller's buffer need not have IXG_TAIL_PAD: copy what exists and
	 * leave the device copy padded */
	HIPCHK(hipSetDevice(c->device));
	int rc = grow_dev(c, (size_t)end + IXG_TAIL_PAD, n);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(c->d_frames, frames, (size_t)end, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemsetAsync(c->d_frames + end, 0, IXG_TAIL_PAD, c->stream));
	if (off)
		HIPCHK(hipMemcpyAsync(c->d_off, off, n * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->d_len, len, n * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
	rc = launch(c, c->d_frames, off ? c->d_off : NULL, c->d_len, stride, n, c->d_out,
		    csum ? c->d_csum : NULL, c->stream);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(out, c->d_out, n * sizeof(*out), hipMemcpyDeviceToHost, c->stream));
	if (csum)
		HIPCHK(hipMemcpyAsync(csum, c->d_csum, n * sizeof(*csum), hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

/* ---- the IX-layout gather ------------------------------ */

int ixg_check_mbufs(void *const *mbufs, uint32_t n)
{
	for (uint32_t i = 0; i < n; i++) {
		if (i + IXG_MBUF_PREFETCH < n)
			__builtin_prefetch(mbufs[i + IXG_MBUF_PREFETCH]);
		size_t l;
		memcpy(&l, mbufs[i], sizeof(l));
		if (l > IXG_MBUF_DATA_LEN) /* an mbuf holds at most 2048 data bytes (mbuf.h) */
			return -EINVAL;
	}
	return 0;
}

/* one frame into the staging at pos: its bytes [12, ixg_stage_ext) */
static inline size_t gather_one(uint8_t *frames, size_t pos, const uint8_t *mb, size_t l, size_t *hi)
{
	if (pos + l > *hi)
		*hi = pos + l;
	if (l <= 12)
		return pos;
	const uint8_t *f = mb + IXG_MBUF_HEADER_LEN;
	const size_t e = ixg_stage_ext(f, l);
	memcpy(frames + pos + 12, f + 12, e - 12);
	return pos + ((e - 12 + 3) & ~(size_t)3);
}

size_t ixg_gather_mbufs(uint8_t *frames, size_t pos, void *const *mbufs, uint32_t n, uint32_t avail, uint64_t *off,
			uint16_t *len, size_t *hi)
{
	for (uint32_t k = 0; k < n; k++) {
		if (k + IXG_MBUF_PREFETCH < avail) { /* the mbuf header line (len) and the frame's line */
			__builtin_prefetch(mbufs[k + IXG_MBUF_PREFETCH]);
			__builtin_prefetch((const uint8_t *)mbufs[k + IXG_MBUF_PREFETCH] + IXG_MBUF_HEADER_LEN);
		}
		const uint8_t *mb = (const uint8_t *)mbufs[k];
		size_t l;
		memcpy(&l, mb, sizeof(l)); /* mbuf->len (inc/ix/mbuf.h:75) */
		off[k] = pos;
		len[k] = (uint16_t)l;
		pos = gather_one(frames, pos, mb, l, hi);
	}
	return pos;
}

size_t ixg_gather_mbufs_zc(const struct ixg_ctx *c, uint8_t *frames, size_t pos, void *const *mbufs, uint32_t n,
			   uint32_t avail, uint64_t *off, uint16_t *len, size_t *hi, uint32_t *nabs, size_t *link)
{
	uint32_t in_place = 0;
	size_t lb = 0;
	for (uint32_t k = 0; k < n; k++) {
		if (k + IXG_MBUF_PREFETCH < avail) /* the header line: frames read in place need no more */
			__builtin_prefetch(mbufs[k + IXG_MBUF_PREFETCH]);
		const uint8_t *mb = (const uint8_t *)mbufs[k];
		const uintptr_t a = (uintptr_t)mb;
		size_t l;
		memcpy(&l, mb, sizeof(l)); /* mbuf->len (inc/ix/mbuf.h:75) */
		len[k] = (uint16_t)l;
		/* frames shorter than IXG_ZC_MIN_LEN are gathered (cheaper than the
		 * kernels' host-link reads of them in place) */
		uint32_t r = l < IXG_ZC_MIN_LEN ? c->nreg : 0;
		/* the mbuf and the bytes the kernels may read past its frame inside
		 * the region (ixg_rx_register_memory) */
		while (r < c->nreg && !(a >= c->reg[r].lo && a + IXG_MBUF_STRIDE + IXG_TAIL_PAD <= c->reg[r].hi))
			r++;
		if (r < c->nreg && !(a & 3)) {
			off[k] = ((uint64_t)(a + IXG_MBUF_HEADER_LEN) + (uint64_t)c->reg[r].delta) | IXG_OFF_ABS;
			in_place++;
			lb += (l + 63u) & ~(size_t)63;
			continue;
		}
		off[k] = pos;
		pos = gather_one(frames, pos, mb, l, hi);
	}
	*nabs += in_place;
	*link += lb;
	return pos;
}

/* the end of the image's frame bytes: the staged span, the furthest frame
 * end (a frame's bytes past ixg_stage_ext are not staged, but the kernels'
 * loads may reach them), then IXG_TAIL_PAD zero bytes; returns where the
 * offsets / lengths may start */
static size_t frames_tail(uint8_t *buf, size_t span, size_t hi)
{
	const size_t end = span + 12 > hi ? span + 12 : hi;
	memset(buf + span + 12, 0, end - (span + 12) + IXG_TAIL_PAD + 16);
	return (end + IXG_TAIL_PAD + 16 + 7) & ~(size_t)7;
}

void ixg_stage_finish_abs(uint8_t *buf, size_t span, size_t hi, const uint64_t *off, const uint16_t *len, uint32_t n,
			  struct ixg_stage *st)
{
	st->o_off = frames_tail(buf, span, hi);
	/* the gathered offsets stay as they are (a failed launch lays the run
	 * out again): the image gets them rebased */
	uint64_t *o = (uint64_t *)(buf + st->o_off);
	uint64_t lo = ~0ull;
	uint32_t lmin = 0xffffu;
	for (uint32_t k = 0; k < n; k++) {
		o[k] = (off[k] & IXG_OFF_ABS) ? (off[k] & ~IXG_OFF_ABS) : (uint64_t)(uintptr_t)buf + off[k];
		if (o[k] < lo)
			lo = o[k];
		if (len[k] < lmin)
			lmin = len[k];
	}
	st->lmin = lmin;
	lo &= ~(uint64_t)15;
	for (uint32_t k = 0; k < n; k++)
		o[k] -= lo;
	st->base = lo;
	st->stride = 0;
	st->lconst = 0;
	st->o_len = st->o_off + (size_t)n * sizeof(uint64_t);
	memcpy(buf + st->o_len, len, (size_t)n * sizeof(uint16_t));
	st->h2d = st->o_len + (size_t)n * sizeof(uint16_t);
}

void ixg_stage_finish(uint8_t *buf, size_t span, size_t hi, const uint64_t *off, const uint16_t *len, uint32_t n,
		      struct ixg_stage *st)
{
	st->base = 0;
	const size_t frames_end = frames_tail(buf, span, hi);
	st->o_off = frames_end;
	/* fixed stride when every frame sits at k * stride (frames staging the
	 * same byte count; the last may differ) and none runs more than 64 bytes
	 * past its slot (ixg_kparams.overlap) */
	const uint64_t s = n > 1 ? off[1] - off[0] : span;
	int uniform = off[0] == 0;
	uint32_t lmin = 0xffffu, lmax = 0;
	for (uint32_t k = 0; k < n; k++) {
		/* s == 0 (every offset 0): only a run of frames that stage nothing
		 * (<= 12 bytes) is uniform; a longer frame staged its bytes at 0 and
		 * would be wiped by the zeroed slots below */
		uniform = uniform && off[k] == (uint64_t)k * s && len[k] <= s + 64u && (s || len[k] <= 12u);
		lmin = len[k] < lmin ? len[k] : lmin;
		lmax = len[k] > lmax ? len[k] : lmax;
	}
	st->lmin = lmin;
	/* a fixed-stride run of one length (a flood of equal frames) sends no
	 * lengths: 2 bytes per frame less over the host link */
	st->lconst = uniform && n && lmin == lmax ? lmin : 0u;
	if (uniform) {
		st->stride = s ? (uint32_t)s : 4;
		if (!s) /* frames of <= 12 bytes: nothing staged, slots of 4 zero bytes */
			memset(buf, 0, (size_t)n * 4 + IXG_TAIL_PAD + 16);
		st->o_len = frames_end > (size_t)n * 4 + IXG_TAIL_PAD + 16 ? frames_end : ((size_t)n * 4 + IXG_TAIL_PAD + 24) & ~(size_t)7;
	} else {
		st->stride = 0;
		memcpy(buf + st->o_off, off, (size_t)n * sizeof(uint64_t));
		st->o_len = st->o_off + (size_t)n * sizeof(uint64_t);
	}
	if (st->lconst) {
		st->h2d = st->o_len;
		return;
	}
	memcpy(buf + st->o_len, len, (size_t)n * sizeof(uint16_t));
	st->h2d = st->o_len + (size_t)n * sizeof(uint16_t);
}

/* ---- the synchronous IX-layout host path ---------------------------------- */

/* ixg_rx_batch_mbufs, pipelined: the batch goes through the device in chunks
 * of at most IXG_PIPE_FRAMES frames / IXG_PIPE_BYTES gathered bytes,
 * alternating between IXG_SLOTS stages, so the CPU gathers chunk k+1 out of
 * the mbufs into pinned staging while chunk k's H2D copy (one per chunk),
 * kernels and D2H copy of records run on the stage's stream. */
#define IXG_PIPE_FRAMES 131072u
#define IXG_PIPE_BYTES (64u << 20)

static int slot_init(struct ixg_slot *sl)
{
	/* ready only once every buffer exists: a failed allocation is retried
	 * on the next call (buffers already made are kept, the rest made) */
	if (sl->ready)
		return 0;
	if (!sl->stream)
		HIPCHK(hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking));
	if (!sl->done)
		HIPCHK(hipEventCreateWithFlags(&sl->done, hipEventDisableTiming));
	if (!sl->ds.d_present) {
		HIPCHK(hipMalloc((void **)&sl->ds.d_present, IXG_PRESENT_WORDS * sizeof(uint32_t)));
		HIPCHK(hipMemset(sl->ds.d_present, 0, IXG_PRESENT_WORDS * sizeof(uint32_t)));
	}
	int rc = ixg_dstate_reserve(&sl->ds, (IXG_PIPE_FRAMES + 63u) / 64u);
	if (rc)
		return rc;
	const size_t bcap = IXG_STAGE_BYTES(IXG_PIPE_BYTES + 256u * 2048u, IXG_PIPE_FRAMES), ncap = IXG_PIPE_FRAMES;
	if (!sl->h_buf)
		HIPCHK(hipHostMalloc((void **)&sl->h_buf, bcap, hipHostMallocDefault));
	if (!sl->d_buf)
		HIPCHK(hipMalloc((void **)&sl->d_buf, bcap));
	if (!sl->h_off && !(sl->h_off = (uint64_t *)malloc(ncap * sizeof(uint64_t))))
		return -ENOMEM;
	if (!sl->h_len && !(sl->h_len = (uint16_t *)malloc(ncap * sizeof(uint16_t))))
		return -ENOMEM;
	if (!sl->h_rec)
		HIPCHK(hipHostMalloc((void **)&sl->h_rec, ncap * sizeof(struct ixg_rx_rec), hipHostMallocDefault));
	if (!sl->d_rec)
		HIPCHK(hipMalloc((void **)&sl->d_rec, ncap * sizeof(struct ixg_rx_rec)));
	sl->ready = 1;
	return 0;
}

static void ixg_slot_free(struct ixg_slot *sl)
{
	if (sl->stream)
		hipStreamSynchronize(sl->stream);
	ixg_dstate_free(&sl->ds);
	hipHostFree(sl->h_buf);
	hipHostFree(sl->h_rec);
	hipFree(sl->d_buf);
	hipFree(sl->d_rec);
	free(sl->h_off);
	free(sl->h_len);
	if (sl->done)
		hipEventDestroy(sl->done);
	if (sl->stream)
		hipStreamDestroy(sl->stream);
	memset(sl, 0, sizeof(*sl));
}

/* wait for a stage's chunk and hand its records to the caller */
static int slot_take(struct ixg_slot *sl, struct ixg_rx_rec *out)
{
	if (!sl->busy)
		return 0;
	sl->busy = 0;
	HIPCHK(hipEventSynchronize(sl->done));
	memcpy(out + sl->first, sl->h_rec, (size_t)sl->n * sizeof(*out));
	return 0;
}

/* enqueue one staged image: H2D, kernels, the echo reflect over ic's
 * candidates, D2H of records (the stream's work) */
int ixg_stage_launch(struct ixg_ctx *c, struct ixg_dstate *ds, const struct ixg_stage *st, uint8_t *h_buf,
		     uint8_t *d_buf, uint32_t n, struct ixg_rx_rec *d_rec, struct ixg_rx_rec *h_rec, int direct,
		     const struct ixg_icmp_items *ic, uint32_t *done_flag, uint32_t done_val, hipStream_t s)
{
	uint8_t *img = d_buf;
	if (direct) {
		img = h_buf; /* the kernels read the pinned image over the host link */
	} else {
		if (st->base)
			return -EINVAL; /* in-place frames are for kernels on host memory only */
		HIPCHK(hipMemcpyAsync(d_buf, h_buf, st->h2d, hipMemcpyHostToDevice, s));
	}
	/* frames: the image, or (in-place frames) offsets from st->base */
	const uint8_t *frames = st->base ? (const uint8_t *)(uintptr_t)st->base : img;
	const uint16_t *lens = (const uint16_t *)(img + st->o_len);
	if (st->lconst) {
		/* one length for the run: the lengths come from device memory,
		 * filled (on this stream, before the kernels) when it changes */
		int rc = ixg_dstate_reserve(ds, ((size_t)n + 63) / 64);
		if (rc)
			return rc;
		if (ds->lenc != st->lconst) {
			HIPCHK(hipMemsetD16Async((hipDeviceptr_t)ds->d_lenc, (unsigned short)st->lconst, ds->defer_cap * 64u,
						 s));
			ds->lenc = st->lconst;
		}
		lens = ds->d_lenc;
	}
	int rc = ixg_launch_ds(c, ds, frames, st->stride ? NULL : (const uint64_t *)(img + st->o_off), lens,
			       st->stride, n, direct ? h_rec : d_rec, NULL, NULL,
			       (st->stride ? IXG_LF_OVERLAP : 0u) | (direct ? IXG_LF_HOST : 0u) |
				       (st->lmin >= IXG_LONG_ONLY_LEN && c->force_mode == IXG_MODE_AUTO ? IXG_LF_LONG : 0u),
			       s);
	if (rc)
		return rc;
	if (ic && ic->n) {
		/* icmp_input's reflect (icmp.c:88-92) for the batch's echo
		 * requests, in their mbufs, before the records are handed back */
		struct ixg_iparams p;
		memset(&p, 0, sizeof(p));
		p.off = ic->addr;
		p.idx = ic->idx;
		p.rec = direct ? h_rec : d_rec;
		p.n = ic->n;
		p.mark = 1;
		memcpy(p.mac, c->icmp_mac, 6);
		const uint32_t be = __builtin_bswap32(c->icmp_host); /* hton32 (icmp.c:55) */
		memcpy(p.host, &be, 4);
		if (ixgrx_icmp_launch(&p, s) != 0)
			return -EIO;
	}
	int fail = 0;
	if (!direct &&
	    hipMemcpyAsync(h_rec, d_rec, (size_t)n * sizeof(struct ixg_rx_rec), hipMemcpyDeviceToHost, s) != hipSuccess)
		fail = 1;
	if (!fail && done_flag && ixgrx_stamp(done_flag, done_val, s) != 0)
		fail = 1;
	if (!fail)
		return 0;
	if (!(ic && ic->n))
		return -EIO; /* nothing enqueued has changed an mbuf: the caller may launch the batch again */
	/* the reflect is enqueued: the mbufs become replies, so the batch cannot
	 * be launched again (the parse would read the replies and the reflect
	 * would swap them back). Complete it here: wait for the
	 * stream, take the records, store the completion word from the host. */
	if (hipStreamSynchronize(s) != hipSuccess)
		return -EPIPE; /* the device failed under the batch: not retryable */
	if (!direct && hipMemcpy(h_rec, d_rec, (size_t)n * sizeof(struct ixg_rx_rec), hipMemcpyDeviceToHost) != hipSuccess)
		return -EPIPE;
	if (done_flag)
		__atomic_store_n(done_flag, done_val, __ATOMIC_RELEASE);
	return 0;
}

int ixg_rx_batch_mbufs(void *vctx, void *const *mbufs, uint32_t n, struct ixg_rx_rec *out)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && (!mbufs || !out)))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (ixg_check_mbufs(mbufs, n))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	int rc = 0;
	uint32_t i = 0, k = 0;
	while (i < n && !rc) {
		struct ixg_slot *sl = &c->slot[k % IXG_SLOTS];
		if ((rc = slot_init(sl)) || (rc = slot_take(sl, out)))
			break;
		/* the chunk: at most IXG_PIPE_FRAMES frames, IXG_PIPE_BYTES bytes */
		uint32_t m = n - i < IXG_PIPE_FRAMES ? n - i : IXG_PIPE_FRAMES;
		size_t span = 0, hi = 0;
		uint32_t done = 0;
		while (done < m && span <= IXG_PIPE_BYTES) {
			const uint32_t step = m - done < 256u ? m - done : 256u;
			span = ixg_gather_mbufs(sl->h_buf, span, mbufs + i + done, step, n - i - done, sl->h_off + done,
						sl->h_len + done, &hi);
			done += step;
		}
		m = done;
		struct ixg_stage st;
		ixg_stage_finish(sl->h_buf, span, hi, sl->h_off, sl->h_len, m, &st);
		if ((rc = ixg_stage_launch(c, &sl->ds, &st, sl->h_buf, sl->d_buf, m, sl->d_rec, sl->h_rec, 0, NULL, NULL, 0,
					   sl->stream)))
			break;
		if (hipEventRecord(sl->done, sl->stream) != hipSuccess) {
			rc = -EIO;
			break;
		}
		sl->first = i;
		sl->n = m;
		sl->busy = 1;
		i += m;
		k++;
	}
	/* drain, oldest stage first */
	for (uint32_t t = 0; t < IXG_SLOTS; t++) {
		int r2 = slot_take(&c->slot[(k + t) % IXG_SLOTS], out);
		if (!rc)
			rc = r2;
	}
	return rc;
}

/* ---- dispatch: what eth_process_recv does per packet, from records ------ */

uint32_t ixg_rx_dispatch(void *const *mbufs, const struct ixg_rx_rec *recs, uint32_t n,
			 const struct ixg_rx_ops *ops, void *user)
{
	uint32_t delivered = 0;
	if (!ops)
		return 0;
	for (uint32_t i = 0; i < n; i++) {
		const struct ixg_rx_rec *r = &recs[i];
		void (*fn)(void *, void *, const struct ixg_rx_rec *) = ops->drop;
		switch (r->verdict) {
		case IXG_V_TCP:
		case IXG_V_TCP6:
			fn = ops->tcp; /* tcp_input_tmp -> tcp_input body (ip.c:93-96) */
			break;
		case IXG_V_UDP:
		case IXG_V_UDP6:
			fn = ops->udp; /* udp_input (ip.c:97-100) */
			break;
		case IXG_V_ICMP_ECHO:
			fn = ops->icmp_echo; /* icmp_input -> icmp_reflect (icmp.c:89-92) */
			break;
		case IXG_V_ARP:
			fn = ops->arp; /* arp_input (ip.c:134-135) */
			break;
		default:
			break;
		}
		if (r->verdict < 0x80)
			delivered++;
		if (fn)
			fn(user, mbufs ? mbufs[i] : NULL, r);
	}
	return delivered;
}

/* ---- PCB demux (tcp_in.c:233-323, 500-510) --------------------------------- */

static int upload(void **dst, const void *src, size_t bytes)
{
	hipFree(*dst);
	*dst = NULL;
	if (!bytes)
		return 0;
	HIPCHK(hipMalloc(dst, bytes));
	HIPCHK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
	return 0;
}

/* tcp_to_idx of a pcb (inc/lwip/lwip/tcp_impl.h:371-387): the crc32q stream
 * of local ip, remote ip and (int)(local_port << 16 | remote_port), as the
 * kernels compute it from a segment's tuple through the byte tables
 * (ixg_rx_hash_tables: k_crc_pos) */
static uint32_t pcb_bucket_of(const struct ixg_pcb_key *k)
{
	uint8_t s[24];
	memset(s, 0, sizeof(s));
	memcpy(s, &k->local_ip, 4);
	memcpy(s + 8, &k->remote_ip, 4);
	const uint32_t ports = (uint32_t)k->remote_port | ((uint32_t)k->local_port << 16);
	memcpy(s + 16, &ports, 4);
	if (ports & 0x80000000u)
		memset(s + 20, 0xff, 4);
	return crc_stream(IXG_PCB_HASH_SEED, s) & (IXG_PCB_BUCKETS - 1u);
}

static int csr_ok(const uint32_t *start, size_t rows)
{
	if (!start || start[0] != 0)
		return 0;
	for (size_t r = 0; r < rows; r++)
		if (start[r + 1] < start[r])
			return 0;
	return 1;
}

int ixg_demux_load(void *vctx, const struct ixg_demux_tables *t)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !t || t->nfg > IXG_ETH_MAX_NUM_FG || t->n_out > IXG_MAX_OUTBOUND)
		return -EINVAL;
	const size_t ng = (size_t)t->nfg + t->n_out; /* local groups, then outbound */
	const size_t na_rows = ng * IXG_PCB_BUCKETS;
	if (!csr_ok(t->active_start, na_rows) || !csr_ok(t->tw_start, ng))
		return -EINVAL;
	const size_t na = t->active_start[na_rows], ntw = t->tw_start[ng];
	if ((na && !t->active) || (ntw && !t->tw) || (t->n_listen && !t->listen))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	HIPCHK(hipStreamSynchronize(c->stream));
	c->demux_loaded = 0;
	int rc;
	if ((rc = upload((void **)&c->d_astart, t->active_start, (na_rows + 1) * sizeof(uint32_t))) ||
	    (rc = upload((void **)&c->d_active, t->active, na * sizeof(struct ixg_pcb_key))) ||
	    (rc = upload((void **)&c->d_listen, t->listen, (size_t)t->n_listen * sizeof(struct ixg_listen_key))))
		return rc;
	/* the bucket lines (ixgrx_walk.h): count, CSR start, the bucket's
	 * TIME-WAIT run (count, start), the first 3 entries of each active list,
	 * in list order */
	uint32_t *bl = (uint32_t *)calloc(na_rows ? na_rows : 1, 64);
	/* each group's TIME-WAIT list split into per-bucket runs, list order kept
	 * within a run (a counting sort by row = group * 512 + bucket) */
	uint32_t *twrow = (uint32_t *)malloc((ntw ? ntw : 1) * sizeof(uint32_t));
	struct ixg_pcb_key *tw2 = (struct ixg_pcb_key *)malloc((ntw ? ntw : 1) * sizeof(struct ixg_pcb_key));
	if (!bl || !twrow || !tw2) {
		free(bl);
		free(twrow);
		free(tw2);
		return -ENOMEM;
	}
	for (size_t r = 0; r < na_rows; r++) {
		const uint32_t s0 = t->active_start[r], cnt = t->active_start[r + 1] - s0;
		uint32_t *row = bl + 16 * r;
		row[0] = cnt;
		row[1] = s0;
		for (uint32_t k = 0; k < cnt && k < 3; k++)
			memcpy(row + 4 + 4 * k, &t->active[s0 + k], sizeof(struct ixg_pcb_key));
	}
	for (size_t g = 0; g < ng; g++)
		for (uint32_t k = t->tw_start[g]; k < t->tw_start[g + 1]; k++) {
			twrow[k] = (uint32_t)(g * IXG_PCB_BUCKETS) + pcb_bucket_of(&t->tw[k]);
			bl[16 * (size_t)twrow[k] + 2]++;
		}
	uint32_t run = 0;
	for (size_t r = 0; r < na_rows; r++) {
		bl[16 * r + 3] = run;
		run += bl[16 * r + 2];
		bl[16 * r + 2] = 0; /* refilled as the entries are placed */
	}
	for (size_t k = 0; k < ntw; k++) {
		uint32_t *row = bl + 16 * (size_t)twrow[k];
		tw2[row[3] + row[2]++] = t->tw[k];
	}
	rc = upload((void **)&c->d_bline, bl, na_rows * 64);
	if (!rc)
		rc = upload((void **)&c->d_tw, tw2, ntw * sizeof(struct ixg_pcb_key));
	free(bl);
	free(twrow);
	free(tw2);
	if (rc)
		return rc;
	c->dmx_nfg = t->nfg;
	c->dmx_nout = t->n_out;
	c->dmx_nlisten = t->n_listen;
	c->demux_loaded = 1;
	return 0;
}

static int demux_launch(struct ixg_ctx *c, const uint8_t *base, const uint64_t *off, uint32_t stride, uint32_t n,
			const struct ixg_rx_rec *rec, struct ixg_demux_rec *out, hipStream_t s)
{
	struct ixg_dparams p;
	memset(&p, 0, sizeof(p));
	p.base = base;
	p.off = off;
	p.rec = rec;
	p.out = out;
	p.active_start = c->d_astart;
	p.bline = c->d_bline;
	p.active = c->d_active;
	p.tw = c->d_tw;
	p.listen = c->d_listen;
	p.stride = stride;
	p.n = n;
	p.fg_base = (uint32_t)c->cfg.dev_idx * IXG_ETH_MAX_NUM_FG;
	p.nfg = c->dmx_nfg;
	p.n_out = c->dmx_nout;
	p.n_listen = c->dmx_nlisten;
	return ixgrx_demux_launch(&p, c->ncu, s) == 0 ? 0 : -EIO;
}

int ixg_demux_batch_dev(void *vctx, const struct ixg_rx_frames *fr, const struct ixg_rx_rec *d_rec, uint32_t n,
			struct ixg_demux_rec *d_out, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || (n && (!fr->base || !d_rec || !d_out)))
		return -EINVAL;
	if (!c->demux_loaded)
		return -ENOENT;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_rec & 15) ||
	    ((uintptr_t)d_out & 7) || ((uintptr_t)fr->off & 7))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	return demux_launch(c, (const uint8_t *)fr->base, fr->off, fr->stride, n, d_rec, d_out, (hipStream_t)stream);
}

int ixg_rx_demux_batch_dev(void *vctx, const struct ixg_rx_frames *fr, uint32_t n, struct ixg_rx_rec *d_out,
			   struct ixg_demux_rec *d_dmx, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || (n && (!fr->base || !fr->len || !d_out || !d_dmx)))
		return -EINVAL;
	if (!c->demux_loaded)
		return -ENOENT;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_out & 15) ||
	    ((uintptr_t)fr->len & 1) || ((uintptr_t)fr->off & 7) || ((uintptr_t)d_dmx & 7))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -EIO;
	return ixg_launch_ds(c, &c->ds, (const uint8_t *)fr->base, fr->off, fr->len, fr->stride, n, d_out, NULL, d_dmx,
			     0, (hipStream_t)stream);
}

/* ---- the rest of the tcp_input head (tcp_in.c:230-241) ---------------------- */

int ixg_rx_tcpx_batch_dev(void *vctx, const struct ixg_rx_frames *fr, uint32_t n, struct ixg_rx_rec *d_out,
			  struct ixg_tcp_ext *d_ext, uint32_t flags, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || (n && (!fr->base || !fr->len || !d_out || !d_ext)) || (flags & ~IXG_TCPX_INPLACE))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_out & 15) ||
	    ((uintptr_t)fr->len & 1) || ((uintptr_t)fr->off & 7) || ((uintptr_t)d_ext & 15))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -EIO;
	return ixg_launch_x(c, &c->ds, (const uint8_t *)fr->base, fr->off, fr->len, fr->stride, n, d_out, NULL, NULL,
			    d_ext, flags, 0, NULL, (hipStream_t)stream);
}

int ixg_rx_icmp_batch_dev(void *vctx, const struct ixg_rx_frames *fr, uint32_t n, struct ixg_rx_rec *d_out,
			  const uint8_t mac[6], uint32_t host_addr, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || !mac || (n && (!fr->base || !fr->len || !d_out)))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_out & 15) ||
	    ((uintptr_t)fr->len & 1) || ((uintptr_t)fr->off & 7))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -EIO;
	struct ixg_icmp_fuse ic;
	memcpy(ic.mac, mac, 6);
	ic.host_addr = host_addr;
	return ixg_launch_x(c, &c->ds, (const uint8_t *)fr->base, fr->off, fr->len, fr->stride, n, d_out, NULL, NULL,
			    NULL, 0, 0, &ic, (hipStream_t)stream);
}

int ixg_tcp_ext_batch_dev(void *vctx, const struct ixg_rx_frames *fr, const struct ixg_rx_rec *d_rec, uint32_t n,
			  struct ixg_tcp_ext *d_ext, uint32_t flags, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || (n && (!fr->base || !d_rec || !d_ext)) || (flags & ~IXG_TCPX_INPLACE))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (((uintptr_t)fr->base & 3) || (!fr->off && (fr->stride & 3)) || ((uintptr_t)d_rec & 15) ||
	    ((uintptr_t)d_ext & 15) || ((uintptr_t)fr->off & 7))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	struct ixg_xparams p;
	memset(&p, 0, sizeof(p));
	p.base = (uint8_t *)(uintptr_t)fr->base;
	p.off = fr->off;
	p.rec = d_rec;
	p.ext = d_ext;
	p.stride = fr->stride;
	p.n = n;
	p.flags = flags;
	return ixgrx_tcpx_launch(&p, stream) == 0 ? 0 : -EIO;
}

int ixg_rx_set_icmp_reply(void *vctx, const uint8_t mac[6], uint32_t host_addr)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !mac)
		return -EINVAL;
	memcpy(c->icmp_mac, mac, 6);
	c->icmp_host = host_addr;
	return 0;
}

int ixg_icmp_reflect_dev(void *vctx, const struct ixg_rx_frames *fr, const struct ixg_rx_rec *d_rec, uint32_t n,
			 const uint8_t mac[6], uint32_t host_addr, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || !mac || (n && (!fr->base || !d_rec)) || ((uintptr_t)d_rec & 7) || ((uintptr_t)fr->off & 7))
		return -EINVAL;
	if (n == 0)
		return 0;
	HIPCHK(hipSetDevice(c->device));
	struct ixg_iparams p;
	memset(&p, 0, sizeof(p));
	p.base = (uint8_t *)(uintptr_t)fr->base;
	p.off = fr->off;
	p.rec = (struct ixg_rx_rec *)(uintptr_t)d_rec; /* read only: p.mark is 0 */
	p.stride = fr->stride;
	p.n = n;
	memcpy(p.mac, mac, 6);
	const uint32_t be = __builtin_bswap32(host_addr); /* hton32 (icmp.c:55) */
	memcpy(p.host, &be, 4);
	return ixgrx_icmp_launch(&p, stream) == 0 ? 0 : -EIO;
}

int ixg_demux_batch_host(void *vctx, const void *frames, const uint64_t *off, const uint16_t *len, uint32_t stride,
			 uint32_t n, const struct ixg_rx_rec *rec, struct ixg_demux_rec *out)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && (!frames || !len || !rec || !out)))
		return -EINVAL;
	if (!c->demux_loaded)
		return -ENOENT;
	if (n == 0)
		return 0;
	if (((uintptr_t)frames & 3) || (!off && (stride & 3)))
		return -EINVAL;
	uint64_t end = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint64_t o = off ? off[i] : (uint64_t)i * stride;
		if (o & 3)
			return -EINVAL;
		if (o + len[i] > end)
			end = o + len[i];
	}
	HIPCHK(hipSetDevice(c->device));
	int rc = grow_dev(c, (size_t)end + IXG_TAIL_PAD, n);
	if (rc)
		return rc;
	if (n > c->d_dmx_cap) {
		hipFree(c->d_dmx);
		c->d_dmx = NULL;
		c->d_dmx_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_dmx, (size_t)c->d_n_cap * sizeof(struct ixg_demux_rec)));
		c->d_dmx_cap = c->d_n_cap; /* grow_dev zeroes it whenever it reallocates */
	}
	HIPCHK(hipMemcpyAsync(c->d_frames, frames, (size_t)end, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemsetAsync(c->d_frames + end, 0, IXG_TAIL_PAD, c->stream));
	if (off)
		HIPCHK(hipMemcpyAsync(c->d_off, off, n * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->d_out, rec, n * sizeof(*rec), hipMemcpyHostToDevice, c->stream));
	rc = demux_launch(c, c->d_frames, off ? c->d_off : NULL, stride, n, c->d_out, c->d_dmx, c->stream);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(out, c->d_dmx, n * sizeof(*out), hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

/* ---- TX header build + checksums ----------------------- */

int ixg_tx_set_macs(void *vctx, const uint8_t src_mac[6], const uint8_t *dmacs, uint32_t n_dmac)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !src_mac || (n_dmac && !dmacs))
		return -EINVAL;
	uint32_t *rows = (uint32_t *)calloc(n_dmac ? 2u * n_dmac : 2u, sizeof(uint32_t));
	if (!rows)
		return -ENOMEM;
	for (uint32_t i = 0; i < n_dmac; i++)
		memcpy(rows + 2u * i, dmacs + 6u * i, 6);
	HIPCHK(hipSetDevice(c->device));
	hipFree(c->d_dmacs);
	c->d_dmacs = NULL;
	c->n_dmac = 0;
	if (hipMalloc((void **)&c->d_dmacs, (n_dmac ? n_dmac : 1u) * 8u) != hipSuccess ||
	    hipMemcpy(c->d_dmacs, rows, (n_dmac ? n_dmac : 1u) * 8u, hipMemcpyHostToDevice) != hipSuccess) {
		free(rows);
		return -ENOMEM;
	}
	free(rows);
	c->n_dmac = n_dmac;
	memcpy(&c->smac_lo, src_mac, 4);
	c->smac_hi = (uint32_t)src_mac[4] | ((uint32_t)src_mac[5] << 8);
	return 0;
}

static int tx_launch(struct ixg_ctx *c, const void *seg_buf, const struct ixg_tx_seg *segs, uint32_t n, void *out,
		     uint16_t *out_len, uint32_t flags, hipStream_t s)
{
	struct ixg_tparams p;
	memset(&p, 0, sizeof(p));
	p.seg_buf = (const uint8_t *)seg_buf;
	p.segs = segs;
	p.out = (uint8_t *)out;
	p.out_len = out_len;
	p.dmacs = c->d_dmacs;
	p.n = n;
	p.n_dmac = c->n_dmac;
	p.smac_lo = c->smac_lo;
	p.smac_hi = c->smac_hi;
	p.flags = flags;
	p.zero = c->d_zero;
	return ixgrx_tx_launch(&p, c->ncu, s) == 0 ? 0 : -EIO;
}

int ixg_tx_batch_dev(void *vctx, const void *seg_buf, const struct ixg_tx_seg *segs, uint32_t n, void *out,
		     uint16_t *out_len, uint32_t flags, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && (!seg_buf || !segs || !out || !out_len)) || (flags & ~IXG_TX_OFFLOAD))
		return -EINVAL;
	if (!c->d_dmacs)
		return -ENOENT;
	if (n == 0)
		return 0;
	HIPCHK(hipSetDevice(c->device));
	return tx_launch(c, seg_buf, segs, n, out, out_len, flags, (hipStream_t)stream);
}

int ixg_tx_batch_host(void *vctx, const void *seg_buf, size_t seg_buf_len, const struct ixg_tx_seg *segs,
		      uint32_t n, void *out, size_t out_size, uint16_t *out_len, uint32_t flags)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || (n && (!seg_buf || !segs || !out || !out_len)) || (flags & ~IXG_TX_OFFLOAD))
		return -EINVAL;
	if (!c->d_dmacs)
		return -ENOENT;
	if (n == 0)
		return 0;
	/* frames must fit the output (the kernel writes whole 16-byte pieces) */
	for (uint32_t i = 0; i < n; i++) {
		uint64_t span = 34u + (uint64_t)segs[i].seg_len + (segs[i].proto == 17 ? 8u : 0u);
		if (segs[i].out_off + ((span + 15u) & ~(uint64_t)15u) > out_size ||
		    segs[i].seg_off + segs[i].seg_len > seg_buf_len)
			return -EINVAL;
	}
	HIPCHK(hipSetDevice(c->device));
	if (seg_buf_len + IXG_TAIL_PAD > c->d_txbuf_cap) {
		hipFree(c->d_txbuf);
		c->d_txbuf = NULL;
		c->d_txbuf_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_txbuf, seg_buf_len + IXG_TAIL_PAD));
		c->d_txbuf_cap = seg_buf_len + IXG_TAIL_PAD;
	}
	if (out_size > c->d_txout_cap) {
		hipFree(c->d_txout);
		c->d_txout = NULL;
		c->d_txout_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_txout, out_size));
		c->d_txout_cap = out_size;
	}
	if (n > c->d_txn_cap) {
		hipFree(c->d_txsegs);
		hipFree(c->d_txlen);
		c->d_txsegs = NULL;
		c->d_txlen = NULL;
		c->d_txn_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_txsegs, (size_t)n * sizeof(struct ixg_tx_seg)));
		HIPCHK(hipMalloc((void **)&c->d_txlen, (size_t)n * sizeof(uint16_t)));
		c->d_txn_cap = n;
	}
	HIPCHK(hipMemcpyAsync(c->d_txbuf, seg_buf, seg_buf_len, hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemsetAsync(c->d_txbuf + seg_buf_len, 0, IXG_TAIL_PAD, c->stream));
	HIPCHK(hipMemcpyAsync(c->d_txsegs, segs, (size_t)n * sizeof(*segs), hipMemcpyHostToDevice, c->stream));
	HIPCHK(hipMemcpyAsync(c->d_txout, out, out_size, hipMemcpyHostToDevice, c->stream));
	int rc = tx_launch(c, c->d_txbuf, c->d_txsegs, n, c->d_txout, c->d_txlen, flags, c->stream);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(out, c->d_txout, out_size, hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipMemcpyAsync(out_len, c->d_txlen, (size_t)n * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
	HIPCHK(hipStreamSynchronize(c->stream));
	return 0;
}

/* ---- event records --------------------------------------- */

int ixg_ev_batch_dev(void *vctx, const struct ixg_rx_frames *fr, const struct ixg_rx_rec *d_rec,
		     const struct ixg_demux_rec *d_dmx, const struct ixg_ev_pcb *d_pcbs, uint32_t n_pcbs,
		     uint32_t n, uint64_t iomap_base, uint32_t flags, struct ixg_bsys_desc *d_ev,
		     uint32_t *d_frame_idx, uint32_t *d_count, void *stream)
{
	struct ixg_ctx *c = (struct ixg_ctx *)vctx;
	if (!c || !fr || !d_count || (flags & ~IXG_EV_UDP_TUPLE))
		return -EINVAL;
	if (n && (!fr->base || !d_rec || !d_ev || (d_dmx && n_pcbs && !d_pcbs) || (!fr->off && (fr->stride & 3))))
		return -EINVAL;
	HIPCHK(hipSetDevice(c->device));
	if (n == 0)
		return hipMemsetAsync(d_count, 0, sizeof(uint32_t), (hipStream_t)stream) == hipSuccess ? 0 : -EIO;
	/* scratch: chunk counts/bases, then group counts/bases (64 chunks a group) */
	size_t nchunks = ((size_t)n + 63) / 64, ngroups = (nchunks + 63) / 64;
	size_t need = ngroups * 64 + ngroups;
	if (need > c->evbase_cap) {
		hipFree(c->d_evbase);
		c->d_evbase = NULL;
		c->evbase_cap = 0;
		HIPCHK(hipMalloc((void **)&c->d_evbase, need * sizeof(uint32_t)));
		c->evbase_cap = need;
	}
	struct ixg_eparams p;
	memset(&p, 0, sizeof(p));
	p.base = (uint8_t *)fr->base;
	p.off = fr->off;
	p.rec = d_rec;
	p.dmx = d_dmx;
	p.pcbs = d_pcbs;
	p.ev = d_ev;
	p.frame_idx = d_frame_idx;
	p.count = d_count;
	p.chunk_base = c->d_evbase;
	p.group_base = c->d_evbase + ngroups * 64;
	p.iomap_base = iomap_base;
	p.stride = fr->stride;
	p.n = n;
	p.n_pcbs = d_dmx ? n_pcbs : 0;
	p.flags = flags;
	return ixgrx_ev_launch(&p, c->ncu, stream) == 0 ? 0 : -EIO;
}
