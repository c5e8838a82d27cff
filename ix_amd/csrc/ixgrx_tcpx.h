/* ixgrx_tcpx.h - private structures shared by the C host library and the
 * tcp_input-head kernel (not part of the public ABI). */
#ifndef IXGRX_TCPX_H
#define IXGRX_TCPX_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_xparams {
	uint8_t *base;                 /* frames (written with IXG_TCPX_INPLACE) */
	const uint64_t *off;           /* or NULL: base + i*stride */
	const struct ixg_rx_rec *rec;
	struct ixg_tcp_ext *ext;
	uint32_t stride;
	uint32_t n;
	uint32_t flags;                /* IXG_TCPX_* */
	uint32_t rsvd;
};
typedef struct ixg_xparams ixg_xparams;

/* implemented in ixgrx_tcpx.hip */
int ixgrx_tcpx_launch(const void *params, void *stream);

#ifdef __cplusplus
}
#endif

#ifdef __HIPCC__
/* The ixg_tcp_ext of one TCP segment, shared by the separate pass
 * (ixgrx_tcpx.hip) and the RX kernels that write it from the header bytes
 * they already hold (ixg_rx_tcpx_batch_dev): D0..D4 are the five dwords
 * from 2 bytes before the TCP header (header bytes -2..17; frame starts are
 * 4-aligned and the header sits at 14 + 4*ihl or 54), w1 / w3 the record's
 * second and fourth words (l4_len, TCP flags). */
struct ixgx_ext {
	uint32_t x, y, z, w;
};
__device__ __forceinline__ uint32_t ixgx_bswap16(uint32_t v) { return ((v & 0xffu) << 8) | ((v >> 8) & 0xffu); }
__device__ __forceinline__ ixgx_ext ixgx_make(uint32_t D0, uint32_t D1, uint32_t D2, uint32_t D3, uint32_t D4,
					       uint32_t w1, uint32_t w3)
{
	const uint32_t src = ixgx_bswap16(D0 >> 16);                        /* tcp_in.c:230 */
	const uint32_t dst = ixgx_bswap16(D1 & 0xffffu);                    /* :231 */
	const uint32_t seq = __builtin_bswap32((D1 >> 16) | (D2 << 16));    /* :236 */
	const uint32_t ack = __builtin_bswap32((D2 >> 16) | (D3 << 16));    /* :237 */
	const uint32_t wnd = ixgx_bswap16(D4 & 0xffffu);                    /* :238 */
	/* :240-241: p->tot_len after the doff strip (the record's l4_len), +1
	 * for FIN or SYN (TCP_FIN | TCP_SYN = 0x03), kept as u16 */
	const uint32_t tcplen = ((w1 >> 16) + (((w3 >> 16) & 3u) ? 1u : 0u)) & 0xffffu;
	return ixgx_ext{seq, ack, wnd | (tcplen << 16), src | (dst << 16)};
}
/* IXG_TCPX_INPLACE: tcp_in.c:230-238 writes the same fields back in host
 * order; t = the dword 2 bytes before the TCP header */
__device__ __forceinline__ void ixgx_inplace(uint32_t *t, uint32_t D0, uint32_t D3, uint32_t D4, const ixgx_ext &e)
{
	const uint32_t src = e.w & 0xffffu, dst = e.w >> 16, seq = e.x, ack = e.y, wnd = e.z & 0xffffu;
	t[0] = (D0 & 0xffffu) | (src << 16);
	t[1] = dst | (seq << 16);
	t[2] = (seq >> 16) | (ack << 16);
	t[3] = (ack >> 16) | (D3 & 0xffff0000u);
	t[4] = wnd | (D4 & 0xffff0000u);
}
#endif
#ifdef __cplusplus
extern "C" {
#endif

#ifdef __cplusplus
}
#endif
#endif
