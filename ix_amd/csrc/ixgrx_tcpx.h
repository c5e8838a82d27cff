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
#endif
