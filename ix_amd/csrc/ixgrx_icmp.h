/* ixgrx_icmp.h - private structures shared by the C host library and the
 * ICMP echo-reflect kernel (not part of the public ABI). */
#ifndef IXGRX_ICMP_H
#define IXGRX_ICMP_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_iparams {
	uint8_t *base;                 /* frames, rewritten in place */
	const uint64_t *off;           /* or NULL: base + i*stride */
	struct ixg_rx_rec *rec;        /* read; with `mark`, IXG_RF_REPLY set */
	const uint32_t *idx;           /* or NULL: item j is frame j; else the
	                                  asynchronous path's candidate list: item
	                                  j is record idx[j], its frame at
	                                  base + off[j] (base NULL: off[j] is the
	                                  frame's device address in its mbuf) */
	uint32_t stride;
	uint32_t n;                    /* items */
	uint8_t mac[8];                /* CFG.mac (6 bytes) */
	uint8_t host[4];               /* hton32(CFG.host_addr): the bytes written */
	uint32_t mark;                 /* 1: set IXG_RF_REPLY in each reflected record */
};
typedef struct ixg_iparams ixg_iparams;

/* implemented in ixgrx_icmp.hip */
int ixgrx_icmp_launch(const void *params, void *stream);

#ifdef __cplusplus
}
#endif
#endif
