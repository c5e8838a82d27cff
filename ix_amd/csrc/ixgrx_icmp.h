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
	const struct ixg_rx_rec *rec;
	uint32_t stride;
	uint32_t n;
	uint8_t mac[8];                /* CFG.mac (6 bytes) */
	uint8_t host[4];               /* hton32(CFG.host_addr): the bytes written */
	uint32_t rsvd;
};
typedef struct ixg_iparams ixg_iparams;

/* implemented in ixgrx_icmp.hip */
int ixgrx_icmp_launch(const void *params, void *stream);

#ifdef __cplusplus
}
#endif
#endif
