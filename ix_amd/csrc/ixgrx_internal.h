/* ixgrx_internal.h - private structures shared by the C host library and
 * the HIP kernels (not part of the public ABI). */
#ifndef IXGRX_INTERNAL_H
#define IXGRX_INTERNAL_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_kparams {
	const uint8_t *base;
	const uint64_t *off;
	const uint16_t *len;
	struct ixg_rx_rec *out;
	uint32_t *csum;
	const uint64_t *tab;   /* 12 x 256: lo = Toeplitz, hi = CRC-32C contribution */
	const uint32_t *tab6;  /* 36 x 256 Toeplitz contributions (IXG_F_IPV6), or NULL */
	uint32_t stride;
	uint32_t n;
	uint32_t crc_const;
	uint32_t flags;
	uint32_t fg_base;      /* dev_idx * 512 */
	uint32_t fg_mask;      /* nb_rx_fgs - 1 */
	uint8_t *defer;        /* per 64-packet chunk: 1 = left for the general
	                          kernel; NULL = general kernel does everything */
	const uint8_t *zero;   /* IXG_ZERO_PAGE zero bytes: stand-in source for
	                          loads that must read nothing */
};
typedef struct ixg_kparams ixg_kparams;

#define IXG_ZERO_PAGE 4096u

/* implemented in ixgrx_kernels.hip */
/* enqueue one batch: the fixed-shape kernel (when p->defer) and the general
 * kernel; grids are sized from the device's CU count and each kernel's
 * occupancy */
int ixgrx_launch(const void *params, int variant, uint32_t ncu, void *stream);
uint32_t ixgrx_kparams_size(void);
uint32_t ixgrx_block(void);

#ifdef __cplusplus
}
#endif
#endif
