/* ixgrx_tx.h - private structures shared by the C host library and the TX
 * header-build kernel (not part of the public ABI). */
#ifndef IXGRX_TX_H
#define IXGRX_TX_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_tparams {
	const uint8_t *seg_buf;
	const struct ixg_tx_seg *segs;
	uint8_t *out;
	uint16_t *out_len;
	const uint32_t *dmacs;  /* n_dmac rows of 2 dwords: the 6 MAC bytes + 2 zero */
	uint32_t n;
	uint32_t n_dmac;
	uint32_t smac_lo;       /* CFG.mac bytes 0..3 (LE) */
	uint32_t smac_hi;       /* bytes 4..5 */
	uint32_t flags;         /* IXG_TX_* */
	uint32_t rsvd;
	const uint8_t *zero;    /* IXG_ZERO_PAGE zero bytes (dummy load source) */
};
typedef struct ixg_tparams ixg_tparams;

/* implemented in ixgrx_tx.hip */
int ixgrx_tx_launch(const void *params, uint32_t ncu, void *stream);

#ifdef __cplusplus
}
#endif
#endif
