/* ixgrx_demux.h - private structures shared by the C host library and the
 * PCB demux kernel (not part of the public ABI). */
#ifndef IXGRX_DEMUX_H
#define IXGRX_DEMUX_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_dparams {
	const uint8_t *base;
	const uint64_t *off;
	const struct ixg_rx_rec *rec;
	struct ixg_demux_rec *out;
	const uint32_t *active_start; /* nfg*512 + 1 */
	const uint32_t *bline;        /* nfg*512 bucket lines (ixgrx_walk.h) */
	const struct ixg_pcb_key *active;
	const struct ixg_pcb_key *tw;
	const struct ixg_listen_key *listen;
	uint32_t stride;
	uint32_t n;
	uint32_t fg_base;             /* dev_idx * 512 */
	uint32_t nfg;
	uint32_t n_out;               /* outbound groups after the nfg local ones */
	uint32_t n_listen;
	uint32_t rsvd;
};
typedef struct ixg_dparams ixg_dparams;

/* implemented in ixgrx_demux.hip */
int ixgrx_demux_launch(const void *params, uint32_t ncu, void *stream);

#ifdef __cplusplus
}
#endif
#endif
