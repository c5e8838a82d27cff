/* ixgrx_ev.h - private structures shared by the C host library and the
 * event-emission kernels (not part of the public ABI). */
#ifndef IXGRX_EV_H
#define IXGRX_EV_H

#include <stdint.h>

#include "../../include/ixgrx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kernel arguments, passed by value */
struct ixg_eparams {
	uint8_t *base;                 /* frames (written only with IXG_EV_UDP_TUPLE) */
	const uint64_t *off;
	const struct ixg_rx_rec *rec;
	const struct ixg_demux_rec *dmx;
	const struct ixg_ev_pcb *pcbs;
	struct ixg_bsys_desc *ev;
	uint32_t *frame_idx;
	uint32_t *count;
	uint32_t *chunk_base;          /* scratch: per-64-frame chunk event count, then its base
	                                * within its group of 64 chunks */
	uint32_t *group_base;          /* scratch: per group of 64 chunks, its event count, then
	                                * its base */
	uint64_t iomap_base;
	uint32_t stride;
	uint32_t n;
	uint32_t n_pcbs;
	uint32_t flags;
};
typedef struct ixg_eparams ixg_eparams;

/* implemented in ixgrx_ev.hip: count, group, scan and emit kernels on `stream` */
int ixgrx_ev_launch(const void *params, uint32_t ncu, void *stream);

#ifdef __cplusplus
}
#endif
#endif
