/*
 * ref_rss.c - the reference's software Toeplitz hash.
 *
 * TEST INFRASTRUCTURE ONLY. compute_toeplitz_hash is static in
 * dp/net/tcp_api.c:581-604, so the file is included unmodified and only the
 * wrapper's reachable code is kept by --gc-sections (no stubs needed).
 */
#include "/root/reference/dp/net/tcp_api.c"

#include "ref_capture.h"

uint32_t ref_toeplitz(const uint8_t *key, uint32_t src_raw, uint32_t dst_raw, uint16_t sport_raw,
		      uint16_t dport_raw)
{
	return compute_toeplitz_hash(key, src_raw, dst_raw, sport_raw, dport_raw);
}
