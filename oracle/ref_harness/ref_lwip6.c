/*
 * ref_lwip6.c - IPv6 pseudo-header checksum from the reference.
 *
 * TEST INFRASTRUCTURE ONLY. dp/lwip/inet_chksum.c built with LWIP_IPV6=1
 * (IX builds it with 0; inc/lwip/lwip/opt.h:2015-2016) for
 * ip6_chksum_pseudo_partial (inet_chksum.c:488-509), the oracle of the
 * IPv6 extension. ip6_chksum_pseudo itself does not link: its base is under
 * #if 0 (inet_chksum.c:283-321).
 */
#define LWIP_IPV6 1
#include "/root/reference/dp/lwip/inet_chksum.c"

#include "ref_capture.h"

uint16_t ref_pseudo6_partial(const void *seg, uint16_t len, uint8_t proto, uint16_t proto_len,
			     const void *src16, const void *dst16)
{
	struct pbuf p;
	ip6_addr_t s, d;
	memset(&p, 0, sizeof(p));
	p.payload = (void *)seg;
	p.len = p.tot_len = len;
	p.type = PBUF_ROM;
	memcpy(&s, src16, 16);
	memcpy(&d, dst16, 16);
	return ip6_chksum_pseudo_partial(&p, proto, proto_len, len, &s, &d);
}
