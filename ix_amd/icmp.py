"""ixg_icmp_reflect_dev (include/ixgrx.h "ICMP echo reflect";
dp/net/icmp.c:44-71,88-91).

icmp_input answers an echo request in the request's own mbuf: type 0, the
Ethernet and IP destinations set to the old sources, CFG.mac and
CFG.host_addr as the new sources, the ICMP checksum recomputed, and hands it
to eth_send_one. ``reflect_dev`` does that rewrite on the device for every
IXG_V_ICMP_ECHO record of a batch, so IX's TX path only has to send the
frames the records name.
"""
from __future__ import annotations

import ctypes

from ix_amd import ixgrx

EXPORTS = ("ixg_icmp_reflect_dev", "ixg_rx_icmp_batch_dev")


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    if getattr(lib, "_ixg_icmp_bound", False):
        return lib
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.ixg_icmp_reflect_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), vp, u32, vp, u32, vp]
    lib.ixg_icmp_reflect_dev.restype = i32
    lib.ixg_rx_icmp_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), u32, vp, vp, u32, vp]
    lib.ixg_rx_icmp_batch_dev.restype = i32
    lib._ixg_icmp_bound = True
    return lib


def reflect_dev(eng: ixgrx.RxEngine, base: int, off: int | None, stride: int, rec: int, n: int, mac: bytes,
                host_addr: int, stream: int | None = None) -> None:
    """Device-resident: base/off/rec are device pointers (int); mac is
    CFG.mac (6 bytes), host_addr CFG.host_addr in host order. Asynchronous
    on `stream`."""
    lib = _bind(eng._lib)
    if len(mac) != 6:
        raise ValueError("mac: 6 bytes")
    fr = ixgrx.RxFrames(base, off or None, 0, stride, 0)
    m = (ctypes.c_uint8 * 6).from_buffer_copy(bytes(mac))
    ixgrx._check(lib.ixg_icmp_reflect_dev(eng._ctx, ctypes.byref(fr), rec, n, m, host_addr, stream or None),
                 "ixg_icmp_reflect_dev", lib)


def rx_batch_dev(eng: ixgrx.RxEngine, base: int, off: int | None, lens: int, stride: int, n: int, rec: int,
                 mac: bytes, host_addr: int, stream: int | None = None) -> None:
    """ixg_rx_icmp_batch_dev: the records (rec, n x 16 B) and the echo
    replies in place in one launch. Device pointers as ints; asynchronous on
    `stream`."""
    lib = _bind(eng._lib)
    if len(mac) != 6:
        raise ValueError("mac: 6 bytes")
    fr = ixgrx.RxFrames(base, off or None, lens, stride, 0)
    m = (ctypes.c_uint8 * 6).from_buffer_copy(bytes(mac))
    ixgrx._check(lib.ixg_rx_icmp_batch_dev(eng._ctx, ctypes.byref(fr), n, rec, m, host_addr, stream or None),
                 "ixg_rx_icmp_batch_dev", lib)
