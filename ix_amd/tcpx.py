"""The rest of the tcp_input head: the host-side mirror of
ixg_tcp_ext_batch_dev (include/ixgrx.h "the rest of the tcp_input head";
SURVEY.md 8(a) a8, dp/net/tcp_in.c:230-241).

After the doff strip, tcp_input converts the TCP header's ports, seqno,
ackno and wnd to host order in place and keeps them, with tcplen, in its
LWIP_Context; tcp_process and tcp_receive read them from there and from the
header. ``batch_dev`` produces those values for a batch on the device (one
16-byte struct ixg_tcp_ext per frame) and, with IXG_TCPX_INPLACE, the
in-place conversion, so the host callee need not parse the header again.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import ixgrx

TCPX_DTYPE = np.dtype([("seqno", "<u4"), ("ackno", "<u4"), ("wnd", "<u2"), ("tcplen", "<u2"),
                       ("src_port", "<u2"), ("dst_port", "<u2")])
assert TCPX_DTYPE.itemsize == 16
IXG_TCPX_INPLACE = 1 << 0
EXPORTS = ("ixg_tcp_ext_batch_dev", "ixg_rx_tcpx_batch_dev")


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    if getattr(lib, "_ixg_tcpx_bound", False):
        return lib
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.ixg_tcp_ext_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), vp, u32, vp, u32, vp]
    lib.ixg_tcp_ext_batch_dev.restype = i32
    lib.ixg_rx_tcpx_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), u32, vp, vp, u32, vp]
    lib.ixg_rx_tcpx_batch_dev.restype = i32
    lib._ixg_tcpx_bound = True
    return lib


def batch_dev(eng: ixgrx.RxEngine, base: int, off: int | None, stride: int, rec: int, n: int, ext: int,
              flags: int = 0, stream: int | None = None) -> None:
    """Device-resident: every pointer is a device pointer (int). Asynchronous
    on `stream`."""
    lib = _bind(eng._lib)
    fr = ixgrx.RxFrames(base, off or None, 0, stride, 0)
    ixgrx._check(lib.ixg_tcp_ext_batch_dev(eng._ctx, ctypes.byref(fr), rec, n, ext, flags, stream or None),
                 "ixg_tcp_ext_batch_dev", lib)


def rx_batch_dev(eng: ixgrx.RxEngine, base: int, off: int | None, lens: int, stride: int, n: int, rec: int,
                 ext: int, flags: int = 0, stream: int | None = None) -> None:
    """ixg_rx_tcpx_batch_dev: RX records and the tcp_input head in one pass
    (fused into the coalesced fixed-shape kernel for 64-byte strides; other
    layouts run RX, then the separate pass). Device pointers (int);
    asynchronous on `stream`."""
    lib = _bind(eng._lib)
    fr = ixgrx.RxFrames(base, off or None, lens, stride, 0)
    ixgrx._check(lib.ixg_rx_tcpx_batch_dev(eng._ctx, ctypes.byref(fr), n, rec, ext, flags, stream or None),
                 "ixg_rx_tcpx_batch_dev", lib)
