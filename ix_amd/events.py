"""Event records: the host-side mirror of ixg_ev_batch_dev (include/ixgrx.h
"event records").

IX's stack hands received data to libix as usys descriptors (struct
bsys_desc, inc/ix/syscall.h:101-104) written by udp_input (usys_udp_recv,
dp/net/udp.c:81-88) and recv_a_pbuf (usys_tcp_recv, dp/net/tcp_api.c:133-147).
``batch_dev`` produces those descriptors on the device from the RX and demux
records of a batch, dense and in frame order, so the event loop
(libix/main.c:56-64, ixev.c:132-166) can consume them as they are.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import ixgrx

EV_DTYPE = np.dtype([("sysnr", "<u8"), ("arga", "<u8"), ("argb", "<u8"), ("argc", "<u8"), ("argd", "<u8")])
PCB_DTYPE = np.dtype([("pcb_idx", "<u8"), ("cookie", "<u8")])
assert EV_DTYPE.itemsize == 40 and PCB_DTYPE.itemsize == 16
USYS_UDP_RECV, USYS_TCP_RECV = 0, 4
IXG_EV_UDP_TUPLE = 1 << 0
EXPORTS = ("ixg_ev_batch_dev",)


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    if getattr(lib, "_ixg_ev_bound", False):
        return lib
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.ixg_ev_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), vp, vp, vp, u32, u32, ctypes.c_uint64, u32,
                                     vp, vp, vp, vp]
    lib.ixg_ev_batch_dev.restype = i32
    lib._ixg_ev_bound = True
    return lib


def batch_dev(eng: ixgrx.RxEngine, base: int, off: int | None, stride: int, rec: int, dmx: int | None,
              pcbs: int | None, n_pcbs: int, n: int, iomap_base: int, flags: int, ev: int, frame_idx: int | None,
              count: int, stream: int | None = None) -> None:
    """Device-resident: every pointer is a device pointer (int); *count (u32)
    receives the number of descriptors written to ev."""
    lib = _bind(eng._lib)
    fr = ixgrx.RxFrames(base, off or None, 0, stride, 0)
    ixgrx._check(lib.ixg_ev_batch_dev(eng._ctx, ctypes.byref(fr), rec, dmx or None, pcbs or None, n_pcbs, n,
                                      iomap_base, flags, ev, frame_idx or None, count, stream or None),
                 "ixg_ev_batch_dev", lib)
