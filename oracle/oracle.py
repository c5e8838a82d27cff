"""ctypes binding of oracle/liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline. The product
(ix_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")

HASH_BITSERIAL, HASH_TABLE = 0, 1
WORK_FULL, WORK_IX = 0, 1

_lib = None


class _Cfg(ctypes.Structure):
    _fields_ = [("rss_key", ctypes.c_uint8 * 40), ("nb_rx_fgs", ctypes.c_uint16),
                ("dev_idx", ctypes.c_uint16), ("flags", ctypes.c_uint32)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, u32, i32, u16, u8 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint16, ctypes.c_uint8
        L.ixgo_rx_batch.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, u32, u32, vp, vp, i32, i32, i32]
        L.ixgo_rx_batch.restype = i32
        L.ixgo_rx_batch_mbufs.argtypes = [ctypes.POINTER(_Cfg), vp, u32, vp, i32, i32, i32]
        L.ixgo_rx_batch_mbufs.restype = i32
        L.ixgo_chksum_internet.argtypes = [vp, i32]
        L.ixgo_chksum_internet.restype = u16
        L.ixgo_toeplitz.argtypes = [vp, vp, i32]
        L.ixgo_toeplitz.restype = u32
        L.ixgo_crc32c_u64.argtypes = [u32, ctypes.c_uint64]
        L.ixgo_crc32c_u64.restype = u32
        L.ixgo_tcp_to_idx.argtypes = [u32, u32, u16, u16]
        L.ixgo_tcp_to_idx.restype = u16
        L.ixgo_pseudo_partial.argtypes = [vp, u16, u8, u16, u32, u32]
        L.ixgo_pseudo_partial.restype = u16
        _lib = L
    return _lib


def _cfg(key: bytes, nb: int, dev: int, flags: int) -> _Cfg:
    c = _Cfg()
    ctypes.memmove(c.rss_key, bytes(key), 40)
    c.nb_rx_fgs, c.dev_idx, c.flags = nb, dev, flags
    return c


def rx_batch(key: bytes, nb: int, dev: int, flags: int, blob: np.ndarray, off, lens: np.ndarray,
             stride: int = 0, threads: int = 1, hash_mode: int = HASH_BITSERIAL, work: int = WORK_FULL):
    """Records ([n,16] uint8) and residual words for a batch."""
    n = int(lens.shape[0])
    rec = np.zeros((n, 16), dtype=np.uint8)
    cs = np.zeros(n, dtype=np.uint32)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    c = _cfg(key, nb, dev, flags)
    lib().ixgo_rx_batch(ctypes.byref(c), blob.ctypes.data, None if offa is None else offa.ctypes.data,
                        lens.ctypes.data, stride, n, rec.ctypes.data, cs.ctypes.data, threads, hash_mode, work)
    return rec, cs


def rx_trace(tr, key: bytes, nb: int = 128, dev: int = 0, flags: int = 0, **kw):
    return rx_batch(key, nb, dev, flags, tr.blob, tr.off, tr.len, tr.stride, **kw)


def rx_mbufs(key: bytes, nb: int, dev: int, flags: int, ptrs: np.ndarray, threads: int = 1,
             hash_mode: int = HASH_BITSERIAL, work: int = WORK_FULL) -> np.ndarray:
    n = int(ptrs.shape[0])
    rec = np.zeros((n, 16), dtype=np.uint8)
    p = np.ascontiguousarray(ptrs, dtype=np.uint64)
    c = _cfg(key, nb, dev, flags)
    lib().ixgo_rx_batch_mbufs(ctypes.byref(c), p.ctypes.data, n, rec.ctypes.data, threads, hash_mode, work)
    return rec
