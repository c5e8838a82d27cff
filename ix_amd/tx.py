"""TX header build + checksums: the host-side mirror of the TX entry points
(include/ixgrx.h "TX").

IX's two TX paths build the Ethernet/IPv4 (+UDP) headers in front of a
segment on the host and leave the checksums to the NIC (TCP:
tcp_output_packet, dp/net/tcp_api.c:773-826) or compute the IP one in
software (UDP: udp_output, dp/net/udp.c:102-130). ``batch_dev`` /
``batch_host`` do that for a whole batch of segments on the GPU:
``struct ixg_tx_seg`` per segment in, one frame per segment out.

``make_segments`` builds synthetic batches (TCP segments as lwIP hands them
to tcp_output_packet: a TCP header with options + payload; UDP payloads as
udp_output receives them).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import ixgrx

SEG_DTYPE = np.dtype([("seg_off", "<u8"), ("out_off", "<u8"), ("src_ip", "<u4"), ("dst_ip", "<u4"),
                      ("seg_len", "<u2"), ("src_port", "<u2"), ("dst_port", "<u2"), ("proto", "u1"),
                      ("tos", "u1"), ("ttl", "u1"), ("rsvd", "u1"), ("dmac_idx", "<u2"), ("rsvd2", "<u4")])
assert SEG_DTYPE.itemsize == 40
IXG_TX_OFFLOAD = 1 << 0
EXPORTS = ("ixg_tx_set_macs", "ixg_tx_batch_dev", "ixg_tx_batch_host")


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    if getattr(lib, "_ixg_tx_bound", False):
        return lib
    vp, u32, i32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
    lib.ixg_tx_set_macs.argtypes = [vp, vp, vp, u32]
    lib.ixg_tx_set_macs.restype = i32
    lib.ixg_tx_batch_dev.argtypes = [vp, vp, vp, u32, vp, vp, u32, vp]
    lib.ixg_tx_batch_dev.restype = i32
    lib.ixg_tx_batch_host.argtypes = [vp, vp, sz, vp, u32, vp, sz, vp, u32]
    lib.ixg_tx_batch_host.restype = i32
    lib._ixg_tx_bound = True
    return lib


def set_macs(eng: ixgrx.RxEngine, src_mac: bytes, dmacs: np.ndarray) -> None:
    """CFG.mac and the next-hop MAC table (rows of 6 bytes)."""
    lib = _bind(eng._lib)
    src = np.frombuffer(bytes(src_mac), dtype=np.uint8).copy()
    d = np.ascontiguousarray(dmacs, dtype=np.uint8).reshape(-1, 6)
    eng._tx_keep = (src, d)
    ixgrx._check(lib.ixg_tx_set_macs(eng._ctx, src.ctypes.data, d.ctypes.data, d.shape[0]), "ixg_tx_set_macs", lib)


def batch_dev(eng: ixgrx.RxEngine, seg_buf: int, segs: int, n: int, out: int, out_len: int, flags: int = 0,
              stream: int | None = None) -> None:
    """Device-resident TX batch: all pointers are device pointers (ints)."""
    lib = _bind(eng._lib)
    ixgrx._check(lib.ixg_tx_batch_dev(eng._ctx, seg_buf, segs, n, out, out_len, flags, stream or None),
                 "ixg_tx_batch_dev", lib)


def batch_host(eng: ixgrx.RxEngine, seg_buf: np.ndarray, segs: np.ndarray, out_size: int, flags: int = 0):
    """Host TX batch: returns (output buffer, frame lengths)."""
    lib = _bind(eng._lib)
    buf = np.ascontiguousarray(seg_buf, dtype=np.uint8)
    sg = np.ascontiguousarray(segs, dtype=SEG_DTYPE)
    n = int(sg.shape[0])
    out = np.zeros(out_size, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint16)
    ixgrx._check(lib.ixg_tx_batch_host(eng._ctx, buf.ctypes.data, buf.size, sg.ctypes.data, n, out.ctypes.data,
                                       out.size, out_len.ctypes.data, flags), "ixg_tx_batch_host", lib)
    return out, out_len


def frame_span(seg_len: np.ndarray, proto: np.ndarray) -> np.ndarray:
    """Bytes a frame occupies in the output: 34 + seg_len (+ 8 for UDP),
    rounded up to 16 (the kernel may write up to the next 16-byte boundary)."""
    L = 34 + seg_len.astype(np.int64) + np.where(proto == 17, 8, 0)
    return (L + 15) // 16 * 16


@dataclass
class TxBatch:
    """A synthetic TX batch: segment bytes + descriptors + MACs."""
    buf: np.ndarray       # uint8 segment bytes
    segs: np.ndarray      # SEG_DTYPE
    src_mac: bytes
    dmacs: np.ndarray     # [n_dmac, 6] uint8
    out_size: int         # output bytes needed

    @property
    def n(self) -> int:
        return int(self.segs.shape[0])


def _tcp_header(rng, n: int, doff: np.ndarray) -> np.ndarray:
    """[n, 60] TCP headers (only the first 4*doff bytes of a row are used):
    random ports/seq/ack/window, flags ACK|PSH, NOP options."""
    h = np.zeros((n, 60), dtype=np.uint8)
    h[:, 0:12] = rng.integers(0, 256, size=(n, 12), dtype=np.uint8)
    h[:, 12] = (doff << 4).astype(np.uint8)
    h[:, 13] = 0x18
    h[:, 14:16] = rng.integers(0, 256, size=(n, 2), dtype=np.uint8)
    h[:, 16:18] = rng.integers(0, 256, size=(n, 2), dtype=np.uint8)  # any value: the build rewrites it
    h[:, 18:20] = 0
    h[:, 20:60] = 1  # NOP
    return h


def make_segments(kind: str, n: int, seed: int, pool: int | None = None, layout: str = "slot") -> TxBatch:
    """Synthetic TX segments.

    kind: "tcp64"   echoserver replies: 20-B TCP header + 0..6 B payload (frames <= 60 B)
          "tcp1514" full-size TCP: 20-B header + 1460 B payload (1514-B frames)
          "mixed"   TCP doff 5..15 with 0..1460-doff*4 B payload, and UDP 0..1472 B payloads
    layout: "slot" = output frames in IX mbuf data slots (2112-B stride, data at
    +64), "packed" = 16-aligned back to back. pool: distinct segments generated
    (tiled to n)."""
    rng = np.random.default_rng(seed)
    m = n if pool is None else min(n, pool)
    if kind == "tcp64":
        proto = np.full(m, 6, np.uint8)
        doff = np.full(m, 5, np.int64)
        plen = rng.integers(0, 7, size=m)
    elif kind == "tcp1514":
        proto = np.full(m, 6, np.uint8)
        doff = np.full(m, 5, np.int64)
        plen = np.full(m, 1460, np.int64)
    elif kind == "mixed":
        proto = np.where(rng.random(m) < 0.5, 6, 17).astype(np.uint8)
        doff = rng.integers(5, 16, size=m)
        plen = np.where(proto == 6, rng.integers(0, 1461, size=m) - 4 * (doff - 5),
                        rng.integers(0, 1473, size=m))
        plen = np.maximum(plen, 0)
    else:
        raise ValueError(kind)
    seg_len = np.where(proto == 6, 4 * doff + plen, plen).astype(np.int64)
    seg_span = (seg_len + 3) // 4 * 4
    seg_off = np.zeros(m, dtype=np.int64)
    if m:
        seg_off[1:] = np.cumsum(seg_span)[:-1]
    total = int(seg_span.sum()) if m else 0
    buf = rng.integers(0, 256, size=total + 64, dtype=np.uint8)
    hdr = _tcp_header(rng, m, doff)
    for dv in np.unique(doff[proto == 6]):
        idx = np.nonzero((proto == 6) & (doff == dv))[0]
        hl = 4 * int(dv)
        gather = seg_off[idx][:, None] + np.arange(hl)[None, :]
        buf[gather] = hdr[idx, :hl]
    if m < n:
        reps = n // m
        assert n % m == 0
        # the tail repeats the pool's first bytes, so the bytes past each
        # repetition's last segment (read as padding) are the same in every
        # repetition
        buf = np.concatenate([np.tile(buf[:total], reps), buf[:64]])
        seg_off = (seg_off[None, :] + total * np.arange(reps)[:, None]).reshape(-1)
        proto, seg_len = np.tile(proto, reps), np.tile(seg_len, reps)
    segs = np.zeros(n, dtype=SEG_DTYPE)
    segs["seg_off"] = seg_off
    segs["seg_len"] = seg_len
    segs["proto"] = proto
    segs["src_ip"] = np.resize(rng.integers(0, 1 << 32, size=m, dtype=np.uint64), n).astype(np.uint32)
    segs["dst_ip"] = np.resize(rng.integers(0, 1 << 32, size=m, dtype=np.uint64), n).astype(np.uint32)
    segs["src_port"] = np.resize(rng.integers(1, 65536, size=m), n)
    segs["dst_port"] = np.resize(rng.integers(1, 65536, size=m), n)
    segs["tos"] = np.where(proto == 6, np.resize(rng.integers(0, 256, size=m), n), 0)
    segs["ttl"] = np.where(proto == 6, np.resize(rng.integers(1, 256, size=m), n), 64)
    ndm = 16
    segs["dmac_idx"] = np.resize(rng.integers(0, ndm, size=m), n)
    if layout == "slot":
        segs["out_off"] = np.arange(n, dtype=np.uint64) * np.uint64(2112) + np.uint64(64)
        out_size = n * 2112 + 64
    else:
        span = frame_span(segs["seg_len"], segs["proto"])
        oo = np.zeros(n, dtype=np.int64)
        if n:
            oo[1:] = np.cumsum(span)[:-1]
        segs["out_off"] = oo
        out_size = int(span.sum()) + 64
    dmacs = rng.integers(0, 256, size=(ndm, 6), dtype=np.uint8)
    src_mac = bytes(rng.integers(0, 256, size=6, dtype=np.uint8))
    return TxBatch(buf, segs, src_mac, dmacs, out_size)
