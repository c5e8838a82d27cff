"""Synthetic Ethernet/IPv4/TCP/UDP packet traces (BASELINE.json configs).

Frames are built with numpy, vectorised per shape class, with valid IP and
L4 checksums unless a corruption fraction is requested. A trace is a
``Trace``: one byte blob plus per-frame offsets and lengths, the layout the
device API (``struct ixg_rx_frames``) takes. Frame starts are 4-byte aligned.

Shapes follow SURVEY.md section 8(d):
  tcp64     C1/C2: L=60 ("64 B" on the wire), ip_len 40, doff 5, no payload
  imix      C3: L in {60, 590, 1514} by 7:4:1, TCP:UDP 50:50
  tcp1514   C4: L=1514, ip_len 1500, doff 5, 1460 B payload
  mixed     C5: IPv4 ihl uniform 5..15 (NOP options) + 50% IPv6 TCP/UDP
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

# Microsoft RSS verification key == DPDK's default rss_key
RSS_KEY = bytes([
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa,
])


@dataclass
class Trace:
    blob: np.ndarray        # uint8, frames + tail padding
    off: np.ndarray | None  # uint64 byte offsets, or None for fixed stride
    len: np.ndarray         # uint16 frame lengths
    stride: int = 0         # when off is None

    @property
    def n(self) -> int:
        return int(self.len.shape[0])

    def frame(self, i: int) -> bytes:
        o = int(self.off[i]) if self.off is not None else i * self.stride
        return bytes(self.blob[o:o + int(self.len[i])])

    def offsets(self) -> np.ndarray:
        if self.off is not None:
            return self.off
        return np.arange(self.n, dtype=np.uint64) * np.uint64(self.stride)

    def wire_bytes(self) -> int:
        return int(self.len.astype(np.int64).sum())


TAIL_PAD = 64  # include/ixgrx.h IXG_TAIL_PAD


def _fold(s: np.ndarray) -> np.ndarray:
    s = s.astype(np.uint64)
    for _ in range(4):
        s = (s & 0xFFFF) + (s >> 16)
    return s


def _sum_be16(a: np.ndarray) -> np.ndarray:
    """One's complement partial sums of big-endian 16-bit words, row-wise.
    a: [n, even] uint8."""
    w = a[:, 0::2].astype(np.uint64) * 256 + a[:, 1::2].astype(np.uint64)
    return w.sum(axis=1)


def _put16(buf: np.ndarray, col: int, v: np.ndarray) -> None:
    v = v.astype(np.uint32)
    buf[:, col] = (v >> 8) & 0xFF
    buf[:, col + 1] = v & 0xFF


def _put32(buf: np.ndarray, col: int, v: np.ndarray) -> None:
    v = v.astype(np.uint64)
    for k in range(4):
        buf[:, col + k] = (v >> (24 - 8 * k)) & 0xFF


def build_ipv4(rng: np.random.Generator, n: int, L: int, proto: int, ihl: int = 5,
               payload_random: bool = True) -> np.ndarray:
    """n frames of length L: Ethernet + IPv4(ihl, NOP options) + TCP(doff 5)
    or UDP, valid checksums. Returns [n, L] uint8."""
    l4 = 14 + 4 * ihl
    hl = 20 if proto == 6 else 8
    ip_len = L - 14
    if ip_len < 4 * ihl + hl:
        raise ValueError("frame too short for headers")
    # Ethernet minimum: 60 B incl. padding; ip_len covers only the real bytes
    if proto == 6 and L == 60 and ihl == 5:
        ip_len = 40
    f = np.zeros((n, L), dtype=np.uint8)
    if payload_random:
        f[:, l4 + hl:14 + ip_len] = rng.integers(0, 256, size=(n, 14 + ip_len - l4 - hl), dtype=np.uint8)
    f[:, 0:6] = np.array([0x02, 0, 0, 0, 0, 0x01], np.uint8)
    f[:, 6:12] = rng.integers(0, 256, size=(n, 6), dtype=np.uint8)
    f[:, 12] = 0x08
    f[:, 13] = 0x00
    f[:, 14] = 0x40 | ihl
    _put16(f, 16, np.full(n, ip_len))
    _put16(f, 18, rng.integers(0, 65536, n))
    f[:, 20] = 0x40  # DF
    f[:, 22] = 64
    f[:, 23] = proto
    f[:, 26:34] = rng.integers(0, 256, size=(n, 8), dtype=np.uint8)
    if ihl > 5:
        f[:, 34:l4] = 0x01  # NOP options
    # ports 1..65535 so both tcp_to_idx sign branches occur
    _put16(f, l4, rng.integers(1, 65536, n))
    _put16(f, l4 + 2, rng.integers(1, 65536, n))
    l4len = ip_len - 4 * ihl
    if proto == 6:
        _put32(f, l4 + 4, rng.integers(0, 1 << 32, n, dtype=np.uint64))
        _put32(f, l4 + 8, rng.integers(0, 1 << 32, n, dtype=np.uint64))
        f[:, l4 + 12] = 0x50
        f[:, l4 + 13] = 0x10  # ACK
        _put16(f, l4 + 14, rng.integers(1, 65536, n))
        ck = l4 + 16
    else:
        _put16(f, l4 + 4, np.full(n, l4len))
        ck = l4 + 6
    # IP header checksum
    s = _sum_be16(f[:, 14:l4])
    _put16(f, 24, (~_fold(s)) & 0xFFFF)
    # L4 checksum: pseudo header + segment (pad odd length)
    seg = f[:, l4:14 + ip_len]
    if seg.shape[1] % 2:
        seg = np.concatenate([seg, np.zeros((n, 1), np.uint8)], axis=1)
    s = _sum_be16(seg) + _sum_be16(f[:, 26:34]) + proto + l4len
    c = (~_fold(s)) & 0xFFFF
    if proto == 17:
        c = np.where(c == 0, 0xFFFF, c)
    _put16(f, ck, c)
    return f


def icmp_echo(rng: np.random.Generator, payload: int, ihl: int = 5) -> bytes:
    """One ICMP echo request (type 8) with `payload` random bytes after the
    8-byte header, valid IP and ICMP checksums, padded to the 60-byte
    Ethernet minimum."""
    l4 = 14 + 4 * ihl
    ip_len = 4 * ihl + 8 + payload
    f = np.zeros((1, max(60, 14 + ip_len)), dtype=np.uint8)
    f[0, 0:6] = [0x02, 0, 0, 0, 0, 0x01]
    f[0, 6:12] = rng.integers(0, 256, 6, dtype=np.uint8)
    f[0, 12] = 0x08
    f[0, 14] = 0x40 | ihl
    _put16(f, 16, np.array([ip_len]))
    _put16(f, 18, rng.integers(0, 65536, 1))
    f[0, 22] = 64
    f[0, 23] = 1
    f[0, 26:34] = rng.integers(0, 256, 8, dtype=np.uint8)
    if ihl > 5:
        f[0, 34:l4] = 0x01
    f[0, l4] = 8
    f[0, l4 + 4:l4 + 8 + payload] = rng.integers(0, 256, 4 + payload, dtype=np.uint8)
    _put16(f, 24, (~_fold(_sum_be16(f[:, 14:l4]))) & 0xFFFF)
    seg = f[:, l4:14 + ip_len]
    if seg.shape[1] % 2:
        seg = np.concatenate([seg, np.zeros((1, 1), np.uint8)], axis=1)
    _put16(f, l4 + 2, (~_fold(_sum_be16(seg))) & 0xFFFF)
    return f[0].tobytes()


def build_ipv6(rng: np.random.Generator, n: int, L: int, proto: int) -> np.ndarray:
    """Ethernet + IPv6 (no extension headers) + TCP/UDP, valid checksums."""
    hl = 20 if proto == 6 else 8
    plen = L - 54
    if plen < hl:
        raise ValueError("frame too short")
    f = np.zeros((n, L), dtype=np.uint8)
    f[:, 54 + hl:] = rng.integers(0, 256, size=(n, L - 54 - hl), dtype=np.uint8)
    f[:, 0:6] = np.array([0x02, 0, 0, 0, 0, 0x01], np.uint8)
    f[:, 6:12] = rng.integers(0, 256, size=(n, 6), dtype=np.uint8)
    f[:, 12] = 0x86
    f[:, 13] = 0xDD
    f[:, 14] = 0x60
    _put16(f, 18, np.full(n, plen))
    f[:, 20] = proto
    f[:, 21] = 64
    f[:, 22:54] = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    _put16(f, 54, rng.integers(1, 65536, n))
    _put16(f, 56, rng.integers(1, 65536, n))
    if proto == 6:
        _put32(f, 58, rng.integers(0, 1 << 32, n, dtype=np.uint64))
        f[:, 66] = 0x50
        f[:, 67] = 0x18
        _put16(f, 68, rng.integers(1, 65536, n))
        ck = 70
    else:
        _put16(f, 58, np.full(n, plen))
        ck = 60
    seg = f[:, 54:]
    if seg.shape[1] % 2:
        seg = np.concatenate([seg, np.zeros((n, 1), np.uint8)], axis=1)
    s = _sum_be16(seg) + _sum_be16(f[:, 22:54]) + proto + plen
    c = (~_fold(s)) & 0xFFFF
    if proto == 17:
        c = np.where(c == 0, 0xFFFF, c)
    _put16(f, ck, c)
    return f


def corrupt(rng: np.random.Generator, f: np.ndarray, frac_ip: float, frac_l4: float,
            l4_ck_col: int | None = None) -> None:
    """Flip checksum bytes in a fraction of frames (in place)."""
    n = f.shape[0]
    if frac_ip > 0:
        m = rng.random(n) < frac_ip
        f[m, 24] ^= 0x5A
    if frac_l4 > 0 and l4_ck_col is not None:
        m = rng.random(n) < frac_l4
        f[m, l4_ck_col] ^= 0xA5


def pack(frames: list[np.ndarray] | list[bytes], stride: int | None = None,
         align: int = 4) -> Trace:
    """Pack frames (rows or bytes) into one blob. stride=None: tight packing
    with `align`-byte aligned starts and a u64 offset array."""
    lens = np.array([len(x) for x in frames], dtype=np.uint16)
    n = len(frames)
    if stride is not None:
        blob = np.zeros(n * stride + TAIL_PAD, dtype=np.uint8)
        for i, x in enumerate(frames):
            blob[i * stride:i * stride + len(x)] = np.frombuffer(bytes(x), np.uint8)
        return Trace(blob, None, lens, stride)
    sizes = (lens.astype(np.uint64) + (align - 1)) // align * align
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(sizes)[:-1]
    total = int(sizes.sum()) if n else 0
    blob = np.zeros(total + TAIL_PAD, dtype=np.uint8)
    for i, x in enumerate(frames):
        o = int(off[i])
        blob[o:o + len(x)] = np.frombuffer(bytes(x), np.uint8)
    return Trace(blob, off, lens, 0)


def pack_rows(rows: np.ndarray, stride: int) -> Trace:
    """Fixed-stride packing of equal-length frames [n, L] (vectorised)."""
    n, L = rows.shape
    assert stride >= L and stride % 4 == 0
    blob = np.zeros(n * stride + TAIL_PAD, dtype=np.uint8)
    blob[:n * stride].reshape(n, stride)[:, :L] = rows
    return Trace(blob, None, np.full(n, L, dtype=np.uint16), stride)


def pack_classes(classes: list[np.ndarray], order: np.ndarray, align: int = 4) -> Trace:
    """Tight packing of several equal-length classes, interleaved by `order`
    (order[i] = class of frame i; frames of a class are taken in turn)."""
    n = order.shape[0]
    Ls = np.array([c.shape[1] for c in classes], dtype=np.uint64)
    lens = Ls[order].astype(np.uint16)
    sizes = (Ls[order] + (align - 1)) // align * align
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(sizes)[:-1]
    total = int(sizes.sum()) if n else 0
    blob = np.zeros(total + TAIL_PAD, dtype=np.uint8)
    for k, rows in enumerate(classes):
        idx = np.nonzero(order == k)[0]
        if idx.size == 0:
            continue
        L = rows.shape[1]
        take = rows[np.arange(idx.size) % rows.shape[0]]
        gather = off[idx][:, None].astype(np.int64) + np.arange(L, dtype=np.int64)[None, :]
        blob[gather] = take
    return Trace(blob, off, lens, 0)


def make_trace(kind: str, n: int, seed: int, bad_ip: float = 0.0, bad_l4: float = 0.0,
               pool: int | None = None) -> Trace:
    """Synthetic trace of `kind` with n frames. pool: number of distinct frames
    generated (tiled to n) for huge traces; None = all distinct."""
    rng = np.random.default_rng(seed)
    m = n if pool is None else min(n, pool)
    if kind == "tcp64":
        rows = build_ipv4(rng, m, 60, 6)
        corrupt(rng, rows, bad_ip, bad_l4, 34 + 16)
        if m < n:
            rows = rows[np.arange(n) % m]
        return pack_rows(rows, 60)
    if kind == "tcp64opt":
        # C2's slots with one option word (ihl 6): every chunk leaves the
        # fixed-shape path (A/B of the deferred path, not a config)
        rows = build_ipv4(rng, m, 60, 6, ihl=6)
        if m < n:
            rows = rows[np.arange(n) % m]
        return pack_rows(rows, 60)
    if kind == "tcp1514":
        rows = build_ipv4(rng, m, 1514, 6)
        corrupt(rng, rows, bad_ip, bad_l4, 34 + 16)
        if m < n:
            rows = rows[np.arange(n) % m]
        return pack_rows(rows, 1516)
    if kind == "imix":
        classes = []
        per = max(1, m // 6)
        for L in (60, 590, 1514):
            for proto in (6, 17):
                rows = build_ipv4(rng, per, L, proto) if not (L == 60 and proto == 17) else \
                    build_ipv4(rng, per, 60, 17)
                corrupt(rng, rows, bad_ip, bad_l4, 34 + (16 if proto == 6 else 6))
                classes.append(rows)
        size_cls = rng.choice(3, size=n, p=[7 / 12, 4 / 12, 1 / 12])
        proto_cls = rng.integers(0, 2, size=n)
        return pack_classes(classes, (size_cls * 2 + proto_cls).astype(np.int64))
    if kind in ("mixed", "mixed_v4", "mixed_v6", "mixed_sorted"):
        # mixed_v4 / mixed_v6: only the IPv4 (ihl 5..15) or only the IPv6
        # classes; mixed_sorted: C5's mix with each 128-frame run of one
        # family (A/B of the divergent parse, not a config)
        classes = []
        per = max(1, m // 24)
        for ihl in range(5, 16):
            for proto in (6, 17):
                L = max(60, 14 + 4 * ihl + (20 if proto == 6 else 8) + 16)
                classes.append(build_ipv4(rng, per, L, proto, ihl=ihl))
        for proto in (6, 17):
            classes.append(build_ipv6(rng, per, 94, proto))
        nv4 = 22
        p6 = {"mixed": 0.5, "mixed_v4": 0.0, "mixed_v6": 1.0, "mixed_sorted": 0.5}[kind]
        is6 = rng.random(n) < p6
        if kind == "mixed_sorted":
            is6 = (np.arange(n) // 128) % 2 == 1
        cls = np.where(is6, nv4 + rng.integers(0, 2, n), rng.integers(0, nv4, n))
        return pack_classes(classes, cls.astype(np.int64))
    raise ValueError(kind)
