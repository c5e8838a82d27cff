#!/usr/bin/env python3
"""Generate the golden RX vectors from the reference's own C code.

Runs oracle/_ref/ixref_rx (built by ``make -C oracle ref`` from the
unmodified sources under /root/reference: dp/net/ip.c, dp/net/icmp.c,
dp/lwip/inet_chksum.c, dp/lwip/pbuf.c, dp/net/tcp_api.c, and the inline
hashes/checksums of inc/) over synthetic and hand-built frames, and stores
inputs + expected records as small .npz fixtures next to this script.

Only this script and its outputs are committed; the reference never travels.
Re-run:  make -C oracle ref && python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from ix_amd import traces  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ixref_rx")
F_NO_CSUM_DROP = 1
F_IPV6 = 2


def fdir_filter(f: bytes, swap: bool = False) -> bytes:
    """struct ixg_fdir_filter matching frame f's 4-tuple (src ip, dst ip,
    sport, dport of an IPv4 frame with ihl from byte 14); swap: the reverse
    direction (does not match f)."""
    l4 = 14 + 4 * (f[14] & 15)
    src, dst = struct.unpack_from("<I", f, 26)[0], struct.unpack_from("<I", f, 30)[0]
    sp, dp = (f[l4] << 8) | f[l4 + 1], (f[l4 + 2] << 8) | f[l4 + 3]
    if swap:
        src, dst, sp, dp = dst, src, dp, sp
    return struct.pack("<IIHH", src, dst, sp, dp)


def run_ref(frames: list[bytes], key: bytes, nb: int, dev: int, flags: int, fdir: list[bytes] | None = None,
            cpu: int = 0, full: bool = False, host: tuple[bytes, int] | None = None):
    """(records, residuals) from the reference's eth_input; full: also the
    rest of the tcp_input head from its tcp_input (tcpx, tcpx_hdr); host =
    (mac, host_addr): also (reflected flags, frames after eth_input) with
    CFG.mac / CFG.host_addr set for icmp_reflect."""
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    offs = np.zeros(len(frames), dtype=np.uint32)
    if frames:
        offs[1:] = np.cumsum(lens.astype(np.uint32))[:-1]
    blob = b"".join(frames)
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(b"IXGRXIN1")
            f.write(struct.pack("<IIHH", len(frames), flags, nb, dev))
            f.write(key)
            f.write(lens.tobytes())
            f.write(offs.tobytes())
            f.write(struct.pack("<I", len(blob)))
            f.write(blob)
            if fdir:
                f.write(b"FDIR")
                f.write(struct.pack("<IHH", len(fdir), cpu, 0))
                f.write(b"".join(fdir))
            if host:
                f.write(b"HOST" + host[0] + b"\0\0" + struct.pack("<I", host[1]))
        subprocess.run([HARNESS, fi, fo], check=True)
        raw = open(fo, "rb").read()
    assert raw[:8] == b"IXGRXOUT"
    n = struct.unpack_from("<I", raw, 8)[0]
    assert n == len(frames)
    rec = np.frombuffer(raw, dtype=np.uint8, count=16 * n, offset=12).reshape(n, 16).copy()
    csum = np.frombuffer(raw, dtype=np.uint32, count=n, offset=12 + 16 * n).copy()
    confirm = np.frombuffer(raw, dtype=np.uint8, count=n, offset=12 + 20 * n)
    # every drop eth_input made has a reference-confirmed reason: with the
    # field the reason blames repaired, the reference eth_input delivers the
    # frame or drops it for a strictly later reason, repaired in turn until
    # it delivers (harness_main.c confirm_drop)
    verdict = rec[:, 2]
    eth_input_reasons = ((verdict >= 0x80) & (verdict <= 0x87)) | ((verdict >= 0x8b) & (verdict <= 0x8d))
    assert not (confirm == 2).any(), f"drop reasons not confirmed by the reference: {np.nonzero(confirm == 2)[0][:20]}"
    assert ((confirm == 1) == eth_input_reasons).all(), "a drop reason without a reference confirmation"
    # the rest of the tcp_input head from the reference's own tcp_input
    # (ref_tcphead.c): struct ixg_tcp_ext per frame and the segment's first 16
    # bytes as tcp_input converted them in place
    o = 12 + 21 * n
    assert raw[o:o + 4] == b"TCPX"
    tcpx = np.frombuffer(raw, dtype=np.uint8, count=16 * n, offset=o + 4).reshape(n, 16).copy()
    tcpx_hdr = np.frombuffer(raw, dtype=np.uint8, count=16 * n, offset=o + 4 + 16 * n).reshape(n, 16).copy()
    o += 4 + 32 * n
    assert raw[o:o + 4] == b"ICMP"
    refl = np.frombuffer(raw, dtype=np.uint8, count=n, offset=o + 4).copy()
    after = np.frombuffer(raw, dtype=np.uint8, count=int(lens.astype(np.int64).sum()), offset=o + 4 + n).copy()
    if host:
        return rec, csum, tcpx, tcpx_hdr, refl, after
    return (rec, csum, tcpx, tcpx_hdr) if full else (rec, csum)


# ---------------------------------------------------------------- frames


def _ip_csum(hdr: bytearray) -> None:
    hdr[10:12] = b"\0\0"
    s = sum(struct.unpack("!%dH" % (len(hdr) // 2), bytes(hdr)))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    hdr[10:12] = struct.pack("!H", (~s) & 0xFFFF)


def _l4_csum(src: bytes, dst: bytes, proto: int, seg: bytearray, ck: int) -> None:
    seg[ck:ck + 2] = b"\0\0"
    data = bytes(seg) + (b"\0" if len(seg) % 2 else b"")
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    s += sum(struct.unpack("!4H", src + dst)) + proto + len(seg)
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    c = (~s) & 0xFFFF
    if proto == 17 and c == 0:
        c = 0xFFFF
    seg[ck:ck + 2] = struct.pack("!H", c)


def ipv4(proto=6, ihl=5, payload=b"", L=None, sport=1234, dport=80, doff=5, flags_off=0x4000,
         ver=4, ip_len=None, udp_len=None, src=b"\x0a\x00\x00\x01", dst=b"\x0a\x00\x00\x02",
         tcp_flags=0x18, icmp_type=8, fix_ip=True, fix_l4=True, l4=None, ethertype=0x0800,
         doff_field=None):
    """Build one frame; every header field can be forced to a bad value."""
    opts = b"\x01" * (4 * ihl - 20) if ihl >= 5 else b""
    if l4 is None:
        if proto == 6:
            th = bytearray(struct.pack("!HHIIBBHHH", sport, dport, 0x01020304, 0x0a0b0c0d,
                                       (doff & 15) << 4, tcp_flags, 512, 0, 0))
            th += b"\x01" * max(0, 4 * doff - 20) if doff > 5 else b""
            if doff_field is not None:  # lie about the header length, keep the bytes
                th[12] = (doff_field & 15) << 4
            l4 = th + payload
            ck = 16
        elif proto == 17:
            n = 8 + len(payload)
            l4 = bytearray(struct.pack("!HHHH", sport, dport, n if udp_len is None else udp_len, 0)) + payload
            ck = 6
        elif proto == 1:
            l4 = bytearray(struct.pack("!BBHHH", icmp_type, 0, 0, 7, 1)) + payload
            ck = 2
        else:
            l4 = bytearray(payload)
            ck = None
    else:
        l4 = bytearray(l4)
        ck = None
    hl = max(ihl, 0) * 4 if ihl >= 5 else 20
    tot = hl + len(l4) if ip_len is None else ip_len
    ip = bytearray(struct.pack("!BBHHHBBH4s4s", (ver << 4) | (ihl & 15), 0, tot & 0xFFFF, 0x1234,
                               flags_off, 64, proto, 0, src, dst)) + opts
    if fix_l4 and ck is not None:
        if proto == 1:
            l4[2:4] = b"\0\0"
            d = bytes(l4) + (b"\0" if len(l4) % 2 else b"")
            s = sum(struct.unpack("!%dH" % (len(d) // 2), d))
            while s >> 16:
                s = (s & 0xFFFF) + (s >> 16)
            l4[2:4] = struct.pack("!H", (~s) & 0xFFFF)
        else:
            _l4_csum(src, dst, proto, l4, ck)
    if fix_ip:
        _ip_csum(ip)
    eth = b"\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02" + struct.pack("!H", ethertype)
    f = bytearray(eth + bytes(ip) + bytes(l4))
    if L is None:
        L = max(60, len(f))
    if len(f) < L:
        f += b"\0" * (L - len(f))
    return bytes(f[:L])


def ipv6(proto=6, payload=b"", L=None, sport=1000, dport=2000, plen=None, ver=6, fix=True):
    src = bytes(range(16))
    dst = bytes(range(100, 116))
    if proto == 6:
        l4 = bytearray(struct.pack("!HHIIBBHHH", sport, dport, 1, 2, 0x50, 0x10, 100, 0, 0)) + payload
        ck = 16
    elif proto == 17:
        l4 = bytearray(struct.pack("!HHHH", sport, dport, 8 + len(payload), 0)) + payload
        ck = 6
    else:
        l4 = bytearray(payload)
        ck = None
    n = len(l4) if plen is None else plen
    if fix and ck is not None:
        l4[ck:ck + 2] = b"\0\0"
        d = bytes(l4) + (b"\0" if len(l4) % 2 else b"")
        s = sum(struct.unpack("!%dH" % (len(d) // 2), d))
        s += sum(struct.unpack("!16H", src + dst)) + proto + len(l4)
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        c = (~s) & 0xFFFF
        l4[ck:ck + 2] = struct.pack("!H", c if c else 0xFFFF)
    hdr = struct.pack("!IHBB", ver << 28, n & 0xFFFF, proto, 64) + src + dst
    f = bytearray(b"\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02\x86\xdd" + hdr + bytes(l4))
    if L is None:
        L = max(60, len(f))
    f += b"\0" * max(0, L - len(f))
    return bytes(f[:L])


def edge_frames() -> list[bytes]:
    """SURVEY.md 8(a) edge-case set."""
    fr: list[bytes] = []
    good = ipv4()
    # frame length < 14 and < 34
    for L in (0, 1, 6, 12, 13, 14, 15, 20, 33, 34, 35):
        fr.append(good[:L])
    fr.append(ipv4(proto=6)[:53])
    # version != 4, ihl 0..15
    for v in (0, 3, 5, 6, 15):
        fr.append(ipv4(ver=v))
    for ihl in range(0, 16):
        fr.append(ipv4(ihl=ihl, payload=b"x" * 10))
        fr.append(ipv4(ihl=ihl, proto=17, payload=b"y" * 9))
    # fragments: MF, offset, DF, RF
    for fo in (0x2000, 0x0001, 0x1fff, 0x2001, 0x4000, 0x8000, 0xC000, 0x6000):
        fr.append(ipv4(flags_off=fo))
        fr.append(ipv4(flags_off=fo, proto=17))
    # ip_len < ihl*4, 14+ip_len > L, ip_len < L (padding)
    for tl in (0, 1, 19, 20, 21, 39, 40, 41, 46, 47, 100, 0xFFFF):
        fr.append(ipv4(ip_len=tl, fix_l4=False))
    fr.append(ipv4(payload=b"p" * 3, L=80))
    # protocols
    for p in (0, 2, 4, 41, 47, 50, 58, 132, 255):
        fr.append(ipv4(proto=p, payload=b"z" * 12))
    # TCP: l4len < 20, doff 0..15, doff*4 > l4len, options, odd lengths
    for n in (0, 1, 8, 19):
        fr.append(ipv4(proto=6, l4=b"\x00\x50\x01\xbb" + b"\x00" * max(0, n - 4), fix_l4=False)
                  if n >= 4 else ipv4(proto=6, l4=b"\x00" * n, fix_l4=False))
    for d in range(0, 16):
        fr.append(ipv4(proto=6, doff=d, payload=b"q" * 7))
        fr.append(ipv4(proto=6, doff=d, payload=b""))
    for pl in (1, 2, 3, 5, 31, 255, 256, 1459, 1460, 1973):
        fr.append(ipv4(proto=6, payload=bytes(range(256)) * (pl // 256) + bytes(range(pl % 256))))
    # doff*4 > l4len with a VALID checksum: aborts the reference as IX builds it
    for d, pl in ((6, 0), (15, 0), (15, 39), (6, 3), (8, 11), (8, 12)):
        fr.append(ipv4(proto=6, doff_field=d, payload=b"d" * pl))
    for fl in (0x01, 0x02, 0x03, 0x12, 0x3f, 0xff, 0xc0):
        fr.append(ipv4(proto=6, tcp_flags=fl))
    # ports >= 32768 on both sides
    for sp, dp in ((1, 1), (32767, 32768), (32768, 32767), (50000, 80), (80, 50000), (65535, 65535),
                   (0, 0), (0x8000, 0x8000)):
        fr.append(ipv4(proto=6, sport=sp, dport=dp))
        fr.append(ipv4(proto=17, sport=sp, dport=dp))
    # UDP: len < 8, > remaining, != ip_len - ihl*4, checksum 0 and 0xffff
    for ul in (0, 1, 7, 8, 9, 20, 26, 27, 46, 47, 1000):
        fr.append(ipv4(proto=17, payload=b"u" * 18, udp_len=ul))
    fr.append(ipv4(proto=17, payload=b"u" * 18, fix_l4=False))  # checksum 0: unchecked
    fr.append(ipv4(proto=17, l4=b"\x00\x35\x00\x35\x00\x04", fix_l4=False))  # l4len < 8
    fr.append(ipv4(proto=17, l4=b"\x00\x35\x00\x35", fix_l4=False, L=38))
    fr.append(ipv4(proto=17, l4=b"\x00\x35\x00\x35", fix_l4=False, L=60))
    for pl in range(0, 40):
        fr.append(ipv4(proto=17, payload=bytes([0xff] * pl)))  # may hit computed 0 -> 0xffff
    # ICMP: short, bad checksum, echo, reply, others
    fr.append(ipv4(proto=1, l4=b"\x08\x00\x00\x00", fix_l4=False))
    fr.append(ipv4(proto=1, l4=b"\x08\x00\xf7\xff\x00\x00\x00\x00", fix_l4=False))
    for t in (0, 3, 8, 11, 13):
        fr.append(ipv4(proto=1, icmp_type=t, payload=b"ping" * 5))
        fr.append(ipv4(proto=1, icmp_type=t, payload=b"odd"))
    bad = bytearray(ipv4(proto=1, icmp_type=8, payload=b"ping"))
    bad[40] ^= 1
    fr.append(bytes(bad))
    fr.append(ipv4(proto=1, l4=b"\x00" * 8, fix_l4=False))  # all-zero ICMP: residual 0xffff
    # IPv6, ARP, VLAN, others
    fr.append(ipv6())
    fr.append(ipv6(proto=17, payload=b"v6" * 10))
    fr.append(ipv4(ethertype=0x0806))
    fr.append(ipv4(ethertype=0x0806)[:14])
    fr.append(ipv4(ethertype=0x0806)[:10])
    fr.append(ipv4(ethertype=0x8100))
    fr.append(ipv4(ethertype=0x88cc))
    fr.append(ipv4(ethertype=0x0000))
    # bad IP checksum, bad L4 checksum, both
    fr.append(ipv4(fix_ip=False))
    fr.append(ipv4(fix_l4=False, payload=b"abc"))
    fr.append(ipv4(fix_ip=False, fix_l4=False, payload=b"abc"))
    fr.append(ipv4(proto=17, fix_ip=False, payload=b"abc"))
    b2 = bytearray(ipv4(proto=6, payload=b"checksum"))
    b2[60] ^= 0x80
    fr.append(bytes(b2))
    # all-zero IP header (ethertype IPv4) and all-zero frame
    fr.append(b"\x02" * 12 + b"\x08\x00" + b"\x00" * 46)
    fr.append(b"\x00" * 60)
    fr.append(b"\xff" * 60)
    # max length frames (mbuf data is 2048 B)
    fr.append(ipv4(proto=6, payload=bytes((i * 7) & 0xFF for i in range(2048 - 54))))
    fr.append(ipv4(proto=17, payload=bytes((i * 13) & 0xFF for i in range(2048 - 42))))
    fr.append(ipv4(proto=6, payload=b"x" * 100, L=2048))
    return fr


def fuzz_frames(rng: np.random.Generator, n: int) -> list[bytes]:
    """Valid frames with structured mutations of the fields the path reads."""
    base = []
    for L, proto, ihl in ((60, 6, 5), (74, 17, 5), (120, 6, 7), (590, 17, 5), (300, 6, 15),
                          (60, 1, 5), (1514, 6, 5), (98, 1, 5)):
        if proto == 1:
            base.append(ipv4(proto=1, icmp_type=8, payload=bytes(rng.integers(0, 256, L - 42, dtype=np.uint8))))
        else:
            rows = traces.build_ipv4(rng, 1, L, proto, ihl=ihl)
            base.append(bytes(rows[0]))
    out = []
    fields = [(12, 2), (14, 1), (16, 2), (20, 2), (23, 1), (24, 2), (26, 8), (34, 4), (38, 2),
              (40, 2), (46, 1), (47, 1), (50, 2)]
    for _ in range(n):
        f = bytearray(base[int(rng.integers(len(base)))])
        k = int(rng.integers(0, 4))
        for _ in range(k):
            col, w = fields[int(rng.integers(len(fields)))]
            if col + w <= len(f):
                f[col:col + w] = bytes(rng.integers(0, 256, w, dtype=np.uint8))
        if rng.random() < 0.2:
            f = f[:int(rng.integers(0, len(f) + 1))]
        out.append(bytes(f))
    return out


def save(name: str, frames: list[bytes], key: bytes, nb: int, dev: int, flags: int, note: str,
         fdir: list[bytes] | None = None, cpu: int = 0):
    rec, csum, tcpx, tcpx_hdr = run_ref(frames, key, nb, dev, flags, fdir, cpu, full=True)
    tr = traces.pack(frames)
    path = os.path.join(HERE, name + ".npz")
    extra = {}
    if fdir:
        # struct ixg_fdir_filter rows (12 bytes each) and the CPU they steer to
        extra = {"fdir": np.frombuffer(b"".join(fdir), np.uint8).reshape(-1, 12), "fdir_cpu": np.uint16(cpu)}
    np.savez_compressed(path, blob=tr.blob, off=tr.off, len=tr.len,
                        key=np.frombuffer(key, np.uint8), nb_rx_fgs=np.uint16(nb),
                        dev_idx=np.uint16(dev), flags=np.uint32(flags), rec=rec, csum=csum,
                        tcpx=tcpx, tcpx_hdr=tcpx_hdr, note=np.array(note), **extra)
    v = rec[:, 2]
    print(f"{name}: {len(frames)} frames, verdicts {dict(zip(*np.unique(v, return_counts=True)))}")


def icmp_frames(rng: np.random.Generator) -> list[bytes]:
    """Echo requests icmp_input reflects (every ICMP length class, odd and
    even, IP options, Ethernet padding past the IP length, the largest mbuf
    frame, host address equal to and different from the frame's
    destination) among frames it does not (other ICMP types, bad checksum,
    short) and non-ICMP frames."""
    fr = []
    for pl in list(range(0, 40)) + [55, 56, 64, 100, 255, 256, 511, 1000, 1472, 2048 - 42]:
        fr.append(ipv4(proto=1, icmp_type=8, payload=bytes(rng.integers(0, 256, pl, dtype=np.uint8))))
    for ihl in range(6, 16):
        fr.append(ipv4(proto=1, icmp_type=8, ihl=ihl, payload=bytes(rng.integers(0, 256, 21, dtype=np.uint8))))
        fr.append(ipv4(proto=1, icmp_type=8, ihl=ihl, payload=bytes(rng.integers(0, 256, 64, dtype=np.uint8))))
    for L in (80, 128, 333):  # Ethernet padding past the IP length
        fr.append(ipv4(proto=1, icmp_type=8, payload=b"pad", L=L))
    for dst in (b"\x0a\x00\x00\x02", b"\xc0\xa8\x01\x07", b"\xff\xff\xff\xff"):
        fr.append(ipv4(proto=1, icmp_type=8, dst=dst, payload=b"addr" * 3))
    for t in (0, 3, 11, 13, 17):
        fr.append(ipv4(proto=1, icmp_type=t, payload=b"other" * 3))
    bad = bytearray(ipv4(proto=1, icmp_type=8, payload=b"bad checksum"))
    bad[44] ^= 4
    fr.append(bytes(bad))
    fr.append(ipv4(proto=1, l4=b"\x08\x00\xf7\xff", fix_l4=False))
    fr.append(ipv4(proto=6, payload=b"tcp"))
    fr.append(ipv4(proto=17, payload=b"udp"))
    return fr


def save_icmp(key: bytes):
    """icmp.npz: frames before and after the reference's eth_input with
    CFG.mac / CFG.host_addr set (icmp_reflect rewrites ICMP_ECHO frames)."""
    rng = np.random.default_rng(0x1B0009)
    frames = icmp_frames(rng)
    frames = frames + [bytes(f) for f in fuzz_frames(rng, 300) if len(f) > 23 and f[23] == 1]
    mac = bytes([0x02, 0x1b, 0x0c, 0xa3, 0x55, 0xee])
    host = 0x0a000002  # 10.0.0.2, the frames' destination: the IP checksum stays valid
    rec, csum, tcpx, tcpx_hdr, refl, after = run_ref(frames, key, 128, 0, 0, host=(mac, host))
    assert (refl == (rec[:, 2] == 0x03)).all(), "reflected frames are the ICMP_ECHO records"
    host2 = 0xc0a80107  # another address: the reference leaves the IP checksum as it was
    _, _, _, _, refl2, after2 = run_ref(frames, key, 128, 0, 0, host=(mac, host2))
    assert (refl2 == refl).all()
    tr = traces.pack(frames)

    def laid_out(cat):  # the concatenated frames -> tr's layout (4-aligned starts)
        out, pos = tr.blob.copy(), 0
        for o, L in zip(tr.off.astype(np.int64), tr.len.astype(np.int64)):
            out[o:o + L] = cat[pos:pos + L]
            pos += L
        return out
    after, after2 = laid_out(after), laid_out(after2)
    np.savez_compressed(os.path.join(HERE, "icmp.npz"), blob=tr.blob, off=tr.off, len=tr.len,
                        key=np.frombuffer(key, np.uint8), nb_rx_fgs=np.uint16(128), dev_idx=np.uint16(0),
                        flags=np.uint32(0), rec=rec, csum=csum, tcpx=tcpx, tcpx_hdr=tcpx_hdr, reflected=refl,
                        mac=np.frombuffer(mac, np.uint8), host_addr=np.uint32(host), after=after,
                        host_addr2=np.uint32(host2), after2=after2,
                        note=np.array("frames after eth_input with icmp_reflect's CFG.mac / CFG.host_addr "
                                      "(host order), two host addresses"))
    print(f"icmp: {len(frames)} frames, {int(refl.sum())} reflected")


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle ref")
    if sys.argv[1:] == ["icmp"]:
        save_icmp(traces.RSS_KEY)
        return
    key = traces.RSS_KEY
    rng = np.random.default_rng(0x1B0001)
    edge = edge_frames()
    tcp64 = [bytes(r) for r in traces.build_ipv4(rng, 600, 60, 6)]
    mix = []
    for L, proto in ((60, 17), (590, 6), (590, 17), (1514, 6), (1514, 17), (61, 6), (333, 17)):
        mix += [bytes(r) for r in traces.build_ipv4(rng, 40, L, proto)]
    for ihl in range(6, 16):
        mix += [bytes(r) for r in traces.build_ipv4(rng, 6, 120, 6, ihl=ihl)]
        mix += [bytes(r) for r in traces.build_ipv4(rng, 6, 121, 17, ihl=ihl)]
    badc = [bytes(r) for r in traces.build_ipv4(rng, 100, 60, 6)]
    badc = [bytes(bytearray(f[:24]) + bytes([f[24] ^ 1]) + f[25:]) if i % 2 else
            bytes(bytearray(f[:50]) + bytes([f[50] ^ 0x10]) + f[51:]) for i, f in enumerate(badc)]
    fuzz = fuzz_frames(rng, 1500)
    v6 = [bytes(r) for r in traces.build_ipv6(rng, 30, 94, 6)] + \
         [bytes(r) for r in traces.build_ipv6(rng, 30, 95, 17)] + \
         [ipv6(), ipv6(proto=17), ipv6(plen=10), ipv6(plen=0), ipv6(ver=4), ipv6(proto=58, payload=b"x" * 8),
          ipv6()[:50], ipv6()[:57], ipv6(proto=17, payload=b"a" * 3)]
    save("default", edge + tcp64 + mix + badc + fuzz, key, 128, 0, 0,
         "MS RSS key, nb_rx_fgs 128, dev 0, checksum drops on")
    save("nocsumdrop_dev3_fg512", edge + badc + fuzz[:500], key, 512, 3, F_NO_CSUM_DROP,
         "NO_CSUM_DROP, nb_rx_fgs 512, dev_idx 3")
    key2 = bytes(rng.integers(0, 256, 40, dtype=np.uint8))
    save("randkey_fg16", tcp64[:200] + mix[:200], key2, 16, 1, 0, "random RSS key, 16 groups, dev 1")
    save("ipv6ext", v6 + edge[:80] + mix[:40], key, 128, 0, F_IPV6,
         "IXG_F_IPV6 extension (v6 RSS over 36 B is unpinned; v6 L4 checksum from ip6_chksum_pseudo_partial)")
    # flow director: filters for a third of the TCP frames (every option
    # length, long and short), the reverse direction of others (no match),
    # UDP / fragment / bad-checksum frames carrying a filtered tuple
    tcp = [f for f in tcp64 + mix if f[23] == 6]
    hit = tcp[::3]
    filt = [fdir_filter(f) for f in hit] + [fdir_filter(f, swap=True) for f in tcp[1::7]]
    udp_same = []
    for f in hit[:40]:
        g = bytearray(f)
        g[23] = 17  # same tuple, UDP: the TCP filter does not apply
        udp_same.append(bytes(g))
    frag_same = []
    for f in hit[40:80]:
        g = bytearray(f)
        g[20] |= 0x20  # MF: a fragment, no L4 match
        frag_same.append(bytes(g))
    badc_hit = [bytes(bytearray(f[:24]) + bytes([f[24] ^ 1]) + f[25:]) for f in hit[80:120]]
    filt += [fdir_filter(f) for f in badc_hit]
    save("fdir", tcp + udp_same + frag_same + badc_hit + edge[:120] + fuzz[:300], key, 64, 2, 0,
         "flow-director filters (FLM -> outbound flow group 8192 + cpu 5), nb_rx_fgs 64, dev_idx 2",
         fdir=filt, cpu=5)
    save_icmp(key)


if __name__ == "__main__":
    main()
