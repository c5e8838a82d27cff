#!/usr/bin/env python3
"""Generate the golden TX vectors from the reference's
own code.

Each segment goes through oracle/_ref/ixref_tx (oracle/ref_harness/
harness_tx.c): the reference's tcp_output_packet + ip_send_one
(dp/net/tcp_api.c:773-826, dp/net/ip.c:192-219) for TCP, with the seed of
the reference's inet_chksum_pseudo (dp/lwip/inet_chksum.c:353-357) in the
checksum field (the offload frame), plus the checksums the NIC computes from
the reference's chksum_internet and inet_chksum_pseudo_partial (the full
frame); udp_output is restated over the reference's ip_setup_header and
chksum_internet (udp.c is unbuildable here). The fixture holds the inputs
and both expected frames per segment.

Re-run:  make -C oracle ref && python tests/golden/make_golden_tx.py
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

from ix_amd import tx  # noqa: E402

TXH = os.path.join(ROOT, "oracle", "_ref", "ixref_tx")


def run_tx(b: tx.TxBatch):
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(b"IXGTXIN\0")
            f.write(struct.pack("<I", b.n))
            f.write(b.src_mac)
            f.write(struct.pack("<I", b.dmacs.shape[0]))
            f.write(np.ascontiguousarray(b.dmacs, dtype=np.uint8).tobytes())
            f.write(np.ascontiguousarray(b.segs).tobytes())
            f.write(struct.pack("<I", b.buf.size))
            f.write(b.buf.tobytes())
        subprocess.run([TXH, fi, fo], check=True)
        raw = open(fo, "rb").read()
    assert raw[:8] == b"IXGTXOT\0"
    n = struct.unpack_from("<I", raw, 8)[0]
    pos = 12
    lens = np.zeros((2, n), dtype=np.uint16)
    frames = np.zeros((2, n, 1536), dtype=np.uint8)
    for i in range(n):
        for k in range(2):
            (L,) = struct.unpack_from("<H", raw, pos)
            pos += 2
            lens[k, i] = L
            frames[k, i, :L] = np.frombuffer(raw, np.uint8, L, pos)
            pos += L
    return lens, frames


def edge_batch() -> tx.TxBatch:
    """Mixed TCP/UDP of every doff and a spread of lengths, plus the edges:
    empty UDP payload, TCP header only, maximum-size segments, invalid
    protocols and a TCP segment shorter than its header."""
    b = tx.make_segments("mixed", 192, seed=0x7A0001, layout="packed")
    s = b.segs
    s["seg_len"][0] = 0
    s["proto"][0] = 17
    s["seg_len"][1] = 20
    s["proto"][1] = 6
    s["proto"][2] = 1                     # not TCP/UDP: length 0
    s["proto"][3] = 6
    s["seg_len"][3] = 19                  # shorter than a TCP header: length 0
    s["proto"][4] = 17
    s["seg_len"][4] = min(1472, int(s["seg_len"][4]))
    s["src_ip"][5] = 0
    s["dst_ip"][5] = 0
    s["src_ip"][6] = 0xFFFFFFFF
    s["dst_ip"][6] = 0xFFFFFFFF
    # re-lay the output for the changed lengths
    span = tx.frame_span(s["seg_len"], s["proto"])
    oo = np.zeros(b.n, dtype=np.int64)
    oo[1:] = np.cumsum(span)[:-1]
    s["out_off"] = oo
    b.out_size = int(span.sum()) + 64
    return b


def main():
    out = os.path.join(HERE, "tx.npz")
    batches = [edge_batch(), tx.make_segments("tcp64", 64, seed=0x7A0002, layout="packed")]
    # one fixture: concatenate (second batch's offsets shifted)
    b0, b1 = batches
    s1 = b1.segs.copy()
    s1["seg_off"] += b0.buf.size
    s1["out_off"] += b0.out_size
    s1["dmac_idx"] %= b0.dmacs.shape[0]
    b = tx.TxBatch(np.concatenate([b0.buf, b1.buf]), np.concatenate([b0.segs, s1]), b0.src_mac, b0.dmacs,
                   b0.out_size + b1.out_size)
    lens, frames = run_tx(b)
    assert (lens[0] == lens[1]).all()
    # the offload frame differs from the full one only in the IP checksum
    # (bytes 24..25) and, for TCP, the TCP checksum field (bytes 50..51)
    diff = np.zeros((b.n, 4), dtype=np.uint8)
    for i in range(b.n):
        L = int(lens[1, i])
        a, f = frames[0, i, :L].copy(), frames[1, i, :L]
        if L:
            diff[i, 0:2] = a[24:26]
            a[24:26] = f[24:26]
            if b.segs["proto"][i] == 6:
                diff[i, 2:4] = a[50:52]
                a[50:52] = f[50:52]
            assert (a == f).all(), i
    blob = np.concatenate([frames[1, i, :int(lens[1, i])] for i in range(b.n)])
    np.savez_compressed(out, buf=b.buf, segs=b.segs.view(np.uint8).reshape(-1, 40), src_mac=np.frombuffer(
        b.src_mac, np.uint8), dmacs=b.dmacs, out_size=np.int64(b.out_size), len=lens[1], frames_full=blob,
        offload_csums=diff)
    print(f"wrote {out}: {b.n} segments, {int((lens[1] > 0).sum())} frames")


if __name__ == "__main__":
    main()
