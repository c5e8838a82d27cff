#!/usr/bin/env python3
"""Generate the golden PCB-demux vectors from the
reference's own code.

Frames go through oracle/_ref/ixref_rx (the reference eth_input path) for
their records; the records, frames and PCB lists then go through
oracle/_ref/ixref_demux, whose active and TIME-WAIT lookups are the
reference's tcp_input_find_list (dp/net/tcp_in.c:122-143, compiled from
/root/reference by `make -C oracle ref`). The listen walk and the no-PCB
outcome are restated there (tcp_in.c:273-304, 500-510; see
harness_demux.c). PCBs are placed in the flow group and bucket the
reference's record gives for their tuple (fg_id, tcp_to_idx).

Re-run:  make -C oracle ref && python tests/golden/make_golden_demux.py
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
sys.path.insert(0, HERE)

from ix_amd import traces  # noqa: E402
from make_golden import ipv4, run_ref  # noqa: E402

DEMUX = os.path.join(ROOT, "oracle", "_ref", "ixref_demux")
PCB = np.dtype([("remote_ip", "<u4"), ("local_ip", "<u4"), ("remote_port", "<u2"), ("local_port", "<u2"),
                ("id", "<u4")])
LISTEN = np.dtype([("local_ip", "<u4"), ("local_port", "<u2"), ("rsvd", "<u2"), ("id", "<u4"),
                   ("rsvd2", "<u4")])
BUCKETS = 512
TCP = 0x01


def run_demux(frames, rec, fg_base, nfg, astart, active, tstart, tw, listen, n_out=0):
    tr = traces.pack(frames)
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(b"IXGDMXI2")
            f.write(struct.pack("<7I", len(frames), fg_base, nfg, n_out, len(listen), len(active), len(tw)))
            for a in (astart, active, tstart, tw, listen):
                f.write(np.ascontiguousarray(a).tobytes())
            f.write(tr.len.astype(np.uint16).tobytes())
            f.write(tr.off.astype(np.uint32).tobytes())
            f.write(struct.pack("<I", len(tr.blob)))
            f.write(tr.blob.tobytes())
            f.write(np.ascontiguousarray(rec).tobytes())
        subprocess.run([DEMUX, fi, fo], check=True)
        raw = open(fo, "rb").read()
    assert raw[:8] == b"IXGDMXOT"
    n = struct.unpack_from("<I", raw, 8)[0]
    assert n == len(frames)
    return np.frombuffer(raw, dtype=np.uint8, count=8 * n, offset=12).reshape(n, 8).copy(), tr


def ip(b: bytes) -> int:
    return int(np.frombuffer(b, "<u4")[0])


def frames_and_records(rng, key, nb, dev, fdir_frac=0.0, cpu=0):
    fr = [bytes(r) for r in traces.build_ipv4(rng, 400, 60, 6)]
    for ihl in range(6, 16):  # ports behind IP options
        fr += [bytes(r) for r in traces.build_ipv4(rng, 3, 120, 6, ihl=ihl)]
    loc = [b"\x0a\x00\x00\x02", b"\x0a\x00\x00\x03"]
    for k in range(60):  # listener ports, exact and other local addresses
        fr.append(ipv4(proto=6, sport=int(rng.integers(1024, 65536)), dport=(80, 443, 8080, 9000)[k % 4],
                       src=bytes(rng.integers(0, 256, 4, dtype=np.uint8)), dst=loc[k % 2],
                       tcp_flags=(0x02, 0x10, 0x04, 0x14, 0x18)[k % 5]))
    for k in range(30):  # RST / other flags, random tuples
        fr.append(ipv4(proto=6, sport=int(rng.integers(1, 65536)), dport=int(rng.integers(1, 65536)),
                       src=bytes(rng.integers(0, 256, 4, dtype=np.uint8)),
                       dst=bytes(rng.integers(0, 256, 4, dtype=np.uint8)), tcp_flags=(0x04, 0x14, 0x11, 0x3f)[k % 4]))
    fr += [ipv4(proto=17), ipv4(proto=1, icmp_type=8, payload=b"ping"), ipv4(ethertype=0x0806),
           ipv4(fix_l4=False, payload=b"bad"), ipv4(proto=6, doff_field=15), ipv4(proto=6)[:40]]
    filt = None
    if fdir_frac:  # flow-director filters on a share of the TCP tuples (outbound connections)
        from make_golden import fdir_filter
        tcp = [f for f in fr if len(f) >= 38 and f[12:14] == b"\x08\x00" and f[23] == 6]
        filt = [fdir_filter(f) for f in tcp if rng.random() < fdir_frac]
    rec, _ = run_ref(fr, key, nb, dev, 0, filt, cpu)
    return fr, rec, filt


def tables(rng, fr, rec, nfg, fg_base, with_listen, n_out=0):
    tr = traces.pack(fr)
    tcp = np.nonzero(rec[:, 2] == TCP)[0]
    act_rows, act_keys, tw_fg, tw_keys = [], [], [], []
    nid = [1000]

    def key_of(i, id_):
        f = tr.blob[int(tr.off[i]):int(tr.off[i]) + int(tr.len[i])].tobytes()
        l4 = 14 + 4 * (f[14] & 15)
        return (ip(f[26:30]), ip(f[30:34]), (f[l4] << 8) | f[l4 + 1], (f[l4 + 2] << 8) | f[l4 + 3], id_)

    def new_id():
        nid[0] += 1
        return nid[0]

    ng = nfg + n_out
    for i in tcp:
        fg = int(rec[i, 0]) | (int(rec[i, 1]) << 8)
        g = fg - fg_base if fg < 8192 else nfg + (fg - 8192)  # fgs[fg_id]: local, or outbound after them
        b = int(rec[i, 12]) | (int(rec[i, 13]) << 8)
        u = rng.random()
        rk = key_of(i, new_id())
        near = list(rk)
        near[int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 16))
        if u < 0.35:  # active, sometimes behind a near miss or a duplicate
            if rng.random() < 0.3:
                act_rows.append((g, b)), act_keys.append(tuple(near[:4]) + (new_id(),))
            act_rows.append((g, b)), act_keys.append(rk)
            if rng.random() < 0.3:
                act_rows.append((g, b)), act_keys.append(rk[:4] + (new_id(),))
        elif u < 0.45:  # TIME-WAIT
            tw_fg.append(g), tw_keys.append(rk)
        elif u < 0.55:  # in both lists: the active one wins
            act_rows.append((g, b)), act_keys.append(rk)
            tw_fg.append(g), tw_keys.append(rk[:4] + (new_id(),))
        elif u < 0.65:  # only a near miss in its bucket
            act_rows.append((g, b)), act_keys.append(tuple(near[:4]) + (new_id(),))
        elif u < 0.7:  # right tuple, wrong bucket
            act_rows.append((g, (b + 1) % BUCKETS)), act_keys.append(rk)
    for _ in range(300):  # unrelated connections
        act_rows.append((int(rng.integers(0, max(128, ng))), int(rng.integers(0, BUCKETS))))
        act_keys.append((int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), int(rng.integers(0, 65536)),
                         int(rng.integers(0, 65536)), new_id()))
    for _ in range(40):
        tw_fg.append(int(rng.integers(0, max(128, ng))))
        tw_keys.append((int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), int(rng.integers(0, 65536)),
                        int(rng.integers(0, 65536)), new_id()))
    keep = [k for k, (g, _) in enumerate(act_rows) if 0 <= g < ng]
    act_rows = [act_rows[k] for k in keep]
    act_keys = [act_keys[k] for k in keep]
    tkeep = [k for k, g in enumerate(tw_fg) if 0 <= g < ng]
    tw_fg = [tw_fg[k] for k in tkeep]
    tw_keys = [tw_keys[k] for k in tkeep]
    row = np.array([g * BUCKETS + b for g, b in act_rows], dtype=np.int64)
    order = np.argsort(row, kind="stable")
    active = np.array(act_keys, dtype=PCB)[order]
    astart = np.zeros(ng * BUCKETS + 1, dtype=np.uint32)
    astart[1:] = np.cumsum(np.bincount(row, minlength=ng * BUCKETS))
    tfg = np.array(tw_fg, dtype=np.int64)
    torder = np.argsort(tfg, kind="stable")
    tw = np.array(tw_keys, dtype=PCB)[torder]
    tstart = np.zeros(ng + 1, dtype=np.uint32)
    tstart[1:] = np.cumsum(np.bincount(tfg, minlength=ng))
    listen = np.zeros(0, dtype=LISTEN)
    if with_listen:
        listen = np.array([(ip(b"\x0a\x00\x00\x03"), 80, 0, 1, 0), (0, 8080, 0, 2, 0), (ip(b"\x0a\x00\x00\x02"), 80, 0, 3, 0),
                           (0, 80, 0, 4, 0), (0, 443, 0, 5, 0), (ip(b"\x0a\x00\x00\x09"), 9000, 0, 6, 0),
                           (0, 7, 0, 7, 0)], dtype=LISTEN)
    return astart, active, tstart, tw, listen


def save(name, rng, key, nb, dev, nfg, with_listen, note, n_out=0, fdir_frac=0.0, cpu=0):
    fr, rec, filt = frames_and_records(rng, key, nb, dev, fdir_frac, cpu)
    fg_base = dev * 512
    astart, active, tstart, tw, listen = tables(rng, fr, rec, nfg, fg_base, with_listen, n_out)
    dmx, tr = run_demux(fr, rec, fg_base, nfg, astart, active, tstart, tw, listen, n_out)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), blob=tr.blob, off=tr.off, len=tr.len,
                        key=np.frombuffer(key, np.uint8), nb_rx_fgs=np.uint16(nb), dev_idx=np.uint16(dev),
                        rec=rec, nfg=np.uint32(nfg), active_start=astart, active=active, tw_start=tstart, tw=tw,
                        listen=listen, demux=dmx, note=np.array(note), n_out=np.uint32(n_out),
                        **({"fdir": np.frombuffer(b"".join(filt), np.uint8).reshape(-1, 12),
                            "fdir_cpu": np.uint16(cpu)} if filt else {}))
    kinds = dmx[:, 4]
    print(f"{name}: {len(fr)} frames, {len(active)} active, {len(tw)} tw, {len(listen)} listen, "
          f"kinds {dict(zip(*np.unique(kinds, return_counts=True)))}")


def main():
    if not os.path.exists(DEMUX):
        sys.exit("build the harness first: make -C oracle ref")
    rng = np.random.default_rng(0x1BD001)
    save("demux_default", rng, traces.RSS_KEY, 128, 2, 128, True,
         "MS key, 128 groups, dev_idx 2; listen list (exact, ANY, last-entry quirk)")
    save("demux_nolisten_nfg64", rng, traces.RSS_KEY, 128, 0, 64, False,
         "no listen list (RESET / DROP), tables for local groups 0..63 only")
    save("demux_fdir_outbound", rng, traces.RSS_KEY, 128, 1, 128, True,
         "flow-director filters on ~40% of the TCP tuples, steered to CPU 3: those frames' lookups use "
         "outbound group ETH_MAX_TOTAL_FG + 3 (snapshot group nfg + 3 of n_out 5)", n_out=5, fdir_frac=0.4, cpu=3)


if __name__ == "__main__":
    main()
