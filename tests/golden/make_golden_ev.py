#!/usr/bin/env python3
"""Generate the golden event-record vectors from the
reference's own code.

Frames and their RX records come from the RX fixture default.npz (the
reference's eth_input, many UDP cases) and the demux fixture
demux_default.npz (the reference's tcp_input_find_list); they go through
oracle/_ref/ixref_ev (oracle/ref_harness/harness_ev.c), whose descriptors are
written by the reference's usys_udp_recv / usys_tcp_recv
(inc/ix/syscall.h:360-365,416-420) with addresses from its
mempool_pagemem_to_iomap (inc/ix/mempool.h:259-263). The emission rule and
udp_input's tuple write are restated there (dp/net/udp.c:81-88 is
unbuildable here; recv_a_pbuf is static behind lwIP's callbacks).

Re-run:  make -C oracle ref && python tests/golden/make_golden_ev.py
"""
from __future__ import annotations

import os
import struct
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
EVH = os.path.join(ROOT, "oracle", "_ref", "ixref_ev")
EV = np.dtype([("sysnr", "<u8"), ("arga", "<u8"), ("argb", "<u8"), ("argc", "<u8"), ("argd", "<u8")])
PCB = np.dtype([("pcb_idx", "<u8"), ("cookie", "<u8")])


def run_ev(blob, off, rec, dmx, pcbs, iomap_base):
    n = len(off)
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fi, "wb") as f:
            f.write(b"IXGEVIN\0")
            f.write(struct.pack("<IIQII", n, len(pcbs), iomap_base, 0 if dmx is None else 1, blob.size))
            f.write(blob.tobytes())
            f.write(np.ascontiguousarray(off, dtype=np.uint64).tobytes())
            f.write(np.ascontiguousarray(rec, dtype=np.uint8).tobytes())
            if dmx is not None:
                f.write(np.ascontiguousarray(dmx, dtype=np.uint8).tobytes())
            f.write(np.ascontiguousarray(pcbs, dtype=PCB).tobytes())
        subprocess.run([EVH, fi, fo], check=True)
        raw = open(fo, "rb").read()
    assert raw[:8] == b"IXGEVOT\0"
    k = struct.unpack_from("<I", raw, 8)[0]
    ev = np.frombuffer(raw, EV, k, 12).copy()
    idx = np.frombuffer(raw, np.uint32, k, 12 + 40 * k).copy()
    bl = struct.unpack_from("<I", raw, 12 + 44 * k)[0]
    out_blob = np.frombuffer(raw, np.uint8, bl, 16 + 44 * k).copy()
    return ev, idx, out_blob


def main():
    rng = np.random.default_rng(0x7E0001)
    out = {}
    for tag, name, with_dmx in (("rx", "default", False), ("dmx", "demux_default", True)):
        z = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
        dmx = z["demux"] if with_dmx else None
        ids = dmx.view(np.uint32)[:, 0] if with_dmx else np.zeros(1, np.uint32)
        n_pcbs = int(ids.max()) + 1 if with_dmx else 0
        pcbs = np.zeros(n_pcbs, dtype=PCB)
        pcbs["pcb_idx"] = rng.integers(0, 1 << 48, size=n_pcbs, dtype=np.uint64)
        pcbs["cookie"] = rng.integers(0, 1 << 63, size=n_pcbs, dtype=np.uint64)
        iomap_base = int(rng.integers(1 << 40, 1 << 46)) & ~0xFFF
        ev, idx, blob = run_ev(z["blob"], z["off"], z["rec"], dmx, pcbs, iomap_base)
        out[tag + "_pcbs"] = pcbs
        out[tag + "_iomap"] = np.uint64(iomap_base)
        out[tag + "_ev"] = ev
        out[tag + "_idx"] = idx
        changed = np.nonzero(blob != z["blob"])[0]
        out[tag + "_tuple_pos"] = changed.astype(np.uint32)   # the tuple writes: positions and bytes
        out[tag + "_tuple_val"] = blob[changed]
        print(f"{name}: {len(ev)} events ({int((ev['sysnr'] == 0).sum())} UDP, "
              f"{int((ev['sysnr'] == 4).sum())} TCP), {changed.size} frame bytes rewritten")
    np.savez_compressed(os.path.join(HERE, "ev.npz"), **out)


if __name__ == "__main__":
    main()
