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
        L.ixgo_rx_batch_fdir.argtypes = [ctypes.POINTER(_Cfg), vp, vp, vp, u32, u32, vp, vp, i32, i32, i32, vp, u32,
                                         u16]
        L.ixgo_rx_batch_fdir.restype = i32
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
        L.ixgo_pseudo_seed.argtypes = [u32, u32, u8, u16]
        L.ixgo_pseudo_seed.restype = u16
        L.ixgo_tx_batch.argtypes = [vp, vp, u32, vp, vp, u32, u32, vp, vp]
        L.ixgo_tx_batch.restype = i32
        L.ixgo_ev_batch.argtypes = [vp, vp, u32, vp, vp, vp, u32, u32, ctypes.c_uint64, u32, vp, vp]
        L.ixgo_ev_batch.restype = u32
        L.ixgo_tcp_ext_batch.argtypes = [vp, vp, u32, vp, u32, u32, vp]
        L.ixgo_tcp_ext_batch.restype = i32
        L.ixgo_icmp_reflect_batch.argtypes = [vp, vp, u32, vp, u32, vp, u32]
        L.ixgo_icmp_reflect_batch.restype = u32
        _lib = L
    return _lib


def _cfg(key: bytes, nb: int, dev: int, flags: int) -> _Cfg:
    c = _Cfg()
    ctypes.memmove(c.rss_key, bytes(key), 40)
    c.nb_rx_fgs, c.dev_idx, c.flags = nb, dev, flags
    return c


# struct ixg_fdir_filter (include/ixgrx.h)
FDIR_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("src_port", "<u2"), ("dst_port", "<u2")])


def rx_batch(key: bytes, nb: int, dev: int, flags: int, blob: np.ndarray, off, lens: np.ndarray,
             stride: int = 0, threads: int = 1, hash_mode: int = HASH_BITSERIAL, work: int = WORK_FULL,
             fdir=None, cpu_id: int = 0):
    """Records ([n,16] uint8) and residual words for a batch; `fdir`: an
    array of FDIR_DTYPE flow-director filters (ixg_rx_set_fdir) or None."""
    n = int(lens.shape[0])
    rec = np.zeros((n, 16), dtype=np.uint8)
    cs = np.zeros(n, dtype=np.uint32)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    c = _cfg(key, nb, dev, flags)
    if fdir is not None and len(fdir):
        fd = np.ascontiguousarray(fdir, dtype=FDIR_DTYPE)
        lib().ixgo_rx_batch_fdir(ctypes.byref(c), blob.ctypes.data, None if offa is None else offa.ctypes.data,
                                 lens.ctypes.data, stride, n, rec.ctypes.data, cs.ctypes.data, threads, hash_mode,
                                 work, fd.ctypes.data, len(fd), cpu_id)
        return rec, cs
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


REF_HARNESS = os.path.join(_HERE, "_ref", "ixref_rx")


def _write_frames(path: str, tr, key: bytes, n: int, nb: int, dev: int, flags: int) -> None:
    """The reference harnesses' frame file ("IXGRXIN1", harness_main.c)."""
    import struct
    offs = tr.offsets()[:n].astype(np.uint64)
    lens = tr.len[:n].astype(np.uint16)
    base = int(offs[0])
    end = int(offs[-1]) + int(lens[-1])
    blob = tr.blob[base:end]
    rel = (offs - base).astype(np.uint32)
    with open(path, "wb") as f:
        f.write(b"IXGRXIN1")
        f.write(struct.pack("<IIHH", n, flags, nb, dev))
        f.write(bytes(key))
        f.write(lens.tobytes())
        f.write(rel.tobytes())
        f.write(struct.pack("<I", len(blob)))
        f.write(blob.tobytes())


def ref_time(tr, key: bytes, seconds: float, nb: int = 128, dev: int = 0, flags: int = 0,
             max_frames: int = 65536):
    """1-core rate of the reference harness (oracle/_ref/ixref_rx, built from
    /root/reference sources by `make -C oracle ref`) over the first
    `max_frames` frames of `tr`, repeated for `seconds`. The harness places
    each frame in a zeroed 2112-B IX mbuf and runs eth_input plus the
    [NIC]-rule checksum/RSS calls: harness overhead included, so not dp/ix's
    own rate (ref_bench is). Returns (pkts/s, sample description) or (None, reason)."""
    import json
    import tempfile
    if not os.path.exists(REF_HARNESS):
        return None, "oracle/_ref/ixref_rx not built"
    n = min(max_frames, tr.n)
    with tempfile.TemporaryDirectory() as d:
        fi, fo = os.path.join(d, "in"), os.path.join(d, "out")
        _write_frames(fi, tr, key, n, nb, dev, flags)
        r = subprocess.run([REF_HARNESS, "-t", str(seconds), fi, fo], check=True, capture_output=True, text=True)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return 1e9 / d["ns_per_pkt"], f"oracle/_ref/ixref_rx (reference dp/net + dp/lwip objects) over {n} frames x " \
                                  f"{d['pkts'] // n} passes in {d['seconds']:.1f}s, 1 core"


REF_BENCH = os.path.join(_HERE, "_ref", "ixref_bench")


def ref_bench(tr, key: bytes, mode: str, procs: int, seconds: float, mbufs_per_proc: int = 1 << 16,
              nb: int = 128, dev: int = 0, max_frames: int = 1 << 16):
    """dp/ix's own RX path on `procs` host cores (oracle/_ref/ixref_bench,
    harness_bench.c: the reference's eth_input -> ip_input -> tcp_input_tmp
    -> tcp_input head with tcp_to_idx over pre-filled IX mbufs; mode "full"
    adds the reference's checksum and Toeplitz functions, the NIC's work).
    Returns the harness's JSON dict, or None when the binary is not built."""
    import json
    import tempfile
    if not os.path.exists(REF_BENCH):
        return None
    n = min(max_frames, tr.n)
    with tempfile.TemporaryDirectory() as d:
        fi = os.path.join(d, "in")
        _write_frames(fi, tr, key, n, nb, dev, 0)
        r = subprocess.run([REF_BENCH, mode, str(procs), str(seconds), str(mbufs_per_proc), fi], check=True,
                           capture_output=True, text=True, timeout=seconds + 120)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["frames"] = n
    return out


class _DemuxTables(ctypes.Structure):
    _fields_ = [("nfg", ctypes.c_uint32), ("n_listen", ctypes.c_uint32), ("active_start", ctypes.c_void_p),
                ("active", ctypes.c_void_p), ("tw_start", ctypes.c_void_p), ("tw", ctypes.c_void_p),
                ("listen", ctypes.c_void_p), ("n_out", ctypes.c_uint32), ("rsvd", ctypes.c_uint32)]


def demux_batch(nfg: int, active_start, active, tw_start, tw, listen, fg_base: int, blob: np.ndarray, off,
                lens: np.ndarray, stride: int, rec: np.ndarray, n_out: int = 0) -> np.ndarray:
    """ixgo_demux_batch (tcp_in.c:233-323, 500-510) over the CSR lists;
    returns the 8-byte demux records as an (n, 8) u8 array."""
    L = lib()
    if not hasattr(L, "_demux_bound"):
        vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
        L.ixgo_demux_batch.argtypes = [ctypes.POINTER(_DemuxTables), u32, vp, vp, vp, u32, u32, vp, vp]
        L.ixgo_demux_batch.restype = i32
        L._demux_bound = True
    arrs = [np.ascontiguousarray(a) for a in (active_start, active, tw_start, tw, listen)]
    t = _DemuxTables()
    t.nfg = nfg
    t.n_out = n_out
    t.n_listen = len(arrs[4])
    t.active_start, t.active, t.tw_start, t.tw, t.listen = [a.ctypes.data if a.size else None for a in arrs]
    n = int(lens.shape[0])
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    rec = np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)
    out = np.zeros((n, 8), dtype=np.uint8)
    L.ixgo_demux_batch(ctypes.byref(t), fg_base, blob.ctypes.data, None if offa is None else offa.ctypes.data,
                       lens.ctypes.data, stride, n, rec.ctypes.data, out.ctypes.data)
    return out


def tx_batch(seg_buf: np.ndarray, segs: np.ndarray, src_mac: bytes, dmacs: np.ndarray, out_size: int,
             flags: int = 0):
    """TX frames for struct ixg_tx_seg rows `segs` (oracle/ixgrx_oracle.c
    ixgo_tx_batch). Returns (output buffer, frame lengths)."""
    L = lib()
    buf = np.ascontiguousarray(seg_buf, dtype=np.uint8)
    sg = np.ascontiguousarray(segs)
    assert sg.dtype.itemsize == 40
    d = np.ascontiguousarray(dmacs, dtype=np.uint8).reshape(-1, 6)
    src = np.frombuffer(bytes(src_mac), dtype=np.uint8).copy()
    n = int(sg.shape[0])
    out = np.zeros(out_size, dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint16)
    L.ixgo_tx_batch(buf.ctypes.data, sg.ctypes.data, n, src.ctypes.data, d.ctypes.data, d.shape[0], flags,
                    out.ctypes.data, out_len.ctypes.data)
    return out, out_len


EV_DTYPE = np.dtype([("sysnr", "<u8"), ("arga", "<u8"), ("argb", "<u8"), ("argc", "<u8"), ("argd", "<u8")])
EV_PCB_DTYPE = np.dtype([("pcb_idx", "<u8"), ("cookie", "<u8")])


def ev_batch(blob: np.ndarray, off, stride: int, rec: np.ndarray, dmx, pcbs, iomap_base: int, flags: int = 0):
    """usys descriptors for a batch (oracle/ixgrx_oracle.c ixgo_ev_batch).
    Returns (events, frame indices, the frames after the optional UDP tuple
    writes)."""
    L = lib()
    b = np.ascontiguousarray(blob, dtype=np.uint8).copy()
    n = int(rec.shape[0])
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    r = np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)
    d = None if dmx is None else np.ascontiguousarray(dmx).view(np.uint8).reshape(n, 8)
    pc = np.ascontiguousarray(pcbs if pcbs is not None else np.zeros(0, EV_PCB_DTYPE), dtype=EV_PCB_DTYPE)
    ev = np.zeros(max(n, 1), dtype=EV_DTYPE)
    fi = np.zeros(max(n, 1), dtype=np.uint32)
    k = L.ixgo_ev_batch(b.ctypes.data, None if offa is None else offa.ctypes.data, stride, r.ctypes.data,
                        None if d is None else d.ctypes.data, pc.ctypes.data if pc.size else None, pc.size, n,
                        iomap_base, flags, ev.ctypes.data, fi.ctypes.data)
    return ev[:k].copy(), fi[:k].copy(), b


TCPX_DTYPE = np.dtype([("seqno", "<u4"), ("ackno", "<u4"), ("wnd", "<u2"), ("tcplen", "<u2"),
                       ("src_port", "<u2"), ("dst_port", "<u2")])


def icmp_reflect_batch(blob: np.ndarray, off, stride: int, rec: np.ndarray, mac: bytes, host_addr: int):
    """ICMP echo reflect (oracle/ixgrx_oracle.c ixgo_icmp_reflect_batch):
    (the frames with every IXG_V_ICMP_ECHO one rewritten, the count)."""
    L = lib()
    b = np.ascontiguousarray(blob, dtype=np.uint8).copy()
    n = int(rec.shape[0])
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    r = np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)
    m = (ctypes.c_uint8 * 6).from_buffer_copy(bytes(mac))
    k = L.ixgo_icmp_reflect_batch(b.ctypes.data, None if offa is None else offa.ctypes.data, stride, r.ctypes.data,
                                  n, m, host_addr)
    return b, int(k)


def tcp_ext_batch(blob: np.ndarray, off, stride: int, rec: np.ndarray, flags: int = 0):
    """The rest of the tcp_input head (oracle/ixgrx_oracle.c
    ixgo_tcp_ext_batch). Returns (struct ixg_tcp_ext rows as (n, 16) u8, the
    frames after the optional in-place conversion)."""
    L = lib()
    b = np.ascontiguousarray(blob, dtype=np.uint8).copy()
    n = int(rec.shape[0])
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    r = np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)
    ext = np.zeros((max(n, 1), 16), dtype=np.uint8)
    L.ixgo_tcp_ext_batch(b.ctypes.data, None if offa is None else offa.ctypes.data, stride, r.ctypes.data, n, flags,
                         ext.ctypes.data)
    return ext[:n].copy(), b
