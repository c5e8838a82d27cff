"""PCB demux tables and the host-side mirror of the demux entry points
(include/ixgrx.h "PCB demux"; the tcp_input step after the head,
dp/net/tcp_in.c:233-323, 500-510).

IX keeps, per flow group, 512 hash buckets of active PCBs
(``fgs[g]->active_tbl[tcp_to_idx(...)]``, inc/ix/ethfg.h:83) and a TIME-WAIT
list, and per CPU a listen list. ``DemuxTables.build`` turns those lists
(given as arrays in list order) into the CSR snapshot ``ixg_demux_load``
copies to the device. A connection's flow group and bucket are the ones its
packets hash to: the RSS Toeplitz hash masked by the RETA size, and
tcp_to_idx of the tuple, computed here from the same host-built byte tables
the kernels use (``ixg_rx_hash_tables``).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import ixgrx

PCB_DTYPE = np.dtype([("remote_ip", "<u4"), ("local_ip", "<u4"), ("remote_port", "<u2"),
                      ("local_port", "<u2"), ("id", "<u4")])
LISTEN_DTYPE = np.dtype([("local_ip", "<u4"), ("local_port", "<u2"), ("rsvd", "<u2"), ("id", "<u4"),
                         ("rsvd2", "<u4")])
DEMUX_DTYPE = np.dtype([("id", "<u4"), ("kind", "u1"), ("rsvd", "u1", (3,))])
assert PCB_DTYPE.itemsize == 16 and LISTEN_DTYPE.itemsize == 16 and DEMUX_DTYPE.itemsize == 8

D_NONE, D_ACTIVE, D_TIMEWAIT, D_LISTEN, D_RESET, D_DROP = range(6)
KINDS = {D_NONE: "NONE", D_ACTIVE: "ACTIVE", D_TIMEWAIT: "TIMEWAIT", D_LISTEN: "LISTEN", D_RESET: "RESET",
         D_DROP: "DROP"}
BUCKETS = 512
EXPORTS = ("ixg_demux_load", "ixg_demux_batch_dev", "ixg_demux_batch_host", "ixg_rx_demux_batch_dev")


class _Tables(ctypes.Structure):
    _fields_ = [("nfg", ctypes.c_uint32), ("n_listen", ctypes.c_uint32), ("active_start", ctypes.c_void_p),
                ("active", ctypes.c_void_p), ("tw_start", ctypes.c_void_p), ("tw", ctypes.c_void_p),
                ("listen", ctypes.c_void_p), ("n_out", ctypes.c_uint32), ("rsvd", ctypes.c_uint32)]


def _bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    if getattr(lib, "_ixg_demux_bound", False):
        return lib
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.ixg_demux_load.argtypes = [vp, ctypes.POINTER(_Tables)]
    lib.ixg_demux_load.restype = i32
    lib.ixg_demux_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), vp, u32, vp, vp]
    lib.ixg_demux_batch_dev.restype = i32
    lib.ixg_demux_batch_host.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp]
    lib.ixg_demux_batch_host.restype = i32
    lib.ixg_rx_demux_batch_dev.argtypes = [vp, ctypes.POINTER(ixgrx.RxFrames), u32, vp, vp, vp]
    lib.ixg_rx_demux_batch_dev.restype = i32
    lib._ixg_demux_bound = True
    return lib


def flow_of(cfg: ixgrx.Config, remote_ip, local_ip, remote_port, local_port):
    """(local flow group, bucket) of connections: the RSS hash of the tuple
    as its packets carry it (src = remote, dst = local; ixgbe.c:329-335,
    tcp_api.c:581-604) masked by nb_rx_fgs, and tcp_to_idx(local, remote,
    local_port, remote_port) (tcp_impl.h:381-387). IPs are raw (network
    order as loaded little-endian), ports host order."""
    tab, cc = ixgrx.hash_tables(cfg)
    rip = np.asarray(remote_ip, dtype=np.uint32)
    lip = np.asarray(local_ip, dtype=np.uint32)
    rp = np.asarray(remote_port, dtype=np.uint32)
    lp = np.asarray(local_port, dtype=np.uint32)
    # tuple bytes in wire order: src ip, dst ip, sport, dport
    tb = [(rip >> (8 * k)) & 0xFF for k in range(4)] + [(lip >> (8 * k)) & 0xFF for k in range(4)]
    tb += [(rp >> 8) & 0xFF, rp & 0xFF, (lp >> 8) & 0xFF, lp & 0xFF]
    h = np.zeros(rip.shape, dtype=np.uint64)
    for pos, b in enumerate(tb):
        h ^= tab[pos][b.astype(np.int64)]
    rss = (h & 0xFFFFFFFF).astype(np.uint32)
    bucket = (((h >> 32).astype(np.uint32) ^ np.uint32(cc)) & (BUCKETS - 1)).astype(np.uint32)
    fg = rss & np.uint32(cfg.nb_rx_fgs - 1)
    return fg.astype(np.uint32), bucket


@dataclass
class DemuxTables:
    """A CSR snapshot of one context's demux lists (struct ixg_demux_tables):
    nfg local flow groups, then n_out outbound groups (one per CPU: group
    nfg + cpu_id holds the connections whose frames the flow director steers
    to outbound flow group ETH_MAX_TOTAL_FG + cpu_id)."""
    nfg: int
    active_start: np.ndarray  # u32, (nfg+n_out)*512 + 1
    active: np.ndarray        # PCB_DTYPE
    tw_start: np.ndarray      # u32, nfg + n_out + 1
    tw: np.ndarray            # PCB_DTYPE
    listen: np.ndarray        # LISTEN_DTYPE
    n_out: int = 0

    @classmethod
    def from_lists(cls, nfg: int, active_fg, active_bucket, active: np.ndarray, tw_fg, tw: np.ndarray,
                   listen: np.ndarray, n_out: int = 0) -> "DemuxTables":
        """Lists given flat, in list order, with each entry's group (a local
        flow group < nfg, or nfg + cpu_id for an outbound group) and bucket
        for active PCBs; a stable sort keeps list order inside every
        (group, bucket) list."""
        active = np.ascontiguousarray(active, dtype=PCB_DTYPE)
        tw = np.ascontiguousarray(tw, dtype=PCB_DTYPE)
        ng = nfg + n_out
        afg = np.asarray(active_fg, dtype=np.int64)
        abk = np.asarray(active_bucket, dtype=np.int64)
        tfg = np.asarray(tw_fg, dtype=np.int64)
        if (afg >= ng).any() or (tfg >= ng).any() or (abk >= BUCKETS).any():
            raise ValueError("flow group or bucket out of range")
        row = afg * BUCKETS + abk
        order = np.argsort(row, kind="stable")
        astart = np.zeros(ng * BUCKETS + 1, dtype=np.uint32)
        astart[1:] = np.cumsum(np.bincount(row, minlength=ng * BUCKETS)[:ng * BUCKETS])
        torder = np.argsort(tfg, kind="stable")
        tstart = np.zeros(ng + 1, dtype=np.uint32)
        tstart[1:] = np.cumsum(np.bincount(tfg, minlength=ng)[:ng])
        return cls(nfg, astart, active[order].copy(), tstart, tw[torder].copy(),
                   np.ascontiguousarray(listen, dtype=LISTEN_DTYPE), n_out)

    @classmethod
    def build(cls, cfg: ixgrx.Config, active: np.ndarray, tw: np.ndarray, listen: np.ndarray,
              outbound=None, n_out: int = 0) -> "DemuxTables":
        """Place each PCB in the flow group and bucket its packets hash to.
        outbound: (active, tw, cpu of each active, cpu of each tw) of the
        CPUs' outbound connections, placed in group nfg + cpu (their bucket
        is tcp_to_idx all the same); n_out: outbound groups (CPUs)."""
        active = np.ascontiguousarray(active, dtype=PCB_DTYPE)
        tw = np.ascontiguousarray(tw, dtype=PCB_DTYPE)
        afg, abk = flow_of(cfg, active["remote_ip"], active["local_ip"], active["remote_port"],
                           active["local_port"])
        tfg, _ = flow_of(cfg, tw["remote_ip"], tw["local_ip"], tw["remote_port"], tw["local_port"])
        if outbound is not None:
            oa, ot, oac, otc = outbound
            oa = np.ascontiguousarray(oa, dtype=PCB_DTYPE)
            ot = np.ascontiguousarray(ot, dtype=PCB_DTYPE)
            _, obk = flow_of(cfg, oa["remote_ip"], oa["local_ip"], oa["remote_port"], oa["local_port"])
            active = np.concatenate([active, oa])
            afg = np.concatenate([afg, cfg.nb_rx_fgs + np.asarray(oac, np.uint32)])
            abk = np.concatenate([abk, obk])
            tw = np.concatenate([tw, ot])
            tfg = np.concatenate([tfg, cfg.nb_rx_fgs + np.asarray(otc, np.uint32)])
        return cls.from_lists(cfg.nb_rx_fgs, afg, abk, active, tfg, tw, listen, n_out)

    def to_c(self) -> _Tables:
        t = _Tables()
        t.nfg = self.nfg
        t.n_out = self.n_out
        t.n_listen = len(self.listen)
        t.active_start = self.active_start.ctypes.data
        t.active = self.active.ctypes.data if len(self.active) else None
        t.tw_start = self.tw_start.ctypes.data
        t.tw = self.tw.ctypes.data if len(self.tw) else None
        t.listen = self.listen.ctypes.data if len(self.listen) else None
        return t


def load(eng: ixgrx.RxEngine, tables: DemuxTables) -> None:
    lib = _bind(eng._lib)
    t = tables.to_c()
    ixgrx._check(lib.ixg_demux_load(eng._ctx, ctypes.byref(t)), "ixg_demux_load", lib)


def batch_dev(eng: ixgrx.RxEngine, base: int, off: int | None, stride: int, n: int, rec: int, out: int,
              stream: int | None = None) -> None:
    """Device-resident demux: all pointers are device pointers (ints)."""
    lib = _bind(eng._lib)
    fr = ixgrx.RxFrames(base, off or None, 0, stride, 0)
    ixgrx._check(lib.ixg_demux_batch_dev(eng._ctx, ctypes.byref(fr), rec, n, out, stream or None),
                 "ixg_demux_batch_dev", lib)


def rx_demux_dev(eng: ixgrx.RxEngine, base: int, off: int | None, length: int, stride: int, n: int, rec: int,
                 out: int, stream: int | None = None) -> None:
    """RX and demux in one pass on the device (the demux fused into the RX
    kernels): records into `rec`, demux records into `out`."""
    lib = _bind(eng._lib)
    fr = ixgrx.RxFrames(base, off or None, length, stride, 0)
    ixgrx._check(lib.ixg_rx_demux_batch_dev(eng._ctx, ctypes.byref(fr), n, rec, out, stream or None),
                 "ixg_rx_demux_batch_dev", lib)


def batch_host(eng: ixgrx.RxEngine, blob: np.ndarray, off, lens: np.ndarray, stride: int,
               rec: np.ndarray) -> np.ndarray:
    lib = _bind(eng._lib)
    n = int(lens.shape[0])
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
    rec = np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)
    out = np.zeros(n, dtype=DEMUX_DTYPE)
    ixgrx._check(lib.ixg_demux_batch_host(eng._ctx, blob.ctypes.data, None if offa is None else offa.ctypes.data,
                                          lens.ctypes.data, stride, n, rec.ctypes.data, out.ctypes.data),
                 "ixg_demux_batch_host", lib)
    return out


def tcp_keys(blob: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """PCB keys (remote = source, local = destination) of IPv4 frames at
    `offsets`, read as the demux kernel reads them: IP src/dst at bytes
    26..33, ports at 14 + 4*ihl. For building synthetic connection tables."""
    o = np.asarray(offsets, dtype=np.int64)
    b = blob

    def le32(p):
        return (b[p].astype(np.uint32) | (b[p + 1].astype(np.uint32) << 8) | (b[p + 2].astype(np.uint32) << 16)
                | (b[p + 3].astype(np.uint32) << 24))
    l4 = o + 14 + 4 * (b[o + 14] & 15).astype(np.int64)
    k = np.zeros(o.size, PCB_DTYPE)
    k["remote_ip"] = le32(o + 26)
    k["local_ip"] = le32(o + 30)
    k["remote_port"] = (b[l4].astype(np.uint32) << 8) | b[l4 + 1]
    k["local_port"] = (b[l4 + 2].astype(np.uint32) << 8) | b[l4 + 3]
    k["id"] = np.arange(o.size, dtype=np.uint32)
    return k
