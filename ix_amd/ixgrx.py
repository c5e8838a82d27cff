"""ctypes binding of the C ABI in include/ixgrx.h (ix_amd/libixgrx.so).

This is the host-side mirror of the drop-in boundary: ``RxEngine`` wraps one
``ixg_rx_init`` context (one per host thread, IX's per-CPU model) and exposes
the three batch entry points. PyTorch, when used, only supplies device
memory and streams; nothing here falls back to a CPU path: if the HIP
library is missing, importing the engine raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libixgrx.so")

ABI_VERSION = 3
IXG_F_NO_CSUM_DROP = 1 << 0
IXG_F_IPV6 = 1 << 1
IXG_TAIL_PAD = 64
IXG_NO_BUCKET = 0xFFFF

# struct ixg_rx_rec (16 bytes)
REC_DTYPE = np.dtype([
    ("fg_id", "<u2"), ("verdict", "u1"), ("flags", "u1"), ("l4_off", "<u2"), ("l4_len", "<u2"),
    ("rss_hash", "<u4"), ("pcb_bucket", "<u2"), ("tcp_flags", "u1"), ("rsvd", "u1"),
])
assert REC_DTYPE.itemsize == 16

VERDICTS = {
    0x01: "TCP", 0x02: "UDP", 0x03: "ICMP_ECHO", 0x04: "ARP", 0x05: "TCP6", 0x06: "UDP6",
    0x80: "DROP_ETHERTYPE", 0x81: "DROP_IP_SHORT", 0x82: "DROP_IP_VERSION", 0x83: "DROP_IP_IHL",
    0x84: "DROP_IP_FRAG", 0x85: "DROP_IP_LEN", 0x86: "DROP_IP_TRUNC", 0x87: "DROP_IP_PROTO",
    0x88: "DROP_TCP_SHORT", 0x89: "DROP_TCP_HDRLEN", 0x8A: "DROP_UDP_LEN", 0x8B: "DROP_ICMP_SHORT",
    0x8C: "DROP_ICMP_CSUM", 0x8D: "DROP_ICMP_TYPE", 0x8E: "DROP_CSUM_IP", 0x8F: "DROP_CSUM_L4",
    0x90: "DROP_IP6",
}
V = {name: code for code, name in VERDICTS.items()}

RF_IP_CSUM_CHECKED, RF_IP_CSUM_OK, RF_L4_CSUM_CHECKED, RF_L4_CSUM_OK, RF_RSS, RF_FDIR = 1, 2, 4, 8, 16, 32
RF_REPLY = 64  # IXG_RF_REPLY: the asynchronous path reflected the echo request in its mbuf

# symbols include/ixgrx.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "ixg_rx_init", "ixg_rx_fini", "ixg_rx_batch_dev", "ixg_rx_batch_mbufs", "ixg_rx_batch_host",
    "ixg_rx_hash_tables", "ixg_abi_version", "ixg_strerror", "ixg_rx_dispatch",
    "ixg_demux_load", "ixg_demux_batch_dev", "ixg_demux_batch_host", "ixg_rx_demux_batch_dev",
    "ixg_tx_set_macs", "ixg_tx_batch_dev", "ixg_tx_batch_host",
    "ixg_ev_batch_dev", "ixg_rx_set_split", "ixg_rx_set_fdir", "ixg_rx_launch_info",
    "ixg_rx_async_init", "ixg_rx_submit_mbufs", "ixg_rx_flush", "ixg_rx_poll", "ixg_rx_async_pending",
    "ixg_rx_async_stats",
    "ixg_rx_register_memory", "ixg_rx_unregister_memory", "ixg_tcp_ext_batch_dev", "ixg_rx_tcpx_batch_dev",
    "ixg_icmp_reflect_dev", "ixg_rx_icmp_batch_dev",
    "ixg_rx_set_icmp_reply",
)

# struct ixg_fdir_filter (12 bytes): raw IPs as in the frame, host-order ports
FDIR_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("src_port", "<u2"), ("dst_port", "<u2")])
assert FDIR_DTYPE.itemsize == 12
IXG_ETH_MAX_TOTAL_FG = 8192

# enum ixg_split (ixg_rx_set_split): how a context's launches divide a batch
SPLITS = {"auto": 0, "fast": 1, "short": 2, "long": 3, "general": 4}


class RxCfg(ctypes.Structure):
    _fields_ = [("rss_key", ctypes.c_uint8 * 40), ("nb_rx_fgs", ctypes.c_uint16),
                ("dev_idx", ctypes.c_uint16), ("flags", ctypes.c_uint32)]


class AsyncCfg(ctypes.Structure):
    """struct ixg_rx_async_cfg"""
    _fields_ = [("batch_frames", ctypes.c_uint32), ("batch_bytes", ctypes.c_uint32),
                ("max_wait_us", ctypes.c_uint32), ("depth", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class AsyncStats(ctypes.Structure):
    """struct ixg_rx_async_stats"""
    _fields_ = [(k, ctypes.c_uint64) for k in (
        "frames_submitted", "frames_returned", "frames_refused", "submit_calls", "poll_calls", "batches",
        "batches_by_time", "gather_ns", "launch_ns", "poll_ns", "wait_ns", "launch_max_ns",
        "image_bytes", "inplace_bytes", "frames_launched",
        "worst_total_ns", "worst_open_ns", "worst_gpu_ns", "worst_visible_ns", "worst_returned_ns",
        "worst_wait_ns", "worst_outside_ns", "worst_naps", "worst_nap_max_ns", "nap_max_ns")]


IXG_ASYNC_DIRECT = 1 << 0
IXG_ASYNC_ICMP_REFLECT = 1 << 1
IXG_ZC_MIN_LEN = 256  # registered frames shorter than this are gathered anyway
ASYNC_DEFAULTS = dict(batch_frames=16384, batch_bytes=512 << 10, max_wait_us=50, depth=2, direct=True)


class RxFrames(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("off", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("stride", ctypes.c_uint32), ("rsvd", ctypes.c_uint32)]


@dataclass
class Config:
    rss_key: bytes = bytes(40)
    nb_rx_fgs: int = 128
    dev_idx: int = 0
    flags: int = 0

    def to_c(self) -> RxCfg:
        c = RxCfg()
        if len(self.rss_key) != 40:
            raise ValueError("rss_key must be 40 bytes")
        ctypes.memmove(c.rss_key, self.rss_key, 40)
        c.nb_rx_fgs = self.nb_rx_fgs
        c.dev_idx = self.dev_idx
        c.flags = self.flags
        return c


_libs: dict[str, ctypes.CDLL] = {}


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libixgrx.so (or another build of it, for A/B timing); raises if
    it has not been built (no silent fallback)."""
    path = os.path.abspath(path)
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: build it with __graft_entry__.build() "
                           "(make -C ix_amd/csrc)")
    # PyTorch bundles its own libamdhip64.so.7. Loading torch first makes
    # libixgrx's NEEDED entry resolve to that already-loaded runtime, so the
    # process has ONE HIP runtime and torch's device pointers and streams
    # are valid for the kernels. (The reverse order leaves torch unable to
    # initialise.) Pure C consumers simply use /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    lib.ixg_rx_init.argtypes = [ctypes.POINTER(RxCfg), i32, ctypes.POINTER(vp)]
    lib.ixg_rx_init.restype = i32
    lib.ixg_rx_fini.argtypes = [vp]
    lib.ixg_rx_fini.restype = None
    lib.ixg_rx_batch_dev.argtypes = [vp, ctypes.POINTER(RxFrames), u32, vp, vp, vp]
    lib.ixg_rx_batch_dev.restype = i32
    lib.ixg_rx_batch_mbufs.argtypes = [vp, vp, u32, vp]
    lib.ixg_rx_batch_mbufs.restype = i32
    lib.ixg_rx_batch_host.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp]
    lib.ixg_rx_batch_host.restype = i32
    lib.ixg_rx_hash_tables.argtypes = [ctypes.POINTER(RxCfg), vp, ctypes.POINTER(u32)]
    lib.ixg_rx_hash_tables.restype = i32
    lib.ixg_abi_version.argtypes = []
    lib.ixg_abi_version.restype = i32
    lib.ixg_strerror.argtypes = [i32]
    lib.ixg_strerror.restype = ctypes.c_char_p
    lib.ixg_rx_dispatch.argtypes = [vp, vp, u32, vp, vp]
    lib.ixg_rx_dispatch.restype = u32
    lib.ixg_rx_set_split.argtypes = [vp, u32]
    lib.ixg_rx_set_split.restype = i32
    lib.ixg_rx_launch_info.argtypes = [vp, vp]
    lib.ixg_rx_launch_info.restype = i32
    lib.ixg_rx_set_fdir.argtypes = [vp, vp, u32, ctypes.c_uint16]
    lib.ixg_rx_set_fdir.restype = i32
    lib.ixg_rx_async_init.argtypes = [vp, ctypes.POINTER(AsyncCfg)]
    lib.ixg_rx_async_init.restype = i32
    lib.ixg_rx_submit_mbufs.argtypes = [vp, vp, u32]
    lib.ixg_rx_submit_mbufs.restype = i32
    lib.ixg_rx_flush.argtypes = [vp]
    lib.ixg_rx_flush.restype = i32
    lib.ixg_rx_poll.argtypes = [vp, vp, vp, u32, i32]
    lib.ixg_rx_poll.restype = i32
    lib.ixg_rx_async_pending.argtypes = [vp]
    lib.ixg_rx_async_pending.restype = i32
    lib.ixg_rx_async_stats.argtypes = [vp, vp, i32]
    lib.ixg_rx_async_stats.restype = i32
    lib.ixg_rx_register_memory.argtypes = [vp, vp, ctypes.c_size_t]
    lib.ixg_rx_register_memory.restype = i32
    lib.ixg_rx_unregister_memory.argtypes = [vp, vp]
    lib.ixg_rx_unregister_memory.restype = i32
    lib.ixg_rx_set_icmp_reply.argtypes = [vp, vp, u32]
    lib.ixg_rx_set_icmp_reply.restype = i32
    if lib.ixg_abi_version() != ABI_VERSION:
        raise RuntimeError("libixgrx ABI version mismatch")
    _libs[path] = lib
    return lib


def _check(rc: int, what: str, lib: ctypes.CDLL | None = None) -> None:
    if rc != 0:
        msg = (lib or load_library()).ixg_strerror(rc).decode()
        raise RuntimeError(f"{what} failed: {rc} ({msg})")


def hash_tables(cfg: Config) -> tuple[np.ndarray, int]:
    """The combined Toeplitz/CRC byte tables the kernels use (host-built)."""
    lib = load_library()
    tab = np.zeros(12 * 256, dtype=np.uint64)
    cc = ctypes.c_uint32(0)
    c = cfg.to_c()
    _check(lib.ixg_rx_hash_tables(ctypes.byref(c), tab.ctypes.data, ctypes.byref(cc)), "ixg_rx_hash_tables")
    return tab.reshape(12, 256), int(cc.value)


@dataclass
class RxEngine:
    """One ixg_rx context on HIP device `device` (lib_path: another build of
    the library, for A/B timing; default ix_amd/libixgrx.so). `split`: the
    launch split (SPLITS; ixg_rx_set_split), "auto" for the drop-in."""
    cfg: Config
    device: int = 0
    lib_path: str = LIB_PATH
    split: str = "auto"
    _ctx: ctypes.c_void_p = field(default_factory=ctypes.c_void_p, init=False)

    def __post_init__(self):
        self._lib = lib = load_library(self.lib_path)
        self._ccfg = self.cfg.to_c()
        _check(lib.ixg_rx_init(ctypes.byref(self._ccfg), self.device, ctypes.byref(self._ctx)), "ixg_rx_init", lib)
        if self.split != "auto":
            self.set_split(self.split)

    def set_split(self, split: str) -> None:
        _check(self._lib.ixg_rx_set_split(self._ctx, SPLITS[split]), "ixg_rx_set_split", self._lib)

    def launch_info(self) -> dict:
        """The last launch's split as the device chose it (ixg_rx_launch_info)."""
        info = np.zeros(3, dtype=np.uint32)
        _check(self._lib.ixg_rx_launch_info(self._ctx, info.ctypes.data), "ixg_rx_launch_info", self._lib)
        modes = {0: "fast", 1: "short", 2: "long"}
        return {"mode": modes.get(int(info[0]), "fast"), "big": bool(info[1]), "sampled": bool(info[2])}

    def set_fdir(self, filters, cpu_id: int = 0) -> None:
        """Flow-director perfect filters (FDIR_DTYPE array; empty = none)."""
        f = np.ascontiguousarray(filters if filters is not None else np.zeros(0, FDIR_DTYPE), dtype=FDIR_DTYPE)
        _check(self._lib.ixg_rx_set_fdir(self._ctx, f.ctypes.data if len(f) else None, len(f), cpu_id),
               "ixg_rx_set_fdir", self._lib)

    def close(self) -> None:
        if self._ctx:
            self._lib.ixg_rx_fini(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch_dev(self, base: int, off: int | None, length: int, stride: int, n: int, out: int,
                  csum: int | None = None, stream: int | None = None) -> None:
        """Device-resident batch: all arguments are device pointers (ints)."""
        fr = RxFrames(base, off or None, length, stride, 0)
        _check(self._lib.ixg_rx_batch_dev(self._ctx, ctypes.byref(fr), n, out, csum or None,
                                          stream or None), "ixg_rx_batch_dev", self._lib)

    def batch_host(self, blob: np.ndarray, off: np.ndarray | None, lens: np.ndarray, stride: int = 0,
                   want_csum: bool = False):
        """Host batch: copies in, runs, copies records (and residuals) back."""
        n = int(lens.shape[0])
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
        offa = None if off is None else np.ascontiguousarray(off, dtype=np.uint64)
        rec = np.zeros(n, dtype=REC_DTYPE)
        cs = np.zeros(n, dtype=np.uint32) if want_csum else None
        _check(self._lib.ixg_rx_batch_host(
            self._ctx, blob.ctypes.data, None if offa is None else offa.ctypes.data, lens.ctypes.data,
            stride, n, rec.ctypes.data, None if cs is None else cs.ctypes.data), "ixg_rx_batch_host", self._lib)
        return (rec, cs) if want_csum else rec

    def batch_trace(self, tr, want_csum: bool = False):
        return self.batch_host(tr.blob, tr.off, tr.len, tr.stride, want_csum)

    def batch_mbufs(self, mbuf_ptrs: np.ndarray) -> np.ndarray:
        """IX layout: array of host mbuf addresses (len @0, data @+64)."""
        ptrs = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        n = int(ptrs.shape[0])
        rec = np.zeros(n, dtype=REC_DTYPE)
        _check(self._lib.ixg_rx_batch_mbufs(self._ctx, ptrs.ctypes.data, n, rec.ctypes.data),
               "ixg_rx_batch_mbufs", self._lib)
        return rec


    # ---- the asynchronous host path (ixg_rx_submit_mbufs / ixg_rx_poll) ----
    def async_init(self, batch_frames: int = 16384, batch_bytes: int = 512 << 10, max_wait_us: int = 50,
                   depth: int = 2, direct: bool = True, icmp_reflect: bool = False) -> None:
        flags = (IXG_ASYNC_DIRECT if direct else 0) | (IXG_ASYNC_ICMP_REFLECT if icmp_reflect else 0)
        c = AsyncCfg(batch_frames, batch_bytes, max_wait_us, depth, flags)
        _check(self._lib.ixg_rx_async_init(self._ctx, ctypes.byref(c)), "ixg_rx_async_init", self._lib)

    def set_icmp_reply(self, mac: bytes, host_addr: int) -> None:
        """CFG.mac / CFG.host_addr of the echo replies IXG_ASYNC_ICMP_REFLECT builds."""
        m = (ctypes.c_uint8 * 6)(*bytes(mac)[:6])
        _check(self._lib.ixg_rx_set_icmp_reply(self._ctx, ctypes.cast(m, ctypes.c_void_p), host_addr),
               "ixg_rx_set_icmp_reply", self._lib)

    def submit_mbufs(self, mbuf_ptrs: np.ndarray) -> int:
        """Frames accepted (may be fewer than given: poll, then submit the rest)."""
        ptrs = np.ascontiguousarray(mbuf_ptrs, dtype=np.uint64)
        rc = self._lib.ixg_rx_submit_mbufs(self._ctx, ptrs.ctypes.data, int(ptrs.shape[0]))
        if rc < 0:
            _check(rc, "ixg_rx_submit_mbufs", self._lib)
        return rc

    def flush(self) -> None:
        _check(self._lib.ixg_rx_flush(self._ctx), "ixg_rx_flush", self._lib)

    def poll(self, max_frames: int, wait: bool = False) -> tuple[np.ndarray, np.ndarray]:
        """(mbuf pointers, records) of up to max_frames finished frames, oldest first."""
        mb = np.zeros(max_frames, dtype=np.uint64)
        rec = np.zeros(max_frames, dtype=REC_DTYPE)
        rc = self._lib.ixg_rx_poll(self._ctx, mb.ctypes.data, rec.ctypes.data, max_frames, 1 if wait else 0)
        if rc < 0:
            _check(rc, "ixg_rx_poll", self._lib)
        return mb[:rc], rec[:rc]

    def register_memory(self, base: int, nbytes: int) -> None:
        """Zero copy: the kernels read frames of mbufs in [base, base+nbytes) in place."""
        _check(self._lib.ixg_rx_register_memory(self._ctx, base, nbytes), "ixg_rx_register_memory", self._lib)

    def unregister_memory(self, base: int) -> None:
        _check(self._lib.ixg_rx_unregister_memory(self._ctx, base), "ixg_rx_unregister_memory", self._lib)

    def pending(self) -> int:
        rc = self._lib.ixg_rx_async_pending(self._ctx)
        if rc < 0:
            _check(rc, "ixg_rx_async_pending", self._lib)
        return rc

    def async_stats(self, reset: bool = False) -> dict:
        """The asynchronous path's counters (ixg_rx_async_stats)."""
        st = AsyncStats()
        _check(self._lib.ixg_rx_async_stats(self._ctx, ctypes.byref(st), int(reset)), "ixg_rx_async_stats", self._lib)
        return {k: int(getattr(st, k)) for k, _ in AsyncStats._fields_}


def make_mbufs(tr) -> tuple[np.ndarray, np.ndarray]:
    """Lay a trace out as IX mbufs (2112-B elements, len @0, data @+64).
    Returns (arena, pointer array); keep the arena alive while using pointers."""
    n = tr.n
    arena = np.zeros(n * 2112 + 64, dtype=np.uint8)
    base = (-arena.ctypes.data) % 64
    if tr.off is None and n and (tr.len == tr.len[0]).all():  # fixed stride, one length: vectorised
        L = int(tr.len[0])
        rows = arena[base:base + n * 2112].reshape(n, 2112)
        rows[:, :8] = np.frombuffer(np.uint64(L).tobytes(), np.uint8)
        rows[:, 64:64 + L] = tr.blob[:n * tr.stride].reshape(n, tr.stride)[:, :L]
        return arena, arena.ctypes.data + base + np.arange(n, dtype=np.uint64) * 2112
    offs = tr.offsets()
    for i in range(n):
        o = base + i * 2112
        L = int(tr.len[i])
        arena[o:o + 8] = np.frombuffer(np.uint64(L).tobytes(), np.uint8)
        arena[o + 64:o + 64 + L] = tr.blob[int(offs[i]):int(offs[i]) + L]
    ptrs = arena.ctypes.data + base + np.arange(n, dtype=np.uint64) * 2112
    return arena, ptrs
