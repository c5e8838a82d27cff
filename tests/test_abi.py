"""The C-ABI library: builds, loads without a GPU, exports what the header
declares, and its host-built hash tables reproduce the reference hashes."""
import ctypes
import os
import re
import struct

import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "ixgrx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ixg_[a-z_0-9]+)\s*\(", txt)))


def test_header_declares_exports():
    assert header_functions() == sorted(ixgrx.EXPORTS)


def test_integration_guide_lists_every_entry_point():
    """INTEGRATION.md section 7 names every function the header declares
    (the guide a maintainer binds from stays complete)."""
    guide = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    missing = [f for f in header_functions() if "`" + f + "`" not in guide]
    assert not missing, missing


def test_library_exports_every_symbol():
    lib = ixgrx.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.ixg_abi_version() == ixgrx.ABI_VERSION


def test_record_layout():
    assert ixgrx.REC_DTYPE.itemsize == 16
    assert [ixgrx.REC_DTYPE.fields[k][1] for k in ("fg_id", "verdict", "flags", "l4_off", "l4_len",
                                                     "rss_hash", "pcb_bucket", "tcp_flags")] == \
        [0, 2, 3, 4, 6, 8, 12, 14]


def test_init_rejects_bad_config():
    lib = ixgrx.load_library()
    ctx = ctypes.c_void_p()
    for nb, dev, fl in ((0, 0, 0), (3, 0, 0), (1024, 0, 0), (128, 200, 0), (128, 0, 0x80)):
        c = ixgrx.Config(traces.RSS_KEY, nb, dev, fl).to_c()
        assert lib.ixg_rx_init(ctypes.byref(c), 0, ctypes.byref(ctx)) == -22  # -EINVAL


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="ixg_rx_init"):
        ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY))


def test_hash_tables_reproduce_reference_hashes():
    """XOR of the 12 table entries == bit-serial Toeplitz and tcp_to_idx."""
    key = bytes(np.random.default_rng(1).integers(0, 256, 40, dtype=np.uint8))
    for k in (traces.RSS_KEY, key):
        tab, cc = ixgrx.hash_tables(ixgrx.Config(k))
        L = oracle.lib()
        rng = np.random.default_rng(7)
        kb = np.frombuffer(k, np.uint8)
        for _ in range(300):
            t = rng.integers(0, 256, 12, dtype=np.uint8)
            h = 0
            for i in range(12):
                h ^= int(tab[i, t[i]])
            assert (h & 0xFFFFFFFF) == L.ixgo_toeplitz(kb.ctypes.data, t.ctypes.data, 12)
            src = struct.unpack("<I", t[0:4].tobytes())[0]
            dst = struct.unpack("<I", t[4:8].tobytes())[0]
            sport = (int(t[8]) << 8) | int(t[9])
            dport = (int(t[10]) << 8) | int(t[11])
            assert (((h >> 32) ^ cc) & 511) == L.ixgo_tcp_to_idx(dst, src, dport, sport)


def test_dispatch_host_only():
    """ixg_rx_dispatch routes records to the eth_input callees (pure host code)."""
    lib = ixgrx.load_library()
    recs = np.zeros(6, dtype=ixgrx.REC_DTYPE)
    recs["verdict"] = [0x01, 0x02, 0x03, 0x04, 0x8E, 0x80]
    seen = []
    CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)
    cbs = [CB(lambda u, m, r, n=n: seen.append((n, m))) for n in ("tcp", "udp", "icmp", "arp", "drop")]

    class Ops(ctypes.Structure):
        _fields_ = [(n, CB) for n in ("tcp", "udp", "icmp_echo", "arp", "drop")]
    ops = Ops(*cbs)
    mb = np.arange(100, 106, dtype=np.uint64)
    got = lib.ixg_rx_dispatch(mb.ctypes.data, recs.ctypes.data, 6, ctypes.cast(ctypes.pointer(ops), ctypes.c_void_p), None)
    assert got == 4
    assert seen == [("tcp", 100), ("udp", 101), ("icmp", 102), ("arp", 103), ("drop", 104), ("drop", 105)]


def test_tx_seg_layout_matches_header():
    """struct ixg_tx_seg as the C compiler lays it out (offsetof via gcc)."""
    import subprocess
    import tempfile
    from ix_amd import tx
    fields = [n for n in tx.SEG_DTYPE.names]
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"ixgrx.h\"\nint main(void){printf(\"%zu\", sizeof(struct ixg_tx_seg));"
    src += "".join(f'printf(" %zu", offsetof(struct ixg_tx_seg, {f}));' for f in fields) + "return 0;}"
    with tempfile.TemporaryDirectory() as td:
        c, exe = os.path.join(td, "t.c"), os.path.join(td, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(x) for x in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    assert got[0] == tx.SEG_DTYPE.itemsize
    assert got[1:] == [tx.SEG_DTYPE.fields[f][1] for f in fields]


def test_null_context_entry_points():
    """Every context entry point rejects a NULL context with -EINVAL before
    touching the device (CPU-checkable part of the ABI)."""
    lib = ixgrx.load_library()
    assert lib.ixg_rx_set_split(None, 0) == -22
    assert lib.ixg_rx_set_fdir(None, None, 0, 0) == -22
    assert lib.ixg_rx_batch_mbufs(None, None, 0, None) == -22
    assert lib.ixg_rx_batch_host(None, None, None, None, 0, 0, None, None) == -22
    assert ixgrx.FDIR_DTYPE.itemsize == 12
