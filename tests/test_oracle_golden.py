"""The CPU restatement (oracle/) against the reference's own outputs.

The golden fixtures were produced by the reference's C code
(tests/golden/make_golden.py over oracle/_ref/ixref_rx); this pins the
oracle before it is trusted to check the HIP kernels.
"""
import struct

import numpy as np
import pytest

from oracle import oracle
from ix_amd import traces


def _fdir(golden):
    """The fixture's flow-director filters (FDIR_DTYPE) and CPU, or (None, 0)."""
    if "fdir" not in golden:
        return None, 0
    return np.ascontiguousarray(golden["fdir"]).view(oracle.FDIR_DTYPE).reshape(-1), int(golden["fdir_cpu"])


@pytest.mark.parametrize("hash_mode", [oracle.HASH_BITSERIAL, oracle.HASH_TABLE])
def test_oracle_matches_reference(golden, hash_mode):
    fd, cpu = _fdir(golden)
    rec, cs = oracle.rx_batch(bytes(golden["key"]), int(golden["nb_rx_fgs"]), int(golden["dev_idx"]),
                              int(golden["flags"]), golden["blob"], golden["off"], golden["len"],
                              hash_mode=hash_mode, fdir=fd, cpu_id=cpu)
    exp = golden["rec"]
    bad = np.nonzero((rec != exp).any(axis=1))[0]
    assert bad.size == 0, f"{golden['name']}: {bad.size} records differ, first {bad[:8]}: " \
                          f"{rec[bad[0]].tolist()} vs {exp[bad[0]].tolist()}"
    badc = np.nonzero(cs != golden["csum"])[0]
    assert badc.size == 0, f"{golden['name']}: residuals differ at {badc[:8]}"


def test_oracle_threads_match_single(golden):
    fd, cpu = _fdir(golden)
    a = oracle.rx_batch(bytes(golden["key"]), int(golden["nb_rx_fgs"]), int(golden["dev_idx"]),
                        int(golden["flags"]), golden["blob"], golden["off"], golden["len"], threads=1, fdir=fd,
                        cpu_id=cpu)
    b = oracle.rx_batch(bytes(golden["key"]), int(golden["nb_rx_fgs"]), int(golden["dev_idx"]),
                        int(golden["flags"]), golden["blob"], golden["off"], golden["len"], threads=4, fdir=fd,
                        cpu_id=cpu)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()


# Microsoft RSS verification suite (IPv4 with TCP ports); the reference's
# compute_toeplitz_hash reproduces all five (checked in the survey container).
RSS_VECTORS = [
    ("66.9.149.187", 2794, "161.142.100.80", 1766, 0x51CCC178),
    ("199.92.111.2", 14230, "65.69.140.83", 4739, 0xC626B0EA),
    ("24.19.198.95", 12898, "12.22.207.184", 38024, 0x5C2B394A),
    ("38.27.205.30", 48228, "209.142.163.6", 2217, 0xAFC7327F),
    ("153.39.163.191", 44251, "202.188.127.2", 1303, 0x10E828A2),
]


def _ip(s):
    return bytes(int(x) for x in s.split("."))


@pytest.mark.parametrize("src,sp,dst,dp,exp", RSS_VECTORS)
def test_toeplitz_known_answers(src, sp, dst, dp, exp):
    inp = _ip(src) + _ip(dst) + struct.pack("!HH", sp, dp)
    key = np.frombuffer(traces.RSS_KEY, np.uint8)
    buf = np.frombuffer(inp, np.uint8)
    assert oracle.lib().ixgo_toeplitz(key.ctypes.data, buf.ctypes.data, 12) == exp


def test_tcp_to_idx_sign_extension():
    # local port 50000 -> bucket 495 in the reference (a
    # zero-extending restatement would give 471)
    L = oracle.lib()
    local = struct.unpack("<I", bytes([10, 0, 0, 2]))[0]
    remote = struct.unpack("<I", bytes([10, 0, 0, 1]))[0]
    got = L.ixgo_tcp_to_idx(local, remote, 50000, 80)
    h = L.ixgo_crc32c_u64(L.ixgo_crc32c_u64(0xA36BDCBE, local), remote)
    zero_ext = L.ixgo_crc32c_u64(h, (50000 << 16) | 80) & 511
    sign_ext = L.ixgo_crc32c_u64(h, ((50000 << 16) | 80) | 0xFFFFFFFF00000000) & 511
    assert got == sign_ext and got != zero_ext


def test_crc32c_known_answer():
    # CRC-32C check value: crc32c("123456789") = 0xE3069283 with init/final
    # inversion; crc32q is the raw register step, so apply them around it.
    L = oracle.lib()
    data = b"123456789" + b"\0" * 7
    crc = 0xFFFFFFFF
    w0 = struct.unpack("<Q", data[:8])[0]
    crc = L.ixgo_crc32c_u64(crc, w0)
    # last byte alone: fold one byte via a u64 step on a zero-padded word is
    # not equal to a 1-byte step, so use the byte-wise definition instead
    b = data[8]
    crc ^= b
    for _ in range(8):
        crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    assert (~crc) & 0xFFFFFFFF == 0xE3069283


def test_chksum_internet_rfc1071_example():
    # RFC 1071 section 3 example: bytes 00 01 f2 03 f4 f5 f6 f7 -> sum ddf2 (BE)
    L = oracle.lib()
    b = np.frombuffer(bytes([0x00, 0x01, 0xF2, 0x03, 0xF4, 0xF5, 0xF6, 0xF7]), np.uint8)
    res = L.ixgo_chksum_internet(b.ctypes.data, 8)
    # result is ~sum in memory (LE) order: ~0xf2dd
    assert res == (~0xF2DD) & 0xFFFF
    z = np.zeros(20, np.uint8)
    assert L.ixgo_chksum_internet(z.ctypes.data, 20) == 0xFFFF  # all-zero header is invalid


def test_fdir_fixture_pins_the_outbound_group():
    """The flow-director fixture's matches carry the reference's outbound
    flow group (eth_recv_handle_fg_transition: ETH_MAX_TOTAL_FG + cpu_id) and
    IXG_RF_FDIR; frames of the same tuple that are UDP or fragments do not
    match."""
    from conftest import load_golden
    g = load_golden("fdir")
    rec = g["rec"]
    fg = rec[:, 0].astype(np.int64) | (rec[:, 1].astype(np.int64) << 8)
    hit = (rec[:, 3] & 0x20) != 0
    assert hit.sum() >= 250
    assert (fg[hit] == 8192 + int(g["fdir_cpu"])).all()
    assert (fg[~hit] < 8192).all()



def test_drop_reasons_confirmed_by_reference():
    """Every drop reason (0x80-0x87, 0x8b-0x8d) is the reference's: the
    harness repairs the field the reason blames and re-runs the reference
    eth_input until it delivers, each repair moving the drop to a strictly
    later check (oracle/ref_harness/harness_main.c confirm_drop; run_ref
    asserts it). Runs where the reference harness is built (this container;
    make -C oracle ref)."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import make_golden as mg
    if not os.path.exists(mg.HARNESS):
        pytest.skip("reference harness not built")
    rng = np.random.default_rng(5)
    frames = mg.edge_frames() + mg.fuzz_frames(rng, 1500)
    rec, _ = mg.run_ref(frames, traces.RSS_KEY, 128, 0, 0)
    reasons = set(rec[:, 2].tolist()) & (set(range(0x80, 0x88)) | {0x8b, 0x8c, 0x8d})
    assert len(reasons) == 11, sorted(hex(r) for r in reasons)  # every eth_input reason exercised
