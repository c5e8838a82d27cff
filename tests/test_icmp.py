"""ICMP echo reflect (dp/net/icmp.c:44-71,88-91; VERDICT r3 Next #9).

icmp_input turns an echo request into a reply in its own mbuf: type 0,
Ethernet and IP addresses swapped with CFG.mac / CFG.host_addr as the new
source, the ICMP checksum recomputed over the message (the IP checksum is
left as it was). tests/golden/icmp.npz holds frames before and after the
reference's own eth_input with icmp_reflect's CFG set (two host addresses:
the frames' destination, and another, which leaves the IP checksum stale as
the reference does). The oracle (ixgo_icmp_reflect_batch) is pinned to it;
the device kernel (ixg_icmp_reflect_dev) is checked against both, bit-exact,
on the golden frames and on large fuzzed batches.
"""
import os

import numpy as np
import pytest

from ix_amd import icmp, ixgrx, traces
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(HERE, "golden", "icmp.npz")))


def _rec(g):
    return g["rec"].view(ixgrx.REC_DTYPE).reshape(-1)


def test_golden_reflects_echo_requests(golden):
    g = golden
    v = _rec(g)["verdict"]
    assert (g["reflected"] == (v == ixgrx.V["ICMP_ECHO"])).all()
    assert 50 < int(g["reflected"].sum()) < len(v)


@pytest.mark.parametrize("which", ["", "2"])
def test_oracle_matches_reference_golden(golden, which):
    g = golden
    out, k = oracle.icmp_reflect_batch(g["blob"], g["off"], 0, g["rec"], bytes(g["mac"]), int(g["host_addr" + which]))
    assert k == int(g["reflected"].sum())
    assert np.array_equal(out, g["after" + which])


def test_oracle_records_match_golden(golden):
    g = golden
    er, _ = oracle.rx_batch(bytes(g["key"]), 128, 0, 0, g["blob"], g["off"], g["len"])
    assert np.array_equal(er, g["rec"])


def _dev_reflect(eng, blob, off, stride, rec, n, mac, host):
    import torch
    dev = torch.device("cuda", 0)
    b = torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
    o = None if off is None else torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).to(dev)
    r = torch.from_numpy(np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)).to(dev)
    icmp.reflect_dev(eng, b.data_ptr(), None if o is None else o.data_ptr(), stride, r.data_ptr(), n, mac, host)
    torch.cuda.synchronize()
    return b.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["", "2"])
def test_gpu_golden(golden, which):
    g = golden
    eng = ixgrx.RxEngine(ixgrx.Config(bytes(g["key"])))
    try:
        blob = np.concatenate([g["blob"], np.zeros(ixgrx.IXG_TAIL_PAD, np.uint8)])
        out = _dev_reflect(eng, blob, g["off"], 0, g["rec"], len(g["len"]), bytes(g["mac"]),
                           int(g["host_addr" + which]))
        assert np.array_equal(out[:g["blob"].size], g["after" + which])
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["offsets", "unaligned", "stride"])
def test_gpu_fuzz_vs_oracle(layout):
    """Large batches: echo requests of every length up to the largest mbuf
    frame among other traffic, records from the device RX path, reflected
    frames bit-exact against the oracle."""
    rng = np.random.default_rng(0x1C3)
    n = 40000
    lens = rng.integers(0, 2048 - 42 + 1, n)
    frames = []
    kinds = rng.random(n)
    for i in range(n):
        if kinds[i] < 0.6:
            pl = int(lens[i]) if layout == "offsets" else int(lens[i]) % 80
            f = traces.icmp_echo(rng, pl)
        elif kinds[i] < 0.8:
            f = bytes(traces.build_ipv4(rng, 1, 60 if layout == "stride" else 590, 6)[0])
        else:
            f = bytearray(traces.icmp_echo(rng, int(lens[i]) % 100))
            f[int(rng.integers(34, len(f)))] ^= 0x20  # bad checksum: not reflected
            f = bytes(f)
        frames.append(f)
    tr = traces.pack(frames, stride=128) if layout == "stride" else traces.pack(frames, align=1 if layout == "unaligned" else 4)
    if layout == "unaligned":
        assert len(set((tr.off % 4).tolist())) == 4  # messages start at every byte phase
    key = traces.RSS_KEY
    er, _ = oracle.rx_trace(tr, key)
    mac, host = bytes([2, 3, 5, 7, 11, 13]), 0x0a0b0c0d
    exp, k = oracle.icmp_reflect_batch(tr.blob, tr.off, tr.stride or 0, er, mac, host)
    assert k > n // 3
    eng = ixgrx.RxEngine(ixgrx.Config(key))
    try:
        out = _dev_reflect(eng, tr.blob, tr.off, tr.stride or 0, er, n, mac, host)
        bad = np.nonzero(out != exp)[0]
        assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_reflect_rejects_bad_arguments():
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY))
    try:
        with pytest.raises(RuntimeError, match="ixg_icmp_reflect_dev"):
            icmp.reflect_dev(eng, 0, None, 64, 16, 1, bytes(6), 0)  # no frames
        with pytest.raises(RuntimeError, match="ixg_icmp_reflect_dev"):
            icmp.reflect_dev(eng, 64, None, 64, 12, 1, bytes(6), 0)  # records not 8-aligned
        icmp.reflect_dev(eng, 0, None, 64, 0, 0, bytes(6), 0)  # nothing to do
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_ping_flood():
    """A batch of nothing but default-size pings (56-byte payload, 64-byte
    messages: each lane rewrites its own) and one of 1400-byte pings (the
    wave takes them one at a time), bit-exact against the oracle."""
    rng = np.random.default_rng(0x1C4)
    key = traces.RSS_KEY
    mac, host = bytes([2, 9, 8, 7, 6, 5]), 0xc0a80001
    eng = ixgrx.RxEngine(ixgrx.Config(key))
    try:
        for pl, n in ((56, 1 << 17), (1400, 1 << 13)):
            pool = [traces.icmp_echo(rng, pl) for _ in range(512)]
            tr = traces.pack(pool * (n // 512))
            er, _ = oracle.rx_trace(tr, key)
            assert (er[:, 2] == ixgrx.V["ICMP_ECHO"]).all()
            exp, k = oracle.icmp_reflect_batch(tr.blob, tr.off, 0, er, mac, host)
            assert k == n
            out = _dev_reflect(eng, tr.blob, tr.off, 0, er, n, mac, host)
            assert np.array_equal(out, exp), f"payload {pl}"
    finally:
        eng.close()
