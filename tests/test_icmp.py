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


def _async_loop(eng, ptrs, rng, max_batch=64):
    got_m, got_r = [], []
    i = 0
    while i < len(ptrs):
        k = int(rng.integers(1, max_batch + 1))
        acc = eng.submit_mbufs(ptrs[i:i + k])
        i += acc
        m, r = eng.poll(4096, wait=acc == 0)
        got_m.append(m)
        got_r.append(r)
    while eng.pending():
        m, r = eng.poll(4096, wait=True)
        got_m.append(m)
        got_r.append(r)
    return np.concatenate(got_m), np.concatenate(got_r)


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("which", ["", "2"])
def test_gpu_async_reflect_golden(golden, which, direct):
    """the asynchronous path with IXG_ASYNC_ICMP_REFLECT
    and the mbuf pool registered returns the reference's echo replies
    (icmp.npz, written by the reference's own icmp_input) already built in
    the mbufs, with IXG_RF_REPLY in their records; other frames and records
    as the reference's."""
    g = golden
    tr = traces.Trace(blob=g["blob"].copy(), off=g["off"], len=g["len"], stride=0)
    arena, ptrs = ixgrx.make_mbufs(tr)
    refl = g["reflected"].astype(bool)
    eng = ixgrx.RxEngine(ixgrx.Config(bytes(g["key"])))
    try:
        eng.async_init(batch_frames=48, batch_bytes=1 << 20, max_wait_us=10000000, depth=3, direct=direct,
                       icmp_reflect=True)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        eng.set_icmp_reply(bytes(g["mac"]), int(g["host_addr" + which]))
        m, r = _async_loop(eng, ptrs, np.random.default_rng(8), max_batch=16)
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    want = g["rec"].copy()
    want[refl, 3] |= ixgrx.RF_REPLY
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), want)
    base = arena.ctypes.data
    after = g["after" + which]
    for i, (p, o, L) in enumerate(zip(ptrs.astype(np.int64), g["off"].astype(np.int64), g["len"].astype(np.int64))):
        assert np.array_equal(arena[p - base + 64:p - base + 64 + L], after[o:o + L]), i


@pytest.mark.gpu
@pytest.mark.parametrize("long_only", [False, True])
def test_gpu_async_reflect_fuzz_vs_oracle(long_only):
    """40K mixed frames (echo requests of every size up to 2 KiB, bad-checksum
    requests, TCP) through submit/poll with IXG_ASYNC_ICMP_REFLECT; a third
    of the mbufs come from an unregistered arena (left to the host's
    icmp_reflect). Mbuf contents and records against the oracle. long_only:
    20K frames of at least 256 B (the batches take the host-memory
    big-frame kernel, then the reflect)."""
    rng = np.random.default_rng(0x1C5 + long_only)
    n = 20000 if long_only else 40000
    lo = 256 - 42 if long_only else 0
    frames = []
    for i in range(n):
        u = rng.random()
        if u < 0.5:
            frames.append(traces.icmp_echo(rng, int(rng.integers(lo, 2048 - 42 + 1))))
        elif u < 0.7:
            f = bytearray(traces.icmp_echo(rng, int(rng.integers(lo, lo + 100))))
            f[int(rng.integers(34, len(f)))] ^= 0x20
            frames.append(bytes(f))
        else:
            sizes = [590, 1514] if long_only else [60, 590, 1514]
            frames.append(bytes(traces.build_ipv4(rng, 1, int(rng.choice(sizes)), 6)[0]))
    tr = traces.pack(frames)
    arena, ptrs = ixgrx.make_mbufs(tr)
    tr2 = traces.pack(frames)
    arena2, ptrs2 = ixgrx.make_mbufs(tr2)
    use2 = rng.random(n) < 0.33
    mix = np.where(use2, ptrs2, ptrs)
    key, mac, host = traces.RSS_KEY, bytes([2, 3, 5, 7, 11, 13]), 0x0a0b0c0d
    er, _ = oracle.rx_trace(tr, key)
    exp_frames, _ = oracle.icmp_reflect_batch(tr.blob, tr.off, 0, er, mac, host)
    eng = ixgrx.RxEngine(ixgrx.Config(key))
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "icmp_reflect": True})
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        eng.set_icmp_reply(mac, host)
        m, r = _async_loop(eng, mix, rng)
    finally:
        eng.close()
    assert np.array_equal(m, mix)
    echo = er[:, 2] == ixgrx.V["ICMP_ECHO"]
    want = er.copy()
    want[echo & ~use2, 3] |= ixgrx.RF_REPLY
    got = r.view(np.uint8).reshape(-1, 16)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} records differ, first {bad[:5]}"
    offs, lens = tr.off.astype(np.int64), tr.len.astype(np.int64)
    b1, b2 = arena.ctypes.data, arena2.ctypes.data
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        p = int(ptrs[i]) - b1 + 64
        want_f = tr.blob[o:o + L] if use2[i] else exp_frames[o:o + L]
        assert np.array_equal(arena[p:p + L], want_f), i
        p2 = int(ptrs2[i]) - b2 + 64
        assert np.array_equal(arena2[p2:p2 + L], tr2.blob[o:o + L]), i   # unregistered: untouched


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["packed", "unaligned", "stride", "gaps", "interleaved"])
def test_gpu_flood_span_path(layout):
    """Waves whose 64 items are all small echo requests in increasing,
    non-overlapping order take the span path (the wave's frames staged in LDS
    and stored back whole): every byte of the buffer, gaps and the bytes
    around each wave's span included, against the oracle; message lengths
    8..128 bytes, a partial last wave, spans at every 16-byte phase.
    interleaved: packed small pings whose offset array deals
    each run of 128 frames out to two waves, even frames to one and odd to
    the other, so each wave's gaps hold the other wave's frames, which it
    rewrites at the same time: no wave may store its gaps back."""
    rng = np.random.default_rng(0x1C6)
    key = traces.RSS_KEY
    mac, host = bytes([2, 4, 6, 8, 10, 12]), 0x0a000001
    n = 64 * 200 + 37
    frames = [traces.icmp_echo(rng, int(rng.integers(0, 21 if layout == "interleaved" else 121))) for _ in range(n)]
    if layout == "interleaved":
        tr = traces.pack(frames)
        perm = np.arange(n)
        m = n - n % 128
        perm[:m] = perm[:m].reshape(-1, 64, 2).transpose(0, 2, 1).reshape(-1)
        frames = [frames[j] for j in perm]
        tr = traces.Trace(blob=tr.blob, off=tr.off[perm].copy(), len=tr.len[perm].copy(), stride=0)
    elif layout == "stride":
        tr = traces.pack(frames, stride=192)
    elif layout == "gaps":
        # random 0..40-byte gaps of random bytes between the frames
        gaps = rng.integers(0, 41, n)
        off = np.zeros(n, np.uint64)
        pos = 8
        for i, f in enumerate(frames):
            pos += int(gaps[i])
            off[i] = pos
            pos += len(f)
        blob = rng.integers(0, 256, pos + 256, dtype=np.uint8)
        for i, f in enumerate(frames):
            blob[int(off[i]):int(off[i]) + len(f)] = np.frombuffer(f, np.uint8)
        tr = traces.Trace(blob=blob, off=off, len=np.array([len(f) for f in frames], np.uint16), stride=0)
    else:
        tr = traces.pack(frames, align=1 if layout == "unaligned" else 4)
    er, _ = oracle.rx_trace(tr, key)
    assert (er[:, 2] == ixgrx.V["ICMP_ECHO"]).all()
    exp, k = oracle.icmp_reflect_batch(tr.blob, tr.off, tr.stride or 0, er, mac, host)
    assert k == n
    eng = ixgrx.RxEngine(ixgrx.Config(key))
    try:
        out = _dev_reflect(eng, tr.blob, tr.off, tr.stride or 0, er, n, mac, host)
    finally:
        eng.close()
    bad = np.nonzero(out != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


# ---- ixg_rx_icmp_batch_dev: RX records and the replies in one call -------------

def _dev_rx_icmp(eng, tr, mac, host):
    import torch
    dev = torch.device("cuda", 0)
    n = tr.n
    b = torch.from_numpy(np.concatenate([np.ascontiguousarray(tr.blob, dtype=np.uint8),
                                         np.zeros(ixgrx.IXG_TAIL_PAD, np.uint8)])).to(dev)
    o = None if tr.off is None or tr.stride else \
        torch.from_numpy(np.ascontiguousarray(tr.off, dtype=np.uint64).view(np.int64)).to(dev)
    ln = torch.from_numpy(np.ascontiguousarray(tr.len, dtype=np.uint16).view(np.int16)).to(dev)
    rec = torch.full((n, 16), 0x5A, dtype=torch.uint8, device=dev)
    icmp.rx_batch_dev(eng, b.data_ptr(), None if o is None else o.data_ptr(), ln.data_ptr(), tr.stride or 0, n,
                      rec.data_ptr(), mac, host)
    torch.cuda.synchronize()
    return rec.cpu().numpy(), b.cpu().numpy()[:tr.blob.size]


def _fused_expect(tr, key, mac, host):
    er, _ = oracle.rx_trace(tr, key)
    exp, k = oracle.icmp_reflect_batch(tr.blob, tr.off, tr.stride or 0, er, mac, host)
    er = er.copy()
    echo = er[:, 2] == ixgrx.V["ICMP_ECHO"]
    er[echo, 3] |= 0x40  # IXG_RF_REPLY
    return er, exp, int(k)


def _check_fused(tr, key, mac, host):
    er, exp, k = _fused_expect(tr, key, mac, host)
    eng = ixgrx.RxEngine(ixgrx.Config(key))
    try:
        rec, out = _dev_rx_icmp(eng, tr, mac, host)
    finally:
        eng.close()
    badr = np.nonzero((rec != er).any(axis=1))[0]
    assert badr.size == 0, f"{badr.size} records differ, first {badr[:6].tolist()}: {rec[badr[0]].tolist()} vs " \
                           f"{er[badr[0]].tolist()}"
    bad = np.nonzero(out != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    return k


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["", "2"])
def test_gpu_rx_icmp_golden(golden, which):
    """The reference's frames (echo requests among every other ICMP and
    non-ICMP case of the fixture) through ixg_rx_icmp_batch_dev: records as
    the reference's with IXG_RF_REPLY on the echo requests, frames as the
    reference's icmp_input left them."""
    g = golden
    off = g["off"].astype(np.uint64)
    frames = [g["blob"][int(o):int(o) + int(L)].tobytes() for o, L in zip(off, g["len"])]
    tr = traces.pack(frames)  # 4-aligned starts (the ABI's requirement)
    k = _check_fused(tr, bytes(g["key"]), bytes(g["mac"]), int(g["host_addr" + which]))
    assert k == int(g["reflected"].sum())


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["offsets", "stride"])
def test_gpu_rx_icmp_mixed_vs_oracle(layout):
    """Default-size pings, long pings, pings with IP options, pings with bad
    checksums, TCP frames, and chunks of 1514-B frames (the long kernel's,
    with pings among them): records (IXG_RF_REPLY on every answered request)
    and every byte against the oracle."""
    rng = np.random.default_rng(0x1C9 + (layout == "stride"))
    frames = []
    for c in range(300):
        big = c % 10 == 3 and layout == "offsets"
        for _ in range(64):
            u = rng.random()
            if big and u < 0.5:
                frames.append(bytes(traces.build_ipv4(rng, 1, 1514, 6)[0]))
            elif u < 0.55:
                frames.append(traces.icmp_echo(rng, int(rng.integers(0, 55 if layout == "stride" else 71))))
            elif u < 0.65:
                frames.append(traces.icmp_echo(rng, int(rng.integers(40, 55)) if layout == "stride"
                                               else int(rng.integers(71, 1400))))
            elif u < 0.72:
                frames.append(traces.icmp_echo(rng, int(rng.integers(0, 60)), ihl=6))
            elif u < 0.8:
                f = bytearray(traces.icmp_echo(rng, int(rng.integers(0, 60))))
                f[int(rng.integers(34, len(f)))] ^= 0x10
                frames.append(bytes(f))
            else:
                frames.append(bytes(traces.build_ipv4(rng, 1, 60, 6)[0]))
    # (stride 96: chunks span-staged, as packed ones)
    tr = traces.pack(frames, stride=96) if layout == "stride" else traces.pack(frames)
    k = _check_fused(tr, traces.RSS_KEY, bytes([2, 3, 5, 7, 11, 13]), 0x0a0b0c0d)
    assert k > len(frames) // 3


@pytest.mark.gpu
def test_gpu_rx_icmp_ping_flood():
    """A flood of default pings (the reflect pass's span path, which marks
    its records too) and a ragged batch end."""
    rng = np.random.default_rng(0x1CB)
    pool = [traces.icmp_echo(rng, 56) for _ in range(512)]
    tr = traces.pack(pool * 256 + pool[:77])
    k = _check_fused(tr, traces.RSS_KEY, bytes([2, 9, 8, 7, 6, 5]), 0xc0a80001)
    assert k == tr.n
