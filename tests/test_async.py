"""The asynchronous, aggregating host path: IX's <=64-frame
per-iteration batches (dp/core/ethqueue.c:71,117-149) submitted over many
run-loop iterations, records polled back later, in submission order. Every
record is compared bit-exactly with the oracle on the same mbufs."""
import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

pytestmark = pytest.mark.gpu

KEY = traces.RSS_KEY


def _mbufs(kind, n, seed, frames=None):
    if frames is not None:
        tr = traces.pack(frames)
    else:
        tr = traces.make_trace(kind, n, seed=seed, bad_ip=0.02, bad_l4=0.02)
    arena, ptrs = ixgrx.make_mbufs(tr)
    return tr, arena, ptrs


def _run_loop(eng, ptrs, rng, max_batch=64, poll_every=1):
    """An IX-like run loop: each iteration submits the next 1..max_batch frames
    (what eth_process_recv would take), then polls without waiting. Returns
    the polled (mbufs, records) in the order poll gave them."""
    got_m, got_r = [], []
    i, it = 0, 0
    n = len(ptrs)
    while i < n:
        k = int(rng.integers(1, max_batch + 1))
        acc = eng.submit_mbufs(ptrs[i:i + k])
        assert 0 <= acc <= k
        i += acc
        it += 1
        if it % poll_every == 0 or acc < k:
            m, r = eng.poll(4096, wait=acc == 0)
            got_m.append(m)
            got_r.append(r)
    while eng.pending():
        m, r = eng.poll(4096, wait=True)
        got_m.append(m)
        got_r.append(r)
    return np.concatenate(got_m), np.concatenate(got_r)


@pytest.mark.parametrize("kind,cfg", [
    ("imix", dict()),                                            # the defaults
    ("tcp64", dict(batch_frames=1000, depth=2)),                 # uniform lengths: fixed-stride staging
    ("mixed", dict(batch_frames=4096, max_wait_us=0)),           # every submit launches (no aggregation)
    ("imix", dict(batch_frames=64, depth=1)),                    # back-pressure: one batch in the ring
    ("imix", dict(batch_frames=4096, depth=8, direct=False)),    # staged copies (H2D image, D2H records)
    ("tcp64", dict(batch_frames=1000, depth=2, direct=False)),
    ("tcp1514", dict(batch_frames=300, batch_bytes=64 << 10, depth=3)),  # the byte limit closes batches
    ("imix", dict(batch_frames=2048, depth=4, direct=True)),     # kernels on pinned host memory
    ("tcp64", dict(batch_frames=512, depth=4, direct=True)),
])
def test_submit_poll_vs_oracle(kind, cfg):
    rng = np.random.default_rng(hash(kind) % 1000 + len(cfg))
    tr, arena, ptrs = _mbufs(kind, 20000, seed=0x1A5000 + len(cfg))
    eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, 0))
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, **cfg})
        m, r = _run_loop(eng, ptrs, rng)
    finally:
        eng.close()
    assert np.array_equal(m, ptrs), "frames must come back in submission order"
    er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8)
    bad = np.nonzero((r.view(np.uint8).reshape(-1, 16) != er).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} records differ, first {bad[:5]}"


def test_batch_sizes_1_to_64_many_iterations():
    """Every per-iteration batch size 1..64, thousands of iterations, polls
    between them, over the fuzz frames (every edge case of SURVEY 8(a))."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as mg
    rng = np.random.default_rng(64)
    frames = mg.fuzz_frames(rng, 30000) + mg.edge_frames()
    frames = [f for f in frames if len(f) <= 2048]
    tr, arena, ptrs = _mbufs(None, 0, 0, frames=frames)
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP):
        eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, flags))
        try:
            eng.async_init(batch_frames=3000, batch_bytes=1 << 20, max_wait_us=20, depth=4)
            got_m, got_r = [], []
            i, size = 0, 1
            while i < len(ptrs):
                acc = eng.submit_mbufs(ptrs[i:i + size])
                i += acc
                size = size % 64 + 1
                m, r = eng.poll(256, wait=acc == 0)
                got_m.append(m)
                got_r.append(r)
            while eng.pending():
                m, r = eng.poll(256, wait=True)
                got_m.append(m)
                got_r.append(r)
        finally:
            eng.close()
        m, r = np.concatenate(got_m), np.concatenate(got_r)
        assert np.array_equal(m, ptrs)
        er = oracle.rx_mbufs(KEY, 128, 0, flags, ptrs, threads=8)
        bad = np.nonzero((r.view(np.uint8).reshape(-1, 16) != er).any(axis=1))[0]
        assert bad.size == 0, f"flags={flags}: {bad.size} records differ, first {bad[:5]}"


def test_back_pressure_and_flush():
    """With one batch of 64 frames in the ring, a submit of 200 takes 64; the
    rest is taken after a poll. flush launches a partial batch; poll with
    wait returns it; nothing is pending afterwards."""
    tr, arena, ptrs = _mbufs("imix", 500, seed=3)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        eng.async_init(batch_frames=64, batch_bytes=1 << 20, max_wait_us=1000000, depth=1)
        assert eng.submit_mbufs(ptrs[:200]) == 64
        assert eng.pending() == 64
        assert eng.submit_mbufs(ptrs[64:200]) == 0
        m, r = eng.poll(1000, wait=True)
        assert np.array_equal(m, ptrs[:64])
        assert eng.submit_mbufs(ptrs[64:100]) == 36  # a partial batch, not due yet
        m2, _ = eng.poll(1000, wait=False)
        assert m2.size == 0 and eng.pending() == 36
        eng.flush()
        m3, r3 = eng.poll(1000, wait=True)
        assert np.array_equal(m3, ptrs[64:100]) and eng.pending() == 0
        er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs[:100], threads=8)
        allr = np.concatenate([r, r3]).view(np.uint8).reshape(-1, 16)
        assert np.array_equal(allr, er)
        with pytest.raises(RuntimeError, match="ixg_rx_async_init"):
            eng.submit_mbufs(ptrs[:3])
            eng.async_init(batch_frames=10)  # frames pending: -EBUSY
    finally:
        eng.close()


def test_poll_returns_at_most_max():
    tr, arena, ptrs = _mbufs("tcp64", 3000, seed=4)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        eng.async_init(batch_frames=1000, depth=4)
        assert eng.submit_mbufs(ptrs) == 3000
        eng.flush()
        parts = []
        while eng.pending():
            m, r = eng.poll(7, wait=True)
            assert 0 < m.size <= 7
            parts.append(r)
        er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8)
        assert np.array_equal(np.concatenate(parts).view(np.uint8).reshape(-1, 16), er)
    finally:
        eng.close()


def test_sync_mbuf_path_skips_macs():
    """ixg_rx_batch_mbufs stages frames without bytes 0..11: MAC bytes that
    differ per frame cannot change any record (nothing on the path reads
    them), for every layout the staging picks (uniform lengths: fixed
    stride; mixed: offsets)."""
    for kind in ("tcp64", "imix", "mixed"):
        tr, arena, ptrs = _mbufs(kind, 5000, seed=5)
        eng = ixgrx.RxEngine(ixgrx.Config(KEY))
        try:
            r1 = eng.batch_mbufs(ptrs)
            view = arena[(int(ptrs[0]) - arena.ctypes.data):]
            for k in range(len(ptrs)):  # scramble the MACs in place
                o = int(ptrs[k]) - int(ptrs[0]) + 64
                view[o:o + 12] = np.frombuffer(np.random.default_rng(k).bytes(12), np.uint8)
            r2 = eng.batch_mbufs(ptrs)
        finally:
            eng.close()
        er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8)
        assert np.array_equal(r1.view(np.uint8).reshape(-1, 16), er), kind
        assert np.array_equal(r2, r1), kind


def _long_frames(n, seed):
    """Frames of at least 256 B only (every batch goes to the general kernel
    alone, IXG_LF_LONG): the IMIX 590/1514-B frames with bad checksums, cut
    to random lengths >= 256 (ip_len then exceeds L: drops), and frames of
    exactly 256 B."""
    rng = np.random.default_rng(seed)
    tr = traces.make_trace("imix", 4 * n, seed=seed, bad_ip=0.02, bad_l4=0.02)
    big = [tr.frame(i) for i in range(tr.n) if tr.len[i] >= 256][:n]
    out = []
    for f in big:
        r = rng.random()
        if r < 0.1:
            f = f[:int(rng.integers(256, len(f) + 1))]
        elif r < 0.15:
            f = f[:256]
        out.append(f)
    return traces.pack(out)


def _long_mixed_frames(n, seed):
    """Long frames of every header shape: IPv4 ihl 5..15 and IPv6, TCP and
    UDP, 256..1514 B, some with bad checksums, some padded past the IP total
    length (the segment ends before L)."""
    rng = np.random.default_rng(seed)
    rows = []
    for ihl in (5, 6, 9, 15):
        for proto in (6, 17):
            for L in (256, 300, 590, 1514):
                f = traces.build_ipv4(rng, 16, L, proto, ihl=ihl)
                traces.corrupt(rng, f, 0.1, 0.1, 14 + 4 * ihl + (16 if proto == 6 else 6))
                rows += [bytes(x) for x in f]
    for proto in (6, 17):
        for L in (256, 1514):
            rows += [bytes(x) for x in traces.build_ipv6(rng, 16, L, proto)]
    out = []
    for k in rng.integers(0, len(rows), n):
        f = rows[k]
        if rng.random() < 0.1:  # padded: bytes past the IP total length
            f = f + bytes(rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8))
        out.append(f)
    return traces.pack(out)


@pytest.mark.parametrize("register,flags", [(False, 0), (True, 0), (False, ixgrx.IXG_F_IPV6),
                                            (True, ixgrx.IXG_F_IPV6)])
def test_long_only_batches(register, flags):
    """Batches whose frames are all >= IXG_LONG_ONLY_LEN go to the
    host-memory big-frame kernel (DIRECT: a few frames per wave); staged and
    in place, every header shape, records as the oracle's."""
    rng = np.random.default_rng(0x10F + flags)
    tr = _long_frames(6000, 0x10F0) if not flags else _long_mixed_frames(6000, 0x10F1)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, flags))
    try:
        eng.async_init(**ixgrx.ASYNC_DEFAULTS)
        if register:
            eng.register_memory(arena.ctypes.data, arena.nbytes)
        m, r = _run_loop(eng, ptrs, rng)
        if register:
            eng.unregister_memory(arena.ctypes.data)
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    er = oracle.rx_mbufs(KEY, 128, 0, flags, ptrs, threads=8)
    bad = np.nonzero((r.view(np.uint8).reshape(-1, 16) != er).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} records differ, first {bad[:5]}"


@pytest.mark.parametrize("kind", ["tcp64", "imix", "mixed", "tcp1514"])
def test_zero_copy_registered_mbufs(kind):
    """Registered mbuf memory: the kernels read the frames in place over the
    host link (no gather); a third of the frames come from an unregistered
    arena in the same batches (gathered). Records as the oracle's, in
    submission order."""
    rng = np.random.default_rng(77)
    tr, arena, ptrs = _mbufs(kind, 20000, seed=0x1A5100)
    tr2, arena2, ptrs2 = _mbufs("imix", 20000, seed=0x1A5101)
    mix = np.where(rng.random(20000) < 0.67, ptrs, ptrs2)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        eng.async_init(**ixgrx.ASYNC_DEFAULTS)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        for p in (ptrs, mix):
            m, r = _run_loop(eng, p, rng)
            assert np.array_equal(m, p)
            er = oracle.rx_mbufs(KEY, 128, 0, 0, p, threads=8)
            bad = np.nonzero((r.view(np.uint8).reshape(-1, 16) != er).any(axis=1))[0]
            assert bad.size == 0, f"{bad.size} records differ, first {bad[:5]}"
        eng.unregister_memory(arena.ctypes.data)
    finally:
        eng.close()


def _filters_for(tr, pick):
    """FDIR_DTYPE filters matching frames `pick` of tr (IPv4 TCP)."""
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    l4 = offs[pick] + 14 + 4 * (b[offs[pick] + 14] & 15).astype(np.int64)
    f = np.zeros(len(pick), ixgrx.FDIR_DTYPE)
    f["src_ip"] = b[(offs[pick] + 26)[:, None] + np.arange(4)].view("<u4").reshape(-1)
    f["dst_ip"] = b[(offs[pick] + 30)[:, None] + np.arange(4)].view("<u4").reshape(-1)
    f["src_port"] = (b[l4].astype(np.uint16) << 8) | b[l4 + 1]
    f["dst_port"] = (b[l4 + 2].astype(np.uint16) << 8) | b[l4 + 3]
    return f


@pytest.mark.parametrize("kind", ["tcp64", "tcp1514"])
def test_set_fdir_with_batches_in_flight(kind):
    """ixg_rx_set_fdir from IX's connect path while the run loop has batches
    submitted and not yet polled: frames submitted before the call
    get the filters in force when they were submitted, frames after it the
    new ones; every record against the oracle with the matching table.
    (1514-B frames: the host-memory big-frame kernel's flow-director match.)"""
    rng = np.random.default_rng(0x1F0)
    tr, arena, ptrs = _mbufs(kind, 30000 if kind == "tcp64" else 12000, seed=0x1F01)
    offs = tr.offsets().astype(np.int64)
    tcp = np.nonzero(tr.blob[offs + 23] == 6)[0]
    f_old, f_new = _filters_for(tr, tcp[0::5]), _filters_for(tr, tcp[1::5])
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        eng.async_init(batch_frames=4096, max_wait_us=1000000, depth=4, direct=True)
        eng.set_fdir(f_old, cpu_id=4)
        half = len(ptrs) // 2
        got_m, got_r = [], []
        i = 0
        while i < half:  # submitted, mostly not polled: batches open and in flight
            acc = eng.submit_mbufs(ptrs[i:min(i + 64, half)])
            if acc == 0:
                m, r = eng.poll(4096, wait=True)
                got_m.append(m)
                got_r.append(r)
            i += acc
        assert eng.pending() > 0
        eng.set_fdir(f_new, cpu_id=4)  # the connect path, mid-stream
        while i < len(ptrs):
            acc = eng.submit_mbufs(ptrs[i:i + 64])
            if acc == 0:
                m, r = eng.poll(4096, wait=True)
                got_m.append(m)
                got_r.append(r)
            i += acc
        while eng.pending():
            m, r = eng.poll(4096, wait=True)
            got_m.append(m)
            got_r.append(r)
        m, r = np.concatenate(got_m), np.concatenate(got_r)
        assert np.array_equal(m, ptrs)
        rr = r.view(np.uint8).reshape(-1, 16)
        # (mbuf k holds frame k of tr)
        e_old = oracle.rx_trace(tr, KEY, threads=8, fdir=f_old, cpu_id=4)[0][:half]
        e_new = oracle.rx_trace(tr, KEY, threads=8, fdir=f_new, cpu_id=4)[0][half:]
        assert np.array_equal(rr[:half], e_old), "frames submitted before set_fdir"
        assert np.array_equal(rr[half:], e_new), "frames submitted after set_fdir"
        assert ((e_old[:, 3] & 0x20) != 0).sum() > 1000 and ((e_new[:, 3] & 0x20) != 0).sum() > 1000
    finally:
        eng.set_fdir(None)
        eng.close()


def _garbage_past_ip_len(kind, n, seed):
    """Frames whose bytes past the IP total length are random (C2's pad
    filled; other IPv4 frames cut short of the frame at random), so a kernel
    that read the not-staged bytes (ixg_stage_ext) would see the next frame's
    bytes there."""
    rng = np.random.default_rng(seed)
    tr = traces.make_trace(kind, n, seed=seed, bad_ip=0.02, bad_l4=0.02)
    frames = []
    for o, L in zip(tr.offsets().astype(np.int64), tr.len.astype(np.int64)):
        f = bytearray(tr.blob[o:o + L].tobytes())
        if L >= 34 and f[12:14] == b"\x08\x00" and f[14] >> 4 == 4:
            ip_len = int.from_bytes(f[16:18], "big")
            if kind != "tcp64" and rng.random() < 0.5:
                cut = int(rng.integers(0, max(1, min(ip_len, L - 14) - 20)))
                ip_len -= cut
                f[16:18] = ip_len.to_bytes(2, "big")
            if 14 + ip_len < L:
                f[14 + ip_len:] = rng.integers(0, 256, L - 14 - ip_len, dtype=np.uint8).tobytes()
        frames.append(bytes(f))
    return frames


@pytest.mark.parametrize("kind,cfg", [
    ("tcp64", dict(batch_frames=4096, depth=2)),               # fixed stride 44: the 6-B pads not staged
    ("tcp64", dict(batch_frames=4096, depth=2, direct=False)),
    ("imix", dict(batch_frames=2048, depth=4)),
    ("mixed", dict(batch_frames=2048, depth=4)),
])
def test_not_staged_bytes_are_not_read(kind, cfg):
    """the gather stages an IPv4 frame's bytes only up to
    max(14 + ip_len, l4 + 20); the kernels, reading the image, see the next
    frame's bytes in the rest and must give the oracle's records of the whole
    frames."""
    frames = _garbage_past_ip_len(kind, 30000, 71)
    tr, arena, ptrs = _mbufs(None, 0, 0, frames=frames)
    exp = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        rec = eng.batch_mbufs(ptrs)
        assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), exp)
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, **cfg})
        m, r = _run_loop(eng, ptrs, np.random.default_rng(72))
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), exp)


@pytest.mark.parametrize("direct", [True, False])
def test_worst_batch_split(direct):
    """ixg_rx_async_stats splits the worst batch's time
    into open (gather -> launch), gpu (launch -> the completion stamp ran, by
    the device's wall clock calibrated at async_init), visible (stamp -> the
    library saw the word) and returned (seen -> last frame polled); the parts
    add up to the total, and a batch that ran on the device has a device
    part. Records still against the oracle."""
    tr, arena, ptrs = _mbufs("imix", 20000, seed=0x5B1)
    rng = np.random.default_rng(0x5B1)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "direct": direct})
        eng.async_stats(reset=True)
        m, r = _run_loop(eng, ptrs, rng)
        st = eng.async_stats()
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8))
    parts = st["worst_open_ns"] + st["worst_gpu_ns"] + st["worst_visible_ns"] + st["worst_returned_ns"]
    assert st["worst_total_ns"] > 0 and parts == st["worst_total_ns"], st
    assert st["worst_gpu_ns"] > 0, st          # the device clock was read and calibrated
    assert st["worst_wait_ns"] <= st["worst_total_ns"]
    assert st["worst_nap_max_ns"] <= st["worst_wait_ns"] and (st["worst_naps"] == 0) == (st["worst_nap_max_ns"] == 0)
