"""The host paths' own logic on the CPU (no GPU): the C host library
(ixgrx_host.c, ixgrx_async.c) linked with tests/fakehip/fakehip.c, a CPU
stand-in for the HIP runtime whose streams defer every copy and launch until
someone synchronizes, and whose RX launch runs the oracle. What this covers:
the MAC-skipping gather, the staged image (fixed-stride and offset layouts),
the asynchronous ring (open / in flight / done, back-pressure, flush,
ordering) and the synchronous pipelined path; any read of results before
synchronizing, or reuse of a buffer whose copy has not run, shows up as
wrong records. tests/test_sanitize.py re-runs this file against the
ASan/UBSan build. The kernels themselves are the -m gpu tests' business."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "build", "fakehip", "libixgrx_fake.so")
KEY = traces.RSS_KEY


@pytest.fixture(scope="module")
def fake():
    path = os.environ.get("IXG_FAKE_LIB")
    if not path:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "fakehip")], check=True)
        path = FAKE
    lib = ixgrx.load_library(path)
    lib.fakehip_set_cfg.argtypes = [ctypes.POINTER(ixgrx.RxCfg)]
    lib.fakehip_launches.restype = ctypes.c_ulong

    def engine(flags=0, nb=128, dev=0):
        cfg = ixgrx.Config(KEY, nb, dev, flags)
        c = cfg.to_c()
        lib.fakehip_set_cfg(ctypes.byref(c))
        return ixgrx.RxEngine(cfg, lib_path=path)
    engine.lib = lib
    return engine


def _mbufs(kind, n, seed):
    tr = traces.make_trace(kind, n, seed=seed, bad_ip=0.02, bad_l4=0.02)
    arena, ptrs = ixgrx.make_mbufs(tr)
    return tr, arena, ptrs


def _expect(ptrs, flags=0):
    return oracle.rx_mbufs(KEY, 128, 0, flags, ptrs, threads=8)


@pytest.mark.parametrize("kind", ["tcp64", "imix", "mixed", "tcp1514"])
def test_sync_mbufs(fake, kind):
    tr, arena, ptrs = _mbufs(kind, 3000, seed=7)
    eng = fake()
    try:
        rec = eng.batch_mbufs(ptrs)
    finally:
        eng.close()
    assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), _expect(ptrs))


def test_sync_mbufs_pipelined(fake):
    """More frames than one pipeline chunk (131072): both stages, in turn."""
    tr, arena, ptrs = _mbufs("tcp64", 300000, seed=8)
    eng = fake()
    try:
        rec = eng.batch_mbufs(ptrs)
        rec2 = eng.batch_mbufs(ptrs[:1000])
    finally:
        eng.close()
    exp = _expect(ptrs)
    assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), exp)
    assert np.array_equal(rec2.view(np.uint8).reshape(-1, 16), exp[:1000])


def test_tiny_frames(fake):
    """Frames of 0..13 bytes (nothing or one byte past the MACs staged), in
    a batch of one length (fixed-stride staging) and mixed."""
    rng = np.random.default_rng(3)
    # runs where every frame but the last stages nothing (<= 12 B)
    # have all offsets 0; they are not a fixed-stride run
    for lens in ([5] * 300, list(rng.integers(0, 14, 500)), [12] * 70, [13] * 65, [10, 10, 60], [5] * 63 + [60],
                 [12] * 64 + [64], [0, 60]):
        frames = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in lens]
        tr = traces.pack(frames)
        arena, ptrs = ixgrx.make_mbufs(tr)
        eng = fake()
        try:
            rec = eng.batch_mbufs(ptrs)
        finally:
            eng.close()
        assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), _expect(ptrs))


def _loop(eng, ptrs, rng, max_batch=64):
    got_m, got_r = [], []
    i = 0
    while i < len(ptrs):
        k = int(rng.integers(1, max_batch + 1))
        acc = eng.submit_mbufs(ptrs[i:i + k])
        assert 0 <= acc <= k
        i += acc
        m, r = eng.poll(1000, wait=acc == 0)
        got_m.append(m)
        got_r.append(r)
    while eng.pending():
        m, r = eng.poll(1000, wait=True)
        got_m.append(m)
        got_r.append(r)
    return np.concatenate(got_m), np.concatenate(got_r)


@pytest.mark.parametrize("kind,cfg", [
    ("imix", dict()),
    ("tcp64", dict(batch_frames=1000, depth=2)),
    ("mixed", dict(batch_frames=4096, max_wait_us=0)),
    ("imix", dict(batch_frames=64, depth=1)),
    ("imix", dict(batch_frames=4096, depth=8, direct=False)),     # staged copies (H2D image, D2H records)
    ("tcp64", dict(batch_frames=1000, depth=2, direct=False)),
    ("tcp1514", dict(batch_frames=300, batch_bytes=64 << 10, depth=3)),
    ("imix", dict(batch_frames=4096, batch_bytes=4096, depth=16)),
    ("tcp64", dict(batch_frames=100, depth=4, direct=True)),
])
def test_async_submit_poll(fake, kind, cfg):
    rng = np.random.default_rng(len(cfg) + len(kind))
    tr, arena, ptrs = _mbufs(kind, 12000, seed=9)
    eng = fake()
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, **cfg})
        m, r = _loop(eng, ptrs, rng)
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))


def test_async_uniform_length_runs(fake):
    """Fixed-stride runs of one length send no lengths (the kernels read the
    length from device memory, refilled on the batch's stream when it
    changes): batches of 64 equal frames whose length changes from batch to
    batch, a ring of 3 batches in flight, every record against the oracle;
    the staged image is 44 B per 60-B frame."""
    rng = np.random.default_rng(0x1E)
    seq = [60, 62, 60, 100, 100, 58, 60, 61, 1514, 60]
    frames = []
    for L in seq * 4:
        tr = traces.make_trace("tcp64", 64, seed=int(rng.integers(1 << 30)), bad_ip=0.05, bad_l4=0.05)
        for i in range(64):
            f = tr.frame(i)
            frames.append(f[:L] if L <= len(f) else f + bytes(rng.integers(0, 256, L - len(f), dtype=np.uint8)))
    arena, ptrs = ixgrx.make_mbufs(traces.pack(frames))
    eng = fake()
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "batch_frames": 64, "depth": 3})
        got_m, got_r = [], []
        for b in range(0, len(ptrs), 64):
            while eng.submit_mbufs(ptrs[b:b + 64]) != 64:
                m, r = eng.poll(1000, wait=True)
                got_m.append(m)
                got_r.append(r)
        while eng.pending():
            m, r = eng.poll(1000, wait=True)
            got_m.append(m)
            got_r.append(r)
        st = eng.async_stats()
    finally:
        eng.close()
    assert np.array_equal(np.concatenate(got_m), ptrs)
    assert np.array_equal(np.concatenate(got_r).view(np.uint8).reshape(-1, 16), _expect(ptrs))
    assert st["frames_launched"] == len(ptrs) and st["inplace_bytes"] == 0
    # C2's 60-B frames alone: [12, 56) staged, nothing else per frame
    tr = traces.make_trace("tcp64", 4096, seed=0x1E1)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng = fake()
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "batch_frames": 4096, "max_wait_us": 1000000})
        _loop(eng, ptrs, rng)
        st = eng.async_stats()
    finally:
        eng.close()
    assert 44.0 <= st["image_bytes"] / st["frames_launched"] < 44.5, st


@pytest.mark.parametrize("direct", [True, False])
def test_async_one_completion_stamp_per_batch(fake, direct):
    """Every launched batch gets exactly one completion stamp, after its
    kernels (and, in copy mode, the records' D2H copy). Records as the
    oracle's."""
    lib = fake.lib
    lib.fakehip_stamps.restype = ctypes.c_ulong
    rng = np.random.default_rng(0x57)
    for kind in ("tcp64", "imix", "tcp1514"):
        tr, arena, ptrs = _mbufs(kind, 3000, seed=0x570)
        eng = fake()
        s0 = lib.fakehip_stamps()
        try:
            eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "batch_frames": 512, "direct": direct})
            m, r = _loop(eng, ptrs, rng)
            st = eng.async_stats()
        finally:
            eng.close()
        assert np.array_equal(m, ptrs)
        assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))
        assert lib.fakehip_stamps() - s0 == st["batches"], kind


@pytest.mark.parametrize("kind,direct,want", [
    ("tcp1514", True, (1, 1, 0)),    # long frames in host memory: the big-frame kernel alone
    ("tcp1514", False, (0, 1, 0)),   # long frames copied to the device: the general kernel alone
    ("imix", True, (1, 0, 1)),       # short frames present: the span kernel samples and defers
    ("tcp64", True, (1, 0, 1)),
])
def test_async_launch_plan(fake, kind, direct, want):
    """What the host tells the kernels about a batch (ixgrx_launch picks the
    kernels from it): host memory, every frame >= IXG_LONG_ONLY_LEN, and
    whether the deferral machinery is in use. Records as the oracle's."""
    lib = fake.lib
    rng = np.random.default_rng(0x5A)
    tr, arena, ptrs = _mbufs(kind, 2000, seed=0x5A0)
    eng = fake()
    try:
        eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, "batch_frames": 512, "direct": direct})
        m, r = _loop(eng, ptrs, rng)
        hm, lo, df = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        lib.fakehip_last_plan(ctypes.byref(hm), ctypes.byref(lo), ctypes.byref(df))
    finally:
        eng.close()
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))
    assert (hm.value, lo.value, df.value) == want


def test_async_aggregates_iterations(fake):
    """64-frame submissions are aggregated: 100 iterations of 64 frames with
    batch_frames 1600 make 4 launches, not 100."""
    tr, arena, ptrs = _mbufs("tcp64", 6400, seed=10)
    eng = fake()
    try:
        eng.async_init(batch_frames=1600, batch_bytes=1 << 24, max_wait_us=10000000, depth=8)
        n0 = fake.lib.fakehip_launches()
        for k in range(100):
            assert eng.submit_mbufs(ptrs[64 * k:64 * k + 64]) == 64
        m, r = eng.poll(10000, wait=True)
        while eng.pending():
            m2, r2 = eng.poll(10000, wait=True)
            m, r = np.concatenate([m, m2]), np.concatenate([r, r2])
        assert fake.lib.fakehip_launches() - n0 == 4
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))


@pytest.mark.parametrize("direct", [True, False])
def test_launches_never_free(fake, direct):
    """hipFree waits for the whole device, i.e. for every other thread's
    batches: batches growing from 1 frame to batch_frames, and synchronous
    calls up to a pipeline chunk, must not free (grow) a device buffer."""
    fake.lib.fakehip_frees.restype = ctypes.c_ulong
    tr, arena, ptrs = _mbufs("tcp64", 140000, seed=12)
    eng = fake()
    try:
        eng.async_init(batch_frames=4096, batch_bytes=1 << 22, max_wait_us=10000000, depth=2, direct=direct)
        f0 = fake.lib.fakehip_frees()
        i = 0
        for k in (1, 65, 700, 4096):
            assert eng.submit_mbufs(ptrs[i:i + k]) == k
            eng.flush()
            m, r = eng.poll(k, wait=True)
            assert np.array_equal(m, ptrs[i:i + k])
            i += k
        for k in (1, 2000, 131072):
            eng.batch_mbufs(ptrs[:k])
        assert fake.lib.fakehip_frees() == f0
    finally:
        eng.close()


def test_async_back_pressure_flush_and_busy(fake):
    tr, arena, ptrs = _mbufs("imix", 400, seed=11)
    eng = fake()
    try:
        eng.async_init(batch_frames=64, batch_bytes=1 << 20, max_wait_us=10000000, depth=1)
        assert eng.submit_mbufs(ptrs[:200]) == 64
        assert eng.submit_mbufs(ptrs[64:200]) == 0
        assert eng.pending() == 64
        m, r = eng.poll(1000, wait=False)  # not ready on the first look
        assert m.size == 0
        m, r = eng.poll(1000, wait=True)
        assert np.array_equal(m, ptrs[:64])
        assert eng.submit_mbufs(ptrs[64:100]) == 36
        assert eng.poll(1000)[0].size == 0 and eng.pending() == 36
        with pytest.raises(RuntimeError, match="ixg_rx_async_init"):
            eng.async_init(batch_frames=10)
        eng.flush()
        m3, r3 = eng.poll(1000, wait=True)
        assert np.array_equal(m3, ptrs[64:100]) and eng.pending() == 0
        eng.async_init(batch_frames=10, depth=2)  # nothing pending: re-configure
        assert eng.submit_mbufs(ptrs[100:125]) == 20  # two batches of 10, then back-pressure
    finally:
        eng.close()
    exp = _expect(ptrs[:100])
    assert np.array_equal(np.concatenate([r, r3]).view(np.uint8).reshape(-1, 16), exp)


def test_async_rejects_oversized_and_bad_cfg(fake):
    tr, arena, ptrs = _mbufs("tcp64", 10, seed=12)
    arena[(int(ptrs[3]) - arena.ctypes.data):][:8] = np.frombuffer(np.uint64(2049).tobytes(), np.uint8)
    eng = fake()
    try:
        with pytest.raises(RuntimeError, match="ixg_rx_submit_mbufs"):
            eng.submit_mbufs(ptrs)
        assert eng.pending() == 0
        for bad in (dict(batch_frames=0), dict(depth=0), dict(depth=17), dict(batch_bytes=100)):
            with pytest.raises(RuntimeError, match="ixg_rx_async_init"):
                eng.async_init(**{**ixgrx.ASYNC_DEFAULTS, **bad})
    finally:
        eng.close()


@pytest.mark.parametrize("kind", ["tcp64", "imix", "mixed", "tcp1514"])
def test_async_zero_copy(fake, kind):
    """Registered mbuf memory (ixg_rx_register_memory): frames of at least
    IXG_ZC_MIN_LEN bytes are read in place, nothing of them is gathered;
    shorter ones, and frames of unregistered mbufs in the same batches, are
    gathered; records as the oracle's, in order."""
    fake.lib.fakehip_inplace_frames.restype = ctypes.c_ulong
    rng = np.random.default_rng(21)
    tr, arena, ptrs = _mbufs(kind, 6000, seed=13)
    tr2, arena2, ptrs2 = _mbufs("imix", 6000, seed=14)  # stays unregistered
    mix = np.where(rng.random(6000) < 0.7, ptrs, ptrs2)
    eng = fake()
    try:
        eng.async_init(**ixgrx.ASYNC_DEFAULTS)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        with pytest.raises(RuntimeError, match="ixg_rx_register_memory"):
            eng.register_memory(arena.ctypes.data + 4096, 1 << 16)  # overlaps
        n0 = fake.lib.fakehip_inplace_frames()
        m, r = _loop(eng, ptrs, rng)
        # every frame of >= IXG_ZC_MIN_LEN bytes whose mbuf (and the tail
        # bytes) lies inside the region is read in place
        hi = arena.ctypes.data + arena.nbytes
        big = tr.len.astype(np.int64) >= ixgrx.IXG_ZC_MIN_LEN
        inside = (ptrs.astype(np.int64) + 2112 + 64 <= hi) & big
        assert fake.lib.fakehip_inplace_frames() - n0 == int(inside.sum()) >= int(big.sum()) - 1
        assert kind not in ("imix", "tcp1514") or inside.sum() > 0
        assert np.array_equal(m, ptrs)
        assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))
        n1 = fake.lib.fakehip_inplace_frames()
        m, r = _loop(eng, mix, rng)
        assert fake.lib.fakehip_inplace_frames() - n1 == int(((mix == ptrs) & (mix.astype(np.int64) + 2176 <= hi) & big).sum())
        assert np.array_equal(m, mix)
        assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(mix))
        eng.unregister_memory(arena.ctypes.data)
        with pytest.raises(RuntimeError, match="ixg_rx_unregister_memory"):
            eng.unregister_memory(arena.ctypes.data)
    finally:
        eng.close()


def test_set_fdir_waits_for_async_batches(fake):
    """ixg_rx_set_fdir from IX's connect path while the run loop has batches
    in flight: the open batch is launched first and every batch
    in flight finishes before the table is rewritten, so no launch reads a
    table other than the one in force when it was made."""
    fake.lib.fakehip_fdir_stale.restype = ctypes.c_ulong
    tr, arena, ptrs = _mbufs("tcp64", 200, seed=31)
    eng = fake()
    try:
        eng.async_init(batch_frames=64, batch_bytes=1 << 20, max_wait_us=10000000, depth=4)
        s0, n0 = fake.lib.fakehip_fdir_stale(), fake.lib.fakehip_launches()
        assert eng.submit_mbufs(ptrs[:64]) == 64       # launched, in flight
        assert eng.submit_mbufs(ptrs[64:94]) == 30     # open
        assert fake.lib.fakehip_launches() == n0       # nothing has run yet
        eng.set_fdir(np.array([(0x0a000001, 0x0a000002, 40000, 80)], dtype=ixgrx.FDIR_DTYPE), cpu_id=3)
        assert fake.lib.fakehip_launches() - n0 == 2   # the open batch went, both ran
        assert eng.submit_mbufs(ptrs[94:200]) == 106
        m, r = eng.poll(1000, wait=True)
        while eng.pending():
            m2, r2 = eng.poll(1000, wait=True)
            m, r = np.concatenate([m, m2]), np.concatenate([r, r2])
        eng.set_fdir(None, cpu_id=0)
        assert fake.lib.fakehip_fdir_stale() == s0
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))


def test_submit_launch_failure_keeps_accepted_frames(fake):
    """A launch that fails after submit accepted frames: submit
    returns the count it took, the next call reports the error once, and the
    frames stay in the open batch, launched again later and returned by poll
    in order, exactly once."""
    tr, arena, ptrs = _mbufs("imix", 200, seed=32)
    eng = fake()
    try:
        eng.async_init(batch_frames=64, batch_bytes=1 << 20, max_wait_us=10000000, depth=2)
        n0 = fake.lib.fakehip_launches()
        fake.lib.fakehip_fail_launches(1)
        assert eng.submit_mbufs(ptrs[:100]) == 64      # the batch filled, its launch failed
        assert eng.pending() == 64
        with pytest.raises(RuntimeError, match="ixg_rx_submit_mbufs"):
            eng.submit_mbufs(ptrs[64:100])           # the error, once
        m, r = eng.poll(1000, wait=True)             # launches the open batch again
        assert fake.lib.fakehip_launches() - n0 == 1
        assert np.array_equal(m, ptrs[:64])
        fake.lib.fakehip_fail_launches(1)
        assert eng.submit_mbufs(ptrs[64:100]) == 36
        with pytest.raises(RuntimeError, match="ixg_rx_flush"):
            eng.flush()                              # its launch fails: reported by flush itself
        assert eng.pending() == 36
        m2, r2 = eng.poll(1000, wait=True)
        assert np.array_equal(m2, ptrs[64:100]) and eng.pending() == 0
    finally:
        eng.close()
    exp = _expect(ptrs[:100])
    assert np.array_equal(np.concatenate([r, r2]).view(np.uint8).reshape(-1, 16), exp)


def test_async_stats_counters(fake):
    """ixg_rx_async_stats: frames in and out, refusals under back-pressure,
    batches launched full vs by time, and the time buckets filled."""
    tr, arena, ptrs = _mbufs("tcp64", 640, seed=33)
    eng = fake()
    try:
        eng.async_init(batch_frames=128, batch_bytes=1 << 20, max_wait_us=10000000, depth=2)
        eng.async_stats(reset=True)
        assert eng.submit_mbufs(ptrs[:64]) == 64
        assert eng.submit_mbufs(ptrs[64:192]) == 128   # batch 1 full (launched), batch 2 open (64)
        assert eng.submit_mbufs(ptrs[192:400]) == 64   # batch 2 full, ring full: 144 refused
        st = eng.async_stats()
        assert st["frames_submitted"] == 256 and st["frames_refused"] == 144 and st["submit_calls"] == 3
        assert st["batches"] == 2 and st["batches_by_time"] == 0
        m, r = eng.poll(1000, wait=True)
        while eng.pending():
            m2, r2 = eng.poll(1000, wait=True)
            m = np.concatenate([m, m2])
        assert eng.submit_mbufs(ptrs[256:300]) == 44
        eng.flush()                                     # launched before full
        m3, _ = eng.poll(1000, wait=True)
        st = eng.async_stats(reset=True)
        assert st["frames_returned"] == 300 and st["batches"] == 3 and st["batches_by_time"] == 1
        assert st["gather_ns"] > 0 and st["launch_ns"] > 0 and st["poll_calls"] >= 3
        # the worst batch's split: the parts add up to
        # the total; no device clock on the fake runtime, so no "gpu" part
        assert st["worst_total_ns"] > 0 and st["worst_gpu_ns"] == 0
        assert st["worst_open_ns"] + st["worst_visible_ns"] + st["worst_returned_ns"] == st["worst_total_ns"]
        assert st["worst_wait_ns"] <= st["worst_total_ns"]
        # poll(wait)'s naps: the worst batch's longest nap is part of its wait
        assert st["worst_nap_max_ns"] <= st["worst_wait_ns"] and st["nap_max_ns"] <= st["wait_ns"]
        assert (st["worst_naps"] == 0) == (st["worst_nap_max_ns"] == 0)
        assert eng.async_stats()["frames_submitted"] == 0   # reset
        assert eng.async_stats()["worst_total_ns"] == 0
    finally:
        eng.close()
    assert np.array_equal(np.concatenate([m, m3]), ptrs[:300])


def test_zero_copy_batch_counts_link_bytes(fake):
    """an in-place frame costs the kernels its length in
    host-link reads, so it counts against batch_bytes: 1514-B frames read in
    place close a batch of 64 KiB at ~43 frames, not at batch_frames."""
    tr, arena, ptrs = _mbufs("tcp1514", 600, seed=41)
    eng = fake()
    try:
        eng.async_init(batch_frames=16384, batch_bytes=64 << 10, max_wait_us=10000000, depth=16)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        n0 = fake.lib.fakehip_launches()
        acc = 0
        for k in range(0, 600, 50):
            acc += eng.submit_mbufs(ptrs[k:k + 50])
        eng.flush()
        m, r = eng.poll(1000, wait=True)
        while eng.pending():
            m2, r2 = eng.poll(1000, wait=True)
            m, r = np.concatenate([m, m2]), np.concatenate([r, r2])
        st = eng.async_stats()
        launches = fake.lib.fakehip_launches() - n0
    finally:
        eng.close()
    link = 1536  # 1514 B in 64-B host-link requests
    per = st["frames_submitted"] / max(st["batches"], 1)
    assert acc == 600 and launches == st["batches"]
    assert per <= (64 << 10) // link + 1, per     # closed by its link bytes
    assert st["batches"] >= 600 * link // ((64 << 10) + link)
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))


def _last_stride(lib):
    s, n = ctypes.c_uint32(), ctypes.c_uint32()
    lib.fakehip_last_launch(ctypes.byref(s), ctypes.byref(n))
    return s.value, n.value


def test_gather_stops_at_ip_len(fake):
    """bytes past max(14 + ip_len, l4 + 20) of an IPv4
    frame (C2's 6-B Ethernet pad) are not staged: C2 frames stage bytes
    12..55, a 44-B stride instead of 48, and the records do not change when
    the pads hold garbage (the gathered image then carries the next frame's
    bytes where a frame's pad was)."""
    rng = np.random.default_rng(42)
    tr = traces.make_trace("tcp64", 4000, seed=43)
    blob = tr.blob.copy()
    offs = tr.offsets().astype(np.int64)
    for o in offs[:, None] + np.arange(54, 60)[None, :]:
        blob[o] = rng.integers(0, 256, o.shape, dtype=np.uint8)
    tr = traces.Trace(blob=blob, len=tr.len, stride=tr.stride, off=tr.off)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng = fake()
    try:
        rec = eng.batch_mbufs(ptrs)
        assert _last_stride(fake.lib) == (44, 4000)
        eng.async_init(batch_frames=1000, batch_bytes=1 << 20, max_wait_us=10000000, depth=4)
        m, r = _loop(eng, ptrs, rng)
        assert _last_stride(fake.lib)[0] == 44
    finally:
        eng.close()
    exp = _expect(ptrs)
    assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), exp)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), exp)


@pytest.mark.parametrize("kind", ["imix", "mixed", "tcp1514"])
def test_gather_garbage_past_ip_len(fake, kind):
    """Frames whose IP total length ends short of the frame (random ip_len
    cuts, random bytes behind them) through the shortened gather, offsets
    layout: records as the oracle's over the whole frames."""
    rng = np.random.default_rng(44)
    tr = traces.make_trace(kind, 3000, seed=45)
    frames = []
    for o, L in zip(tr.offsets().astype(np.int64), tr.len.astype(np.int64)):
        f = bytearray(tr.blob[o:o + L].tobytes())
        if L >= 34 and f[12:14] == b"\x08\x00" and rng.random() < 0.5:
            ip_len = int.from_bytes(f[16:18], "big")
            cut = int(rng.integers(0, max(1, min(ip_len, L - 14) - 20)))
            f[16:18] = (ip_len - cut).to_bytes(2, "big")
            f[14 + ip_len - cut:] = rng.integers(0, 256, L - (14 + ip_len - cut), dtype=np.uint8).tobytes()
        frames.append(bytes(f))
    tr2 = traces.pack(frames)
    arena, ptrs = ixgrx.make_mbufs(tr2)
    eng = fake()
    try:
        rec = eng.batch_mbufs(ptrs)
        eng.async_init(batch_frames=700, batch_bytes=1 << 18, max_wait_us=10000000, depth=3)
        m, r = _loop(eng, ptrs, rng)
    finally:
        eng.close()
    exp = _expect(ptrs)
    assert np.array_equal(rec.view(np.uint8).reshape(-1, 16), exp)
    assert np.array_equal(m, ptrs)
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), exp)


def test_zero_copy_launch_failure_retried(fake):
    """a zero-copy batch whose launch fails is launched again
    later; the in-place frames' offsets must be laid out again from the
    gathered ones (the old layout step rewrote them in place, so the retry
    rebased them twice: a GPU page fault, here fakehip's abort)."""
    fake.lib.fakehip_inplace_frames.restype = ctypes.c_ulong
    tr, arena, ptrs = _mbufs("tcp1514", 300, seed=46)
    eng = fake()
    try:
        eng.async_init(batch_frames=128, batch_bytes=1 << 24, max_wait_us=10000000, depth=2)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        n0 = fake.lib.fakehip_inplace_frames()
        assert eng.submit_mbufs(ptrs[:100]) == 100
        fake.lib.fakehip_fail_launches(1)
        assert eng.submit_mbufs(ptrs[100:200]) == 28    # batch 1 full: its launch fails
        with pytest.raises(RuntimeError, match="ixg_rx_poll"):
            eng.poll(1000, wait=False)                  # the error, once
        m, r = eng.poll(1000, wait=True)                # launched again, in place
        while eng.pending():
            m2, r2 = eng.poll(1000, wait=True)
            m, r = np.concatenate([m, m2]), np.concatenate([r, r2])
        assert fake.lib.fakehip_inplace_frames() - n0 == 128
    finally:
        eng.close()
    assert np.array_equal(m, ptrs[:128])
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs[:128]))


@pytest.mark.parametrize("direct", [True, False])
def test_async_icmp_reflect_golden(fake, direct):
    """IXG_ASYNC_ICMP_REFLECT: the golden frames of the
    reference's icmp_input (tests/golden/icmp.npz) through submit/poll with
    the mbuf pool registered: every echo request comes back already turned
    into the reply the reference builds in its mbuf, with IXG_RF_REPLY in
    its record; every other frame and record is untouched."""
    fake.lib.fakehip_icmp_items.restype = ctypes.c_ulong
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "icmp.npz")))
    tr = traces.Trace(blob=g["blob"].copy(), off=g["off"], len=g["len"], stride=0)
    arena, ptrs = ixgrx.make_mbufs(tr)
    exp = _expect(ptrs)
    refl = g["reflected"].astype(bool)
    eng = fake()
    try:
        eng.async_init(batch_frames=40, batch_bytes=1 << 20, max_wait_us=10000000, depth=3, direct=direct,
                       icmp_reflect=True)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        eng.set_icmp_reply(bytes(g["mac"]), int(g["host_addr"]))
        n0 = fake.lib.fakehip_icmp_items()
        m, r = _loop(eng, ptrs, np.random.default_rng(5), max_batch=16)
        items = fake.lib.fakehip_icmp_items() - n0
    finally:
        eng.close()
    assert np.array_equal(m, ptrs)
    got = r.view(np.uint8).reshape(-1, 16)
    want = exp.copy()
    want[refl, 3] |= ixgrx.RF_REPLY
    assert np.array_equal(got, want)
    assert items >= int(refl.sum())          # candidates: IPv4 protocol 1 frames in the region
    base = arena.ctypes.data
    for i, (p, o, L) in enumerate(zip(ptrs.astype(np.int64), g["off"].astype(np.int64), g["len"].astype(np.int64))):
        mb = arena[p - base + 64:p - base + 64 + L]
        assert np.array_equal(mb, g["after"][o:o + L]), i


def test_async_icmp_reflect_needs_registered_mbufs(fake):
    """Echo requests whose mbufs are not in a registered region are left to
    the host's icmp_reflect: record unchanged (no IXG_RF_REPLY), frame
    untouched."""
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "icmp.npz")))
    tr = traces.Trace(blob=g["blob"].copy(), off=g["off"], len=g["len"], stride=0)
    arena, ptrs = ixgrx.make_mbufs(tr)
    before = arena.copy()
    eng = fake()
    try:
        eng.async_init(batch_frames=64, batch_bytes=1 << 20, max_wait_us=10000000, depth=3, icmp_reflect=True)
        eng.set_icmp_reply(bytes(g["mac"]), int(g["host_addr"]))
        m, r = _loop(eng, ptrs, np.random.default_rng(6))
    finally:
        eng.close()
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), _expect(ptrs))
    assert np.array_equal(arena, before)


@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("inject", ["stamp", "launch"])
def test_async_icmp_reflect_failures_reflect_once(fake, direct, inject):
    """a launch that fails after the echo reflect was enqueued
    (the completion stamp, here) must not leave the batch to be launched
    again: the retry would parse the replies and reflect them back into
    requests. Such a batch is completed on the spot; a batch whose RX launch
    itself fails (nothing enqueued has touched an mbuf) is retried. Either
    way every echo request comes back reflected exactly once, as the
    reference's icmp_input leaves it (tests/golden/icmp.npz)."""
    fake.lib.fakehip_fail_stamps.argtypes = [ctypes.c_int]
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "icmp.npz")))
    tr = traces.Trace(blob=g["blob"].copy(), off=g["off"], len=g["len"], stride=0)
    arena, ptrs = ixgrx.make_mbufs(tr)
    exp = _expect(ptrs)
    refl = g["reflected"].astype(bool)
    rng = np.random.default_rng(11)
    eng = fake()
    errors = 0
    try:
        eng.async_init(batch_frames=24, batch_bytes=1 << 20, max_wait_us=10000000, depth=3, direct=direct,
                       icmp_reflect=True)
        eng.register_memory(arena.ctypes.data, arena.nbytes)
        eng.set_icmp_reply(bytes(g["mac"]), int(g["host_addr"]))
        got_m, got_r = [], []
        i = 0
        while i < len(ptrs) or eng.pending():
            if i < len(ptrs) and rng.integers(0, 3) == 0:
                (fake.lib.fakehip_fail_stamps if inject == "stamp" else fake.lib.fakehip_fail_launches)(1)
            acc = 0
            if i < len(ptrs):
                k = int(rng.integers(1, 17))
                try:
                    acc = eng.submit_mbufs(ptrs[i:i + k])
                except RuntimeError:
                    errors += 1
                    continue
                i += acc
            try:
                m, r = eng.poll(1000, wait=acc == 0)
            except RuntimeError:
                errors += 1
                continue
            got_m.append(m)
            got_r.append(r)
        fake.lib.fakehip_fail_stamps(0)
        fake.lib.fakehip_fail_launches(0)
    finally:
        eng.close()
    if inject == "launch":
        assert errors > 0
    m, r = np.concatenate(got_m), np.concatenate(got_r)
    assert np.array_equal(m, ptrs)
    want = exp.copy()
    want[refl, 3] |= ixgrx.RF_REPLY
    assert np.array_equal(r.view(np.uint8).reshape(-1, 16), want)
    base = arena.ctypes.data
    for j, (p, o, L) in enumerate(zip(ptrs.astype(np.int64), g["off"].astype(np.int64), g["len"].astype(np.int64))):
        assert np.array_equal(arena[p - base + 64:p - base + 64 + L], g["after"][o:o + L]), j
