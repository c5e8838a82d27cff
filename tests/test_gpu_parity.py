"""HIP kernels vs the reference (golden fixtures) and vs the oracle.

All comparisons are bit-exact on the whole 16-byte record and on the
residual words. Sizes: the oracle finishes in seconds; full BASELINE sizes
are covered by size-independent properties (a tiled trace's records are the
tiled records of its pool).
"""
import os
import sys

import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402  (frame builders only; the harness is not run here)

KEY = traces.RSS_KEY


def _recs_u8(rec):
    return rec.view(np.uint8).reshape(-1, 16)


def _diff(got, exp, what):
    g = _recs_u8(got) if got.dtype == ixgrx.REC_DTYPE else got
    bad = np.nonzero((g != exp).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} records differ; first {bad[:6].tolist()}: " \
                          f"gpu {g[bad[0]].tolist()} vs exp {exp[bad[0]].tolist()}"


@pytest.fixture(scope="module", params=["auto", "general", "fast", "short", "long"])
def engines(request):
    """Engines on the default path (the device-side sampler picks the split),
    with the general kernel alone (no defer flags), and with each launch
    split forced (ixg_rx_set_split): fixed-shape kernel first, short kernel
    walking every chunk, long kernel walking every chunk."""
    cache = {}

    def get(key=KEY, nb=128, dev=0, flags=0):
        k = (bytes(key), nb, dev, flags)
        if k not in cache:
            cache[k] = ixgrx.RxEngine(ixgrx.Config(bytes(key), nb, dev, flags), split=request.param)
        return cache[k]
    yield get
    for e in cache.values():
        e.close()


def test_golden_fixtures(golden, engines):
    eng = engines(bytes(golden["key"]), int(golden["nb_rx_fgs"]), int(golden["dev_idx"]), int(golden["flags"]))
    if "fdir" in golden:  # the flow-director fixture: the reference's outbound-group mapping
        eng.set_fdir(np.ascontiguousarray(golden["fdir"]).view(ixgrx.FDIR_DTYPE).reshape(-1), int(golden["fdir_cpu"]))
    try:
        rec, cs = eng.batch_host(golden["blob"], golden["off"], golden["len"], want_csum=True)
    finally:
        eng.set_fdir(None)
    _diff(rec, golden["rec"], golden["name"])
    bad = np.nonzero(cs != golden["csum"])[0]
    assert bad.size == 0, f"residuals differ at {bad[:8].tolist()}"


@pytest.mark.parametrize("kind,n,flags", [
    ("tcp64", 50000, 0), ("imix", 30000, 0), ("tcp1514", 8000, 0), ("mixed", 30000, 0),
    ("mixed", 30000, ixgrx.IXG_F_IPV6), ("imix", 20000, ixgrx.IXG_F_NO_CSUM_DROP),
    ("tcp64opt", 50000, 0),  # C2's 60-B slots, ihl 6: every coalesced chunk deferred
])
def test_synthetic_vs_oracle(kind, n, flags, engines):
    tr = traces.make_trace(kind, n, seed=0x1B0000 + n, bad_ip=0.01, bad_l4=0.01)
    eng = engines(flags=flags)
    rec, cs = eng.batch_trace(tr, want_csum=True)
    er, ec = oracle.rx_trace(tr, KEY, flags=flags, threads=8, hash_mode=oracle.HASH_TABLE)
    _diff(rec, er, kind)
    assert (cs == ec).all()


def test_fuzz_vs_oracle(engines):
    rng = np.random.default_rng(99)
    frames = mg.fuzz_frames(rng, 40000) + mg.edge_frames()
    tr = traces.pack(frames)
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP, ixgrx.IXG_F_IPV6):
        rec, cs = engines(flags=flags).batch_trace(tr, want_csum=True)
        er, ec = oracle.rx_trace(tr, KEY, flags=flags, threads=8)
        _diff(rec, er, f"fuzz flags={flags}")
        assert (cs == ec).all()


def test_random_keys_and_groups(engines):
    rng = np.random.default_rng(5)
    tr = traces.make_trace("imix", 5000, seed=11)
    for _ in range(3):
        key = bytes(rng.integers(0, 256, 40, dtype=np.uint8))
        nb = int(2 ** rng.integers(0, 10))
        dev = int(rng.integers(0, 100))
        rec = engines(key, nb, dev, 0).batch_trace(tr)
        er, _ = oracle.rx_trace(tr, key, nb, dev, 0, threads=8)
        _diff(rec, er, f"key/nb={nb}/dev={dev}")


def test_mbuf_path(engines):
    tr = traces.make_trace("imix", 3000, seed=21, bad_ip=0.02, bad_l4=0.02)
    arena, ptrs = ixgrx.make_mbufs(tr)
    rec = engines().batch_mbufs(ptrs)
    er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs)
    _diff(rec, er, "mbufs")


@pytest.mark.parametrize("kind,n", [("imix", 150000), ("tcp1514", 50000)])
def test_mbuf_path_pipelined(kind, n, engines):
    """A batch larger than one pipeline chunk (131072 frames / 64 MiB): the
    chunks go through the two stages in turn and records land in order."""
    tr = traces.make_trace(kind, n, seed=22, bad_ip=0.01, bad_l4=0.01)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng = engines()
    rec = eng.batch_mbufs(ptrs)
    er = oracle.rx_mbufs(KEY, 128, 0, 0, ptrs, threads=8)
    _diff(rec, er, "mbufs pipelined")
    rec2 = eng.batch_mbufs(ptrs[: n // 3])  # the stages are reusable, and a short batch after a long one
    _diff(rec2, er[: n // 3], "mbufs pipelined, second call")


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 1000, 4097])
def test_ragged_sizes(n, engines):
    tr = traces.make_trace("mixed", n, seed=n)
    rec = engines(flags=ixgrx.IXG_F_IPV6).batch_trace(tr)
    er, _ = oracle.rx_trace(tr, KEY, flags=ixgrx.IXG_F_IPV6)
    _diff(rec, er, f"n={n}")


def test_empty_batch(engines):
    rec = engines().batch_host(np.zeros(64, np.uint8), None, np.zeros(0, np.uint16), 64)
    assert rec.shape == (0,)


def test_strided_and_permuted_offsets(engines):
    tr = traces.make_trace("imix", 4000, seed=3)
    perm = np.random.default_rng(0).permutation(tr.n)
    off = tr.off[perm]
    lens = tr.len[perm]
    rec = engines().batch_host(tr.blob, off, lens)
    er, _ = oracle.rx_batch(KEY, 128, 0, 0, tr.blob, off, lens)
    _diff(rec, er, "permuted")
    rows = traces.build_ipv4(np.random.default_rng(1), 3000, 60, 6)
    t2 = traces.pack_rows(rows, 128)
    rec = engines().batch_trace(t2)
    er, _ = oracle.rx_trace(t2, KEY)
    _diff(rec, er, "stride128")


def test_device_path_torch_stream(engines):
    import torch
    tr = traces.make_trace("tcp64", 100000, seed=8, bad_ip=0.01, bad_l4=0.01)
    dev = torch.device("cuda:0")
    blob = torch.from_numpy(tr.blob).to(dev)
    lens = torch.from_numpy(tr.len.astype(np.int16)).to(dev)
    out = torch.empty((tr.n, 16), dtype=torch.uint8, device=dev)
    cs = torch.empty(tr.n, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        engines().batch_dev(blob.data_ptr(), None, lens.data_ptr(), tr.stride, tr.n, out.data_ptr(),
                            cs.data_ptr(), s.cuda_stream)
    s.synchronize()
    er, ec = oracle.rx_trace(tr, KEY, threads=8, hash_mode=oracle.HASH_TABLE)
    _diff(out.cpu().numpy(), er, "device path")
    assert (cs.cpu().numpy().view(np.uint32) == ec).all()


@pytest.mark.parametrize("kind", ["mixed", "imix"])
def test_offsets_past_2_and_4_gib(kind, engines):
    """u64 offsets with bit 31 and bit 32 set (batches over 2 GiB, like C3's
    6 GB and C4's): frames placed across the 2 GiB and 4 GiB marks of one
    4.3 GB buffer. Covers the kernels' 64-bit wave broadcasts of frame
    offsets (the span kernel's staging decision read a low word >= 2^31 as
    negative and sign-extended it; those chunks silently took per-lane
    loads)."""
    import torch
    tr = traces.make_trace(kind, 20000, seed=77, bad_ip=0.01, bad_l4=0.01)
    er, ec = oracle.rx_trace(tr, KEY, threads=8, hash_mode=oracle.HASH_TABLE)
    dev = torch.device("cuda:0")
    span = int(tr.off[-1]) + int(tr.len[-1])
    src = torch.from_numpy(np.ascontiguousarray(tr.blob[:span])).to(dev)
    buf = torch.zeros((1 << 32) + span + 4096, dtype=torch.uint8, device=dev)
    lens = torch.from_numpy(tr.len.astype(np.int16)).to(dev)
    out = torch.empty((tr.n, 16), dtype=torch.uint8, device=dev)
    cs = torch.empty(tr.n, dtype=torch.int32, device=dev)
    try:
        for base in ((1 << 31) - span // 2, (1 << 32) - span // 3):
            base &= ~15
            buf[base:base + span] = src
            off = torch.from_numpy(tr.offsets().astype(np.int64) + base).to(dev)
            out.zero_()
            engines().batch_dev(buf.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, tr.n, out.data_ptr(),
                                cs.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            _diff(out.cpu().numpy(), er, f"{kind} at base {base:#x}")
            assert (cs.cpu().numpy().view(np.uint32) == ec).all()
    finally:
        del buf
        torch.cuda.empty_cache()


def test_full_size_tcp64_tiled(engines):
    """C2 at full size (16M frames): records must be the pool's records tiled."""
    import torch
    n, pool = 16 * 1024 * 1024, 65536
    tr = traces.make_trace("tcp64", pool, seed=0x1B0002)
    er, _ = oracle.rx_trace(tr, KEY, threads=8, hash_mode=oracle.HASH_TABLE)
    dev = torch.device("cuda:0")
    frames = torch.from_numpy(tr.blob[:pool * 60]).to(dev).view(pool, 60)
    big = frames.repeat(n // pool, 1).reshape(-1)
    blob = torch.zeros(big.numel() + 64, dtype=torch.uint8, device=dev)
    blob[:big.numel()] = big
    lens = torch.full((n,), 60, dtype=torch.int16, device=dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    engines().batch_dev(blob.data_ptr(), None, lens.data_ptr(), 60, n, out.data_ptr(), None,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = torch.from_numpy(er).to(dev).repeat(n // pool, 1)
    assert torch.equal(out, exp)


def test_full_size_1514_tiled(engines):
    """C4 per-GPU shard shape (1514 B frames) at 1M frames: tiled property."""
    import torch
    n, pool = 1 << 20, 4096
    tr = traces.make_trace("tcp1514", pool, seed=0x1B0004)
    er, _ = oracle.rx_trace(tr, KEY, threads=8, hash_mode=oracle.HASH_TABLE)
    dev = torch.device("cuda:0")
    S = tr.stride
    frames = torch.from_numpy(tr.blob[:pool * S]).to(dev).view(pool, S)
    blob = torch.zeros(n * S + 64, dtype=torch.uint8, device=dev)
    blob[:n * S].view(n, S).copy_(frames.repeat(n // pool, 1))
    lens = torch.full((n,), 1514, dtype=torch.int16, device=dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    engines().batch_dev(blob.data_ptr(), None, lens.data_ptr(), S, n, out.data_ptr(), None,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = torch.from_numpy(er).to(dev).repeat(n // pool, 1)
    assert torch.equal(out, exp)


@pytest.mark.parametrize("S", [4, 16, 32, 48, 60, 64])
def test_fixed_strides_up_to_64(S, engines):
    """The coalesced fixed-shape path (stride <= 64): valid 60 B frames where
    they fit the slot, plus random bytes and lengths 0..64 (frames longer
    than the stride overlap the next slot), ragged last chunk."""
    rng = np.random.default_rng(S)
    n = 64 * 37 + 13
    blob = rng.integers(0, 256, n * S + 64 + 64, dtype=np.uint8)
    lens = rng.integers(0, 65, n).astype(np.uint16)
    if S >= 60:
        rows = traces.build_ipv4(rng, n, 60, 6)
        good = rng.random(n) < 0.8
        for i in np.nonzero(good)[0]:
            blob[i * S:i * S + 60] = rows[i]
            lens[i] = 60
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP):
        rec, cs = engines(flags=flags).batch_host(blob, None, lens, S, want_csum=True)
        er, ec = oracle.rx_batch(KEY, 128, 0, flags, blob, None, lens, S)
        _diff(rec, er, f"stride {S}")
        assert (cs == ec).all()


def test_fixed_stride_all_fast_and_misaligned_base(engines):
    """A batch whose chunks are all fixed-shape, at a 16-B aligned base
    (coalesced kernel) and at a base 4 bytes off (lane-load kernel)."""
    import torch
    tr = traces.make_trace("tcp64", 64 * 500 + 7, seed=12, bad_ip=0.01, bad_l4=0.01)
    er, ec = oracle.rx_trace(tr, KEY, threads=8)
    dev = torch.device("cuda:0")
    for shift in (0, 4):
        raw = torch.zeros(tr.blob.shape[0] + 64, dtype=torch.uint8, device=dev)
        raw[shift:shift + tr.blob.shape[0]] = torch.from_numpy(tr.blob).to(dev)
        lens = torch.from_numpy(tr.len.astype(np.int16)).to(dev)
        out = torch.empty((tr.n, 16), dtype=torch.uint8, device=dev)
        cs = torch.empty(tr.n, dtype=torch.int32, device=dev)
        engines().batch_dev(raw.data_ptr() + shift, None, lens.data_ptr(), tr.stride, tr.n, out.data_ptr(),
                            cs.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        _diff(out.cpu().numpy(), er, f"shift {shift}")
        assert (cs.cpu().numpy().view(np.uint32) == ec).all()


def _tcp_frames_uniform(rng, n, ipl, doff, pad_to):
    """n IPv4/TCP frames with ip_len `ipl`, data offsets `doff` (per frame,
    any of 0..15: doff*4 > l4len is tcp_input's HDRLEN drop), frame lengths
    pad_to (per frame, >= 14 + ipl: Ethernet padding past the datagram), valid
    checksums. Returns (rows [n, 64], lengths)."""
    rows = np.zeros((n, 64), np.uint8)
    rows[:, :14 + ipl] = traces.build_ipv4(rng, n, 14 + ipl, 6)
    traces._put16(rows, 16, np.full(n, ipl))  # (build_ipv4 makes 60-B TCP frames ip_len 40)
    rows[:, 24:26] = 0
    traces._put16(rows, 24, (~traces._fold(traces._sum_be16(rows[:, 14:34]))) & 0xFFFF)
    rows[:, 46] = (doff.astype(np.uint8) << 4)
    rows[:, 47] = rng.integers(0, 256, n, dtype=np.uint8)  # every TCP flag combination
    rows[:, 50:52] = 0
    seg = rows[:, 34:14 + ipl]
    if seg.shape[1] % 2:
        seg = np.concatenate([seg, np.zeros((n, 1), np.uint8)], axis=1)
    s = traces._sum_be16(seg) + traces._sum_be16(rows[:, 26:34]) + 6 + (ipl - 20)
    traces._put16(rows, 50, (~traces._fold(s)) & 0xFFFF)
    return rows, pad_to.astype(np.uint16)


@pytest.mark.parametrize("S", [60, 64])
def test_lean_tcp_chunks(S, engines):
    """The coalesced kernel's lean path (every frame of a chunk an accepted
    TCP segment of one IP length): chunk-uniform ip_len 40..50, every data
    offset tcp_input accepts (0 and 5..(ip_len-20)/4), Ethernet padding,
    every TCP flag byte, bad IP / TCP checksums, the outbound flow director,
    and chunks that leave the lean path for the general fixed-shape parse:
    one frame with a data offset past the segment (DROP_TCP_HDRLEN), one UDP
    frame, one fragment, one frame of another ip_len. Ragged last chunk."""
    import torch
    rng = np.random.default_rng(0x1EA0 + S)
    nch = 160
    n = 64 * nch - 23
    ipls = rng.integers(20, 26, nch) * 2  # 40..50, per chunk
    if S == 60:
        ipls = np.minimum(ipls, 46)
    blob = np.zeros(n * S + 128, np.uint8)
    lens = np.zeros(n, np.uint16)
    for c in range(nch):
        m = min(64, n - 64 * c)
        ipl = int(ipls[c])
        dmax = (ipl - 20) // 4
        doff = rng.choice(np.array([0] + list(range(5, dmax + 1))), m)
        pad = rng.integers(14 + ipl, S + 1, m)
        rows, L = _tcp_frames_uniform(rng, m, ipl, doff, pad)
        kind = c % 8
        if kind == 1:      # data offset past the segment
            rows[rng.integers(0, m), 46] = 0xF0
        elif kind == 2:    # a UDP frame
            rows[rng.integers(0, m), 23] = 17
        elif kind == 3:    # a fragment
            rows[rng.integers(0, m), 21] = 0x08
        elif kind == 4 and ipl < 50 and 14 + ipl + 2 <= S:  # another ip_len
            j = rng.integers(0, m)
            r2, _ = _tcp_frames_uniform(rng, 1, ipl + 2, np.array([5]), np.array([14 + ipl + 2]))
            rows[j] = r2[0]
            L[j] = max(int(L[j]), 14 + ipl + 2)
        bad = rng.random(m) < 0.05
        rows[bad, 24] ^= 0x11
        bad = rng.random(m) < 0.05
        rows[bad, 51] ^= 0x22
        for k in range(m):
            i = 64 * c + k
            blob[i * S:i * S + int(L[k])] = rows[k, :int(L[k])]
        lens[64 * c:64 * c + m] = L
    tr = traces.Trace(blob, None, lens, S)
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(blob).to(dev)
    tl = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    cs = torch.empty(n, dtype=torch.int32, device=dev)
    offs = tr.offsets().astype(np.int64)
    tcp = np.nonzero(blob[offs + 23] == 6)[0]
    filt = np.zeros(40, ixgrx.FDIR_DTYPE)
    pick = rng.choice(tcp, filt.size, replace=False)
    for k, i in enumerate(pick):
        o = int(offs[i])
        filt[k] = (int.from_bytes(bytes(blob[o + 26:o + 30]), "little"), int.from_bytes(bytes(blob[o + 30:o + 34]), "little"),
                   int(blob[o + 34]) << 8 | int(blob[o + 35]), int(blob[o + 36]) << 8 | int(blob[o + 37]))
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP):
        eng = engines(flags=flags)
        for fdir in (None, filt):
            eng.set_fdir(fdir, 3)
            try:
                eng.batch_dev(tb.data_ptr(), None, tl.data_ptr(), S, n, out.data_ptr(), cs.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
            finally:
                eng.set_fdir(None)
            er, ec = oracle.rx_batch(KEY, 128, 0, flags, blob, None, lens, S, threads=8, fdir=fdir, cpu_id=3)
            _diff(out.cpu().numpy(), er, f"lean S={S} flags={flags} fdir={fdir is not None}")
            assert (cs.cpu().numpy().view(np.uint32) == ec).all()


def test_small_stride_with_long_lengths(engines):
    """Fixed stride <= 64 (the coalesced kernel) with some lengths far past
    the stride: those frames read on into their neighbours' bytes, so their
    chunks are long-class and take the general kernel's streaming path."""
    import torch
    rng = np.random.default_rng(31)
    n, S = 64 * 300 + 5, 64
    blob = rng.integers(0, 256, size=n * S + 2048, dtype=np.uint8)
    base = traces.make_trace("imix", n, seed=32)
    # real IPv4 headers at every slot start, lengths mostly <= 64, some long
    for i in range(n):
        f = base.frame(i)
        blob[i * S:i * S + min(S, len(f))] = np.frombuffer(f[:S], np.uint8)
    lens = np.minimum(base.len, 64).astype(np.uint16)
    longs = rng.random(n) < 0.05
    lens[longs] = rng.integers(112, 1600, size=int(longs.sum()))
    tr = traces.Trace(blob, None, lens, S)
    er, _ = oracle.rx_trace(tr, KEY, threads=8)
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(blob).to(dev)
    tl = torch.from_numpy(lens.view(np.int16)).to(dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    engines().batch_dev(tb.data_ptr(), None, tl.data_ptr(), S, n, out.data_ptr(), None,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _diff(out.cpu().numpy(), er, "stride 64, long lengths")


def test_jumbo_frames(engines):
    """Segments far past one streaming round (96 + 2 KiB): jumbo TCP/UDP
    frames of odd and even lengths, some with bad checksums."""
    rng = np.random.default_rng(77)
    frames = []
    for L in (2143, 2144, 2145, 2160, 3001, 4096, 9014, 16000, 30001, 65000):
        for proto in (6, 17):
            rows = traces.build_ipv4(rng, 3, L, proto)
            traces.corrupt(rng, rows, 0.0, 0.34, 34 + (16 if proto == 6 else 6))
            frames += [bytes(r) for r in rows]
    tr = traces.pack(frames)
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP):
        rec, cs = engines(flags=flags).batch_trace(tr, want_csum=True)
        er, ec = oracle.rx_trace(tr, KEY, flags=flags)
        _diff(rec, er, "jumbo")
        assert (cs == ec).all()


def _big_frames(rng, n):
    """Frames of 256 B or more only, so every chunk takes the long kernel's
    big-chunk path (prefixes from the streaming rounds): valid IPv4 TCP/UDP
    with ihl 5..15 and IPv6 of every length class around the 16-byte piece
    and 2 KiB round boundaries, ICMP echo, fuzzed headers and segments
    ending before the frame does (ip_len short of L: Ethernet trailer
    bytes), some with bad checksums."""
    frames = []
    for L in (256, 257, 258, 259, 271, 272, 273, 590, 1023, 1514, 2047, 2048, 2049, 2063, 2064, 2065, 2200):
        for proto in (6, 17):
            for ihl in (5, 9, 15):
                rows = traces.build_ipv4(rng, 2, L, proto, ihl=ihl)
                traces.corrupt(rng, rows, 0.25, 0.25, 14 + 4 * ihl + (16 if proto == 6 else 6))
                frames += [bytes(r) for r in rows]
            frames += [bytes(r) for r in traces.build_ipv6(rng, 2, L, proto)]
    for L in (256, 700, 1514):
        frames.append(mg.ipv4(proto=1, icmp_type=8, payload=bytes(rng.integers(0, 256, L - 42, dtype=np.uint8))))
    for f in mg.fuzz_frames(rng, n):
        f = bytearray(f)
        if len(f) < 256 or rng.random() < 0.3:
            # trailer bytes past the IP datagram (or a longer frame around a
            # truncated one)
            f += bytes(rng.integers(0, 256, int(rng.integers(256, 1200)), dtype=np.uint8))
        frames.append(bytes(f))
    order = rng.permutation(len(frames))
    return [frames[i] for i in order]


def test_big_chunks(engines):
    rng = np.random.default_rng(0xB16)
    frames = _big_frames(rng, 6000)
    assert min(len(f) for f in frames) >= 256
    tr = traces.pack(frames)
    for flags in (0, ixgrx.IXG_F_NO_CSUM_DROP, ixgrx.IXG_F_IPV6):
        rec, cs = engines(flags=flags).batch_trace(tr, want_csum=True)
        er, ec = oracle.rx_trace(tr, KEY, flags=flags, threads=8)
        _diff(rec, er, f"big chunks flags={flags}")
        assert (cs == ec).all()
    # the same frames at a fixed stride (the stride-layout kernels)
    S = (max(len(f) for f in frames) + 3) // 4 * 4
    ts = traces.pack(frames[:3000], stride=S)
    rec, cs = engines().batch_trace(ts, want_csum=True)
    er, ec = oracle.rx_trace(ts, KEY, threads=8)
    _diff(rec, er, "big chunks, stride")
    assert (cs == ec).all()


@pytest.mark.parametrize("kind", ["tcp64", "imix", "mixed"])
def test_hip_graph_replay(kind):
    """ixg_rx_batch_dev captured once into a HIP graph (torch.cuda.graph) and
    replayed over new frames copied into the same buffers: every replay is
    bit-exact (the per-launch class stamps are baked into the graph, so a
    replay may see a previous replay's stamps; that costs a scan, never a
    wrong record)."""
    import torch
    flags = 2 if kind == "mixed" else 0
    n = 20000
    # three batches in one layout (offsets, lengths): the second and third
    # with IP-header / last-byte corruptions in every 7th / 5th frame
    tr0 = traces.make_trace(kind, n, seed=900)
    offs = tr0.offsets().astype(np.int64)
    traces_ = [tr0]
    for k, (step, pos) in enumerate(((7, lambda i: offs[i] + 24), (5, lambda i: offs[i] + tr0.len[i].astype(np.int64) - 1))):
        b = tr0.blob.copy()
        idx = np.arange(k, n, step)
        b[pos(idx)] ^= 0x5A
        traces_.append(traces.Trace(b, tr0.off, tr0.len, tr0.stride))
    eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, flags))
    try:
        dev = torch.device("cuda:0")
        size = tr0.blob.size + 64
        blob = torch.zeros(size, dtype=torch.uint8, device=dev)
        off = None if tr0.off is None else torch.from_numpy(tr0.off.view(np.int64)).to(dev)
        lens = torch.from_numpy(tr0.len.view(np.int16)).to(dev)
        out = torch.zeros((n, 16), dtype=torch.uint8, device=dev)

        def load(t):
            blob.zero_()
            blob[:t.blob.size].copy_(torch.from_numpy(t.blob))
            lens.copy_(torch.from_numpy(t.len.view(np.int16)))
        load(tr0)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):  # first call outside capture: grows the flag buffer
            eng.batch_dev(blob.data_ptr(), None if off is None else off.data_ptr(), lens.data_ptr(), tr0.stride, n,
                          out.data_ptr(), None, s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            eng.batch_dev(blob.data_ptr(), None if off is None else off.data_ptr(), lens.data_ptr(), tr0.stride, n,
                          out.data_ptr(), None, s.cuda_stream)
        for t in traces_ + traces_[::-1]:
            load(t)
            out.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            er, _ = oracle.rx_trace(t, KEY, flags=flags, threads=8)
            _diff(out.cpu().numpy(), er, f"graph replay {kind}")
    finally:
        eng.close()


def test_hip_graph_replay_mode_change():
    """One captured launch over a fixed slot layout (u64 offsets, 1536-B
    slots) replayed over batches that the device-side sampler sends down
    different splits: 64-B frames (FAST), 1514-B frames (LONG), short
    option-laden / IPv6-free mixed frames (SHORT) and back. A replay reuses
    the captured class stamps, so a later replay can see classes a previous
    one deferred; every record must still be the oracle's."""
    import torch
    n, S = 12288, 1536
    kinds = ["tcp64", "tcp1514", "mixed", "tcp64", "imix", "tcp1514"]
    batches = []
    for k, kind in enumerate(kinds):
        t = traces.make_trace(kind, n, seed=0x1B7000 + k)
        offs = t.offsets().astype(np.int64)
        blob = np.zeros(n * S + 64, np.uint8)
        for i in range(n):
            L = int(t.len[i])
            blob[i * S:i * S + L] = t.blob[offs[i]:offs[i] + L]
        batches.append(traces.Trace(blob, np.arange(n, dtype=np.uint64) * S, t.len.copy(), 0))
    eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, 0))
    try:
        dev = torch.device("cuda:0")
        blob = torch.zeros(n * S + 64, dtype=torch.uint8, device=dev)
        off = torch.from_numpy(batches[0].off.view(np.int64)).to(dev)
        lens = torch.zeros(n, dtype=torch.int16, device=dev)
        out = torch.zeros((n, 16), dtype=torch.uint8, device=dev)

        def load(t):
            blob.copy_(torch.from_numpy(t.blob))
            lens.copy_(torch.from_numpy(t.len.view(np.int16)))
        load(batches[0])
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            eng.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), None,
                          s.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            eng.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), None,
                          s.cuda_stream)
        for kind, t in zip(kinds, batches):
            load(t)
            out.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            er, _ = oracle.rx_trace(t, KEY, threads=8)
            _diff(out.cpu().numpy(), er, f"graph replay, {kind} batch")
    finally:
        eng.close()


def test_mbufs_reject_oversized_len():
    """An IX mbuf holds at most 2048 data bytes (IXG_MBUF_DATA_LEN): a larger
    mbuf->len is -EINVAL, not a gather of the next mbuf's bytes."""
    tr = traces.make_trace("tcp64", 256, seed=0x1B7100)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        rec = eng.batch_mbufs(ptrs)
        er, _ = oracle.rx_trace(tr, KEY)
        _diff(rec, er, "mbufs")
        base = int(ptrs[37]) - arena.ctypes.data
        for bad in (2049, 4096, 0xffff, 1 << 40):
            arena[base:base + 8] = np.frombuffer(np.uint64(bad).tobytes(), np.uint8)
            with pytest.raises(RuntimeError, match="invalid argument"):
                eng.batch_mbufs(ptrs)
        arena[base:base + 8] = np.frombuffer(np.uint64(2048).tobytes(), np.uint8)
        eng.batch_mbufs(ptrs)  # the maximum itself is accepted
    finally:
        eng.close()


@pytest.mark.parametrize("kind,layout", [("tcp64", "stride"), ("tcp64", "packed"), ("imix", "packed"),
                                         ("mixed", "packed"), ("tcp1514", "stride")])
def test_fdir_vs_oracle(kind, layout, engines):
    """Flow-director filters over every kernel and layout: filters for a
    quarter of the batch's TCP flows (plus reverse-direction ones that must
    not match), checked against the oracle; then the filters are removed and
    the records are the plain RSS ones again."""
    import torch
    n = 20000
    tr = traces.make_trace(kind, n, seed=0x1B7200 + n, bad_ip=0.01, bad_l4=0.01)
    if layout == "packed" and tr.off is None:
        tr = traces.Trace(tr.blob, tr.offsets().copy(), tr.len, 0)
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    tcp = np.nonzero((b[offs + 12] == 8) & (b[offs + 13] == 0) & (b[offs + 23] == 6))[0]
    pick = tcp[::4]
    l4 = offs[pick] + 14 + 4 * (b[offs[pick] + 14] & 15).astype(np.int64)
    f = np.zeros(len(pick) * 2, ixgrx.FDIR_DTYPE)
    for k, (src, dst, sp, dp) in enumerate(((26, 30, 0, 2), (30, 26, 2, 0))):
        rows = f[k::2]
        rows["src_ip"] = b[(offs[pick] + src)[:, None] + np.arange(4)].view("<u4").reshape(-1)
        rows["dst_ip"] = b[(offs[pick] + dst)[:, None] + np.arange(4)].view("<u4").reshape(-1)
        rows["src_port"] = (b[l4 + sp].astype(np.uint16) << 8) | b[l4 + sp + 1]
        rows["dst_port"] = (b[l4 + dp].astype(np.uint16) << 8) | b[l4 + dp + 1]
    eng = engines()
    er, _ = oracle.rx_trace(tr, KEY, threads=8, fdir=f, cpu_id=9)
    assert ((er[:, 3] & 0x20) != 0).sum() >= len(pick) // 2
    eng.set_fdir(f, cpu_id=9)
    try:
        dev = torch.device("cuda:0")
        blob = torch.from_numpy(np.concatenate([tr.blob, np.zeros(64, np.uint8)])).to(dev)
        lens = torch.from_numpy(tr.len.view(np.int16)).to(dev)
        off = None if tr.off is None else torch.from_numpy(tr.off.view(np.int64)).to(dev)
        out = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
        eng.batch_dev(blob.data_ptr(), None if off is None else off.data_ptr(), lens.data_ptr(), tr.stride, n,
                      out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        _diff(out.cpu().numpy(), er, f"fdir {kind} {layout}")
    finally:
        eng.set_fdir(None)
    plain, _ = oracle.rx_trace(tr, KEY, threads=8)
    _diff(eng.batch_trace(tr), plain, f"fdir removed {kind} {layout}")



@pytest.mark.parametrize("layout", ["stride", "packed"])
def test_big_kernel_mixed_chunks(layout, engines):
    """The big-chunk kernel (LONG mode, most chunks big) takes the big chunks
    of IPv4 ihl 5 frames and flags the rest for the general kernel: chunks
    with an IPv4-options frame, with a short frame, with an IPv6 frame, with
    bad checksums, and a partial last chunk, all against the oracle."""
    rng = np.random.default_rng(0xB16)
    n_chunks = 96
    rows = [bytes(r) for r in traces.build_ipv4(rng, 64 * n_chunks, 1514, 6)]
    rows += [bytes(r) for r in traces.build_ipv4(rng, 37, 1000, 17)]  # partial last chunk (UDP)
    frames = list(rows)
    opt = [bytes(r) for r in traces.build_ipv4(rng, 8, 1514, 6, ihl=7)]
    for k in range(8):  # chunks 10..17: one IPv4-options frame each (big, not ihl 5)
        frames[64 * (10 + k) + 5 * k] = opt[k]
    for k in range(8):  # chunks 20..27: one short frame each (not big)
        frames[64 * (20 + k) + 3] = bytes(traces.build_ipv4(rng, 1, 60, 6)[0])
    for k in range(4):  # chunks 30..33: an IPv6 frame
        frames[64 * (30 + k) + 9] = mg.ipv6(payload=b"z" * 1400)
    for k in range(8):  # chunks 40..47: bad IP / L4 checksums
        f = bytearray(frames[64 * (40 + k) + k])
        f[24 if k % 2 else 60] ^= 1
        frames[64 * (40 + k) + k] = bytes(f)
    tr = traces.pack(frames, stride=1516) if layout == "stride" else traces.pack(frames)
    for flags in (0, ixgrx.IXG_F_IPV6):
        rec, cs = engines(flags=flags).batch_trace(tr, want_csum=True)
        er, ec = oracle.rx_trace(tr, KEY, flags=flags, threads=8)
        _diff(rec, er, f"big mixed {layout} flags={flags}")
        assert (cs == ec).all()
