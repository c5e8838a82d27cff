"""The long kernel's flat walk (ixg_rx_glong_*): a chunk whose
64 frames lie in ascending order in one span of at most 30 KiB is streamed
as 1-KiB rows, its tails summed through prefix sums over the span; every
other chunk takes the per-lane fallback (or, when most sampled chunks are big,
the per-segment walk). These cases steer chunks down each branch and at the
edges of the prefix-sum arithmetic; every record is compared bit-exactly with
the oracle (dp/net + dp/lwip restated, pinned to the reference's goldens).
"""
import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

pytestmark = pytest.mark.gpu

KEY = traces.RSS_KEY


def _check(tr, flags=0, splits=("auto", "long")):
    er, _ = oracle.rx_trace(tr, KEY, flags=flags, threads=8)
    for sp in splits:
        eng = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, flags), split=sp)
        try:
            rec = eng.batch_trace(tr).view(np.uint8).reshape(-1, 16)
        finally:
            eng.close()
        bad = np.nonzero((rec != er).any(axis=1))[0]
        assert bad.size == 0, f"split {sp}: {bad.size} records differ, first {bad[:6].tolist()}: " \
                              f"{rec[bad[0]].tolist()} vs {er[bad[0]].tolist()}"
    return er


def _frames(rng, lens, proto=6):
    out = []
    for L in lens:
        out.append(bytes(traces.build_ipv4(rng, 1, int(L), proto)[0]))
    return out


def test_spans_around_the_limit():
    """Chunks of 1514-B and 60-B frames whose spans fall just under and just
    over 30 KiB (flat, then the fallback), in one wave's run of chunks, with
    bad checksums in the tails of some."""
    rng = np.random.default_rng(0xF1A7)
    lens = []
    for k in range(96):
        big = 16 + (k % 8)  # 16..23 frames of 1514 B per chunk: spans ~26..37 KiB
        c = [1514] * big + [60] * (64 - big)
        rng.shuffle(c)
        lens += c
    frames = _frames(rng, lens)
    big_i = [i for i, f in enumerate(frames) if len(f) > 200]
    for i in rng.choice(big_i, 300, replace=False):
        f = bytearray(frames[i])
        f[int(rng.integers(100, len(f)))] ^= 0x40  # a tail byte: the L4 checksum fails
        frames[i] = bytes(f)
    er = _check(traces.pack(frames))
    assert (er[:, 2] == ixgrx.V["DROP_CSUM_L4"]).sum() > 100


def test_frames_out_of_order():
    """Offsets permuted within each pair of chunks: no chunk is flat."""
    rng = np.random.default_rng(0xF1A8)
    tr = traces.make_trace("imix", 128 * 40, seed=0xF1A8, bad_ip=0.02, bad_l4=0.02)
    perm = np.concatenate([128 * k + rng.permutation(128) for k in range(40)])
    tr2 = traces.Trace(blob=tr.blob, off=tr.off[perm].copy(), len=tr.len[perm].copy(), stride=0)
    _check(tr2)


def test_gaps_between_frames():
    """Packed frames with gaps of random bytes between them (still ascending:
    flat as long as the span fits), tails summed across the gaps."""
    rng = np.random.default_rng(0xF1A9)
    tr = traces.make_trace("imix", 64 * 60, seed=0xF1A9, bad_l4=0.03)
    frames = [tr.frame(i) for i in range(tr.n)]
    off = np.zeros(len(frames), np.uint64)
    pos = 16
    for i, f in enumerate(frames):
        pos += 4 * int(rng.integers(0, 24))
        off[i] = pos
        pos += (len(f) + 3) & ~3
    blob = rng.integers(0, 256, pos + 256, dtype=np.uint8)
    for i, f in enumerate(frames):
        blob[int(off[i]):int(off[i]) + len(f)] = np.frombuffer(f, np.uint8)
    _check(traces.Trace(blob=blob, off=off, len=tr.len.copy(), stride=0))


def test_segments_ending_short_of_the_frame():
    """IPv4 total lengths cut 17..300 bytes short of the frame (the segment
    ends in another piece than the frame: its end piece is loaded on its own),
    and by 1..16 bytes (the same piece)."""
    rng = np.random.default_rng(0xF1AA)
    lens = rng.choice([200, 300, 590, 600], 64 * 50)
    frames = []
    for k, L in enumerate(lens):
        cut = int(rng.integers(1, 17)) if rng.random() < 0.5 else int(rng.integers(17, min(301, int(L) - 80)))
        f = traces.build_ipv4(rng, 1, int(L) - cut, 6)[0]  # valid sums over ip_len = L - cut - 14
        if k % 4 == 0:
            f[int(rng.integers(60, len(f)))] ^= 0x08  # a payload byte: DROP_CSUM_L4
        frames.append(bytes(f) + bytes(rng.integers(0, 256, cut, dtype=np.uint8)))
    er = _check(traces.pack(frames))
    assert (er[:, 2] == ixgrx.V["DROP_CSUM_L4"]).sum() > 600
    assert (er[:, 2] == ixgrx.V["DROP_CSUM_L4"]).sum() < 1000


def test_icmp_messages_of_zero_bytes():
    """ICMP messages longer than the 96-byte prefix whose bytes are all zero:
    the tail's prefix-sum difference is the negative zero, which must not
    pass for the checksum of a message that sums to 0 (chksum_internet
    0xffff: DROP_ICMP_CSUM, dp/net/icmp.c:82)."""
    rng = np.random.default_rng(0xF1AB)
    frames = []
    for k in range(64 * 30):
        L = int(rng.integers(120, 700))
        f = np.zeros(L, np.uint8)
        f[12], f[13], f[14] = 0x08, 0x00, 0x45
        ip_len = L - 14
        f[16], f[17] = ip_len >> 8, ip_len & 0xFF
        f[22], f[23] = 64, 1  # ttl, ICMP
        f[26:34] = rng.integers(0, 256, 8, dtype=np.uint8)
        s = int(sum((int(f[i]) << 8) | int(f[i + 1]) for i in range(14, 34, 2)))
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        ck = (~s) & 0xFFFF
        f[24], f[25] = ck >> 8, ck & 0xFF
        if k % 3 == 0:  # some echo requests with valid checksums among them
            f = np.frombuffer(traces.icmp_echo(rng, L - 42), np.uint8)
        frames.append(bytes(f))
    er = _check(traces.pack(frames))
    assert (er[:, 2] == ixgrx.V["DROP_ICMP_CSUM"]).sum() > 1000
    assert (er[:, 2] == ixgrx.V["ICMP_ECHO"]).sum() > 400


@pytest.mark.parametrize("seed", [1, 2])
def test_imix_large_vs_oracle(seed):
    """A full IMIX batch (several waves' runs of chunks, ~1.5 % of chunks
    over 30 KiB) with 1 % bad checksums."""
    tr = traces.make_trace("imix", 400000, seed=0xF1B0 + seed, bad_ip=0.01, bad_l4=0.01)
    _check(tr, splits=("auto",))
