"""The ring kernel (ixg_rx_ring_o): LONG-mode launches of
packed u64-offset batches in device memory, staged through a block-wide LDS
ring by a loader wave and consumed by the block's other waves.

Bit-exact against the oracle: the records and the residual words. Besides
IMIX batches of every size class (one chunk, a few chunks per block, enough
chunks per block that the ring wraps many times), the cases that must leave
chunks to the long kernel behind it: spans past the ring's per-chunk limit,
offsets out of order, frames outside their chunk's span; arrays the ring
cannot DMA (not 16-byte aligned: the ring is skipped); launches that switch
between the ring and the other plans on one context and in one HIP graph.
`launch_info` confirms which plan the device chose, so a test of the ring
fails if the ring did not run.
"""
import numpy as np
import pytest

from ix_amd import ixgrx, traces
from oracle import oracle

pytestmark = pytest.mark.gpu

KEY = traces.RSS_KEY


def _diff(got, exp, what):
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} records differ; first {bad[:6].tolist()}: " \
                          f"gpu {got[bad[0]].tolist()} vs exp {exp[bad[0]].tolist()}"


@pytest.fixture(scope="module")
def eng():
    cache = {}

    def get(flags=0):
        if flags not in cache:
            cache[flags] = ixgrx.RxEngine(ixgrx.Config(KEY, 128, 0, flags))
        return cache[flags]
    yield get
    for e in cache.values():
        e.close()


def _run(e, blob, off, lens, mis=(0, 0, 0)):
    """One device-resident launch; mis = byte misalignment of (frames,
    offsets, lengths) against 16-byte boundaries (0 = aligned)."""
    import torch
    dev = torch.device("cuda:0")
    n = int(lens.shape[0])
    b = torch.zeros(blob.size + 64 + 16, dtype=torch.uint8, device=dev)
    b[mis[0]:mis[0] + blob.size] = torch.from_numpy(np.ascontiguousarray(blob))
    o = torch.zeros(n * 8 + 16, dtype=torch.uint8, device=dev)
    o[mis[1]:mis[1] + n * 8] = torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.uint8))
    ln = torch.zeros(n * 2 + 16, dtype=torch.uint8, device=dev)
    ln[mis[2]:mis[2] + n * 2] = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint16).view(np.uint8))
    out = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=dev)
    cs = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    e.batch_dev(b.data_ptr() + mis[0], o.data_ptr() + mis[1], ln.data_ptr() + mis[2], 0, n, out.data_ptr(),
                cs.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out[:n].cpu().numpy(), cs[:n].cpu().numpy().view(np.uint32), e.launch_info()


def _check(e, tr, flags, what, expect_ring=True, mis=(0, 0, 0), off=None, lens=None):
    off = tr.offsets() if off is None else off
    lens = tr.len if lens is None else lens
    rec, cs, info = _run(e, tr.blob, off, lens, mis)
    er, ec = oracle.rx_batch(KEY, 128, 0, flags, tr.blob, off, lens)
    _diff(rec, er, what)
    assert (cs == ec).all(), f"{what}: residuals differ"
    if expect_ring is not None:
        assert info["ring"] == expect_ring, f"{what}: launch plan {info}"
    return info


@pytest.mark.parametrize("n", [64, 1000, 64 * 257 + 5, 64 * 256 * 24 + 37])
@pytest.mark.parametrize("flags", [0, ixgrx.IXG_F_NO_CSUM_DROP, ixgrx.IXG_F_IPV6])
def test_ring_imix_sizes(eng, n, flags):
    """IMIX (C3's mix, 1 % bad IP / L4 checksums): one chunk; a few chunks
    per block; more than 24 chunks per block (the ring wraps several times
    per block)."""
    tr = traces.make_trace("imix", n, seed=0x1B5000 + n + flags, bad_ip=0.01, bad_l4=0.01)
    info = _check(eng(flags), tr, flags, f"imix n={n} flags={flags}")
    assert info["mode"] == "long"


def test_ring_fuzz_in_long_chunks(eng):
    """Every header shape the reference handles (the fuzz and edge frames of
    the golden builder: options, fragments, ICMP, UDP, truncations, IPv6,
    non-IP) spread one per chunk among long IMIX frames, so each chunk goes
    through the ring's tail sums and the full parse."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as mg
    rng = np.random.default_rng(7)
    odd = mg.fuzz_frames(rng, 3000) + mg.edge_frames()
    base = traces.make_trace("imix", 64 * len(odd), seed=8, bad_ip=0.02, bad_l4=0.02)
    frames = []
    offs, lens = base.offsets(), base.len
    for k, f in enumerate(odd):
        for j in range(63):
            i = 63 * k + j
            frames.append(bytes(base.blob[offs[i]:offs[i] + lens[i]]))
        frames.append(f)
    tr = traces.pack(frames)
    for flags in (0, ixgrx.IXG_F_IPV6, ixgrx.IXG_F_NO_CSUM_DROP):
        _check(eng(flags), tr, flags, f"fuzz in long chunks flags={flags}")


def test_ring_spans_past_the_limit(eng):
    """Chunks whose span exceeds the ring's per-chunk limit (40 KiB: 30
    1514-B frames and 34 short ones) between ordinary IMIX chunks: those are
    left to the long kernel, the others go through the ring."""
    rng = np.random.default_rng(11)
    im = traces.make_trace("imix", 64 * 600, seed=12)
    big = traces.make_trace("tcp1514", 64 * 600, seed=13)
    small = traces.make_trace("tcp64", 64 * 600, seed=14)
    frames = []
    for c in range(600):
        if c % 3 == 1:
            pick = rng.permutation(64) < 30
            for j in range(64):
                src = big if pick[j] else small
                i = 64 * c + j
                o = int(src.offsets()[i])
                frames.append(bytes(src.blob[o:o + int(src.len[i])]))
        else:
            for j in range(64):
                i = 64 * c + j
                o = int(im.offsets()[i])
                frames.append(bytes(im.blob[o:o + int(im.len[i])]))
    tr = traces.pack(frames)
    _check(eng(), tr, 0, "spans past the limit")


def test_ring_unordered_offsets(eng):
    """Offsets out of order: a third of the chunks reversed, some frames
    swapped across chunks (a frame outside its chunk's span), the rest
    packed. The ring must leave every such chunk to the long kernel."""
    tr = traces.make_trace("imix", 64 * 2000, seed=15, bad_ip=0.01, bad_l4=0.01)
    off = tr.offsets().copy()
    lens = tr.len.copy()
    rng = np.random.default_rng(16)
    for c in range(0, 2000, 3):
        sl = slice(64 * c, 64 * c + 64)
        off[sl] = off[sl][::-1].copy()
        lens[sl] = lens[sl][::-1].copy()
    for _ in range(100):
        a, b = rng.integers(0, tr.n, 2)
        off[[a, b]] = off[[b, a]]
        lens[[a, b]] = lens[[b, a]]
    _check(eng(), tr, 0, "unordered", off=off, lens=lens)


@pytest.mark.parametrize("mis", [(4, 0, 0), (0, 8, 0), (0, 0, 2)])
def test_ring_skipped_for_unaligned_arrays(eng, mis):
    """The ring DMAs 16-byte pieces of the frames, offsets and lengths: any of
    the three not 16-byte aligned and the launch keeps the long kernel."""
    tr = traces.make_trace("imix", 64 * 300, seed=17)
    info = _check(eng(), tr, 0, f"unaligned {mis}", expect_ring=False, mis=mis)
    assert info["mode"] == "long"


def test_ring_back_to_back_plans(eng):
    """One context, launches switching plans: ring (IMIX), short (mixed),
    big chunks (1514-B in the offset layout: the long kernel, strided), ring
    again; each against the oracle (the ring writes every chunk's flag and
    resets its stamp when it does not run, so nothing stale leaks into the
    next launch)."""
    e = eng()
    im = traces.make_trace("imix", 64 * 900, seed=18, bad_ip=0.01, bad_l4=0.01)
    mx = traces.make_trace("mixed", 64 * 900, seed=19)
    bg = traces.make_trace("tcp1514", 64 * 400, seed=20)
    bgo = traces.Trace(bg.blob, bg.offsets().copy(), bg.len, 0)
    for tr, ring in ((im, True), (mx, False), (bgo, False), (im, True), (bgo, False)):
        _check(e, tr, 0, f"back to back {tr.n}", expect_ring=ring)


def test_ring_graph_replay(eng):
    """A captured launch replayed over different batches of the same shape,
    one of them big chunks (the ring exits, the long kernel takes all): the
    stamps the kernels read at replay time decide the plan."""
    import torch
    e = eng()
    n = 64 * 800
    trs = [traces.make_trace("imix", n, seed=21), traces.make_trace("imix", n, seed=22)]
    bg = traces.make_trace("tcp1514", n, seed=23)
    dev = torch.device("cuda:0")
    size = max(int(t.offsets()[-1]) + int(t.len[-1]) for t in trs + [bg]) + 4096
    blob = torch.zeros(size, dtype=torch.uint8, device=dev)
    off = torch.zeros(n, dtype=torch.int64, device=dev)
    lens = torch.zeros(n, dtype=torch.int16, device=dev)
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)

    def load(t):
        blob.zero_()
        blob[:t.blob.size] = torch.from_numpy(t.blob)
        off.copy_(torch.from_numpy(t.offsets().astype(np.int64)))
        lens.copy_(torch.from_numpy(t.len.view(np.int16)))
    s = torch.cuda.Stream()
    load(trs[0])
    torch.cuda.synchronize()
    e.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), None, s.cuda_stream)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        e.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), None, s.cuda_stream)
    for t in (trs[1], bg, trs[0], bg, trs[1]):
        load(t)
        out.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        er, _ = oracle.rx_batch(KEY, 128, 0, 0, t.blob, t.offsets(), t.len)
        _diff(out.cpu().numpy(), er, f"graph replay n={n}")


def test_ring_c3_full_size_tiled(eng):
    """C3 at full size (16M IMIX frames, 6 GB): the pool's records tiled,
    the first repetition against the oracle, through the ring."""
    import torch
    n, pool = 16 * 1024 * 1024, 1 << 16
    tr = traces.make_trace("imix", pool, seed=24, bad_ip=0.01, bad_l4=0.01)
    reps = n // pool
    dev = torch.device("cuda:0")
    span = int(tr.off[-1]) + ((int(tr.len[-1]) + 3) // 4) * 4
    blob = torch.zeros(reps * span + 4096, dtype=torch.uint8, device=dev)
    blob[:reps * span].view(reps, span).copy_(torch.from_numpy(tr.blob[:span]).to(dev).unsqueeze(0).expand(reps, -1))
    o = torch.from_numpy(tr.off.view(np.int64)).to(dev)
    off = (o.unsqueeze(0) + torch.arange(reps, device=dev).unsqueeze(1) * span).reshape(-1).contiguous()
    lens = torch.from_numpy(tr.len.view(np.int16)).to(dev).repeat(reps).contiguous()
    out = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    try:
        e = eng()
        e.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, out.data_ptr(), None,
                    torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert e.launch_info()["ring"]
        v = out.view(reps, pool, 16)
        assert bool(torch.equal(v, v[:1].expand(reps, -1, -1))), "tiled records differ"
        er, _ = oracle.rx_trace(tr, KEY, threads=8, hash_mode=oracle.HASH_TABLE)
        _diff(v[0].cpu().numpy(), er, "C3 full size, first repetition")
    finally:
        del blob, off, lens, out
        torch.cuda.empty_cache()
