"""The rest of the tcp_input head (dp/net/tcp_in.c:230-241):
seqno / ackno / wnd / tcplen and the ports in host order, per frame
(struct ixg_tcp_ext), and the in-place header conversion (IXG_TCPX_INPLACE).

The golden fixtures' `tcpx` / `tcpx_hdr` come from the reference's own
tcp_input, compiled from dp/net/tcp_in.c and run over every TCP segment with
empty PCB lists (oracle/ref_harness/ref_tcphead.c): its LWIP_Context fields
as tcp_rst received them and the header bytes as it converted them in place.
The oracle is pinned to those; the HIP kernel (ixg_tcp_ext_batch_dev) is
checked against the goldens and the oracle on the GPU.
"""
import numpy as np
import pytest

from ix_amd import traces
from oracle import oracle

TCP, TCP6 = 0x01, 0x05
INPLACE = 1


def _l4(golden):
    """Each frame's TCP header offset (valid for TCP / TCP6 records)."""
    v = golden["rec"][:, 2]
    off = golden["off"].astype(np.int64)
    ihl = golden["blob"][np.minimum(off + 14, golden["blob"].size - 1)] & 15
    return np.where(v == TCP6, 54, 14 + 4 * ihl.astype(np.int64)), v


def test_oracle_ext_matches_reference(golden):
    ext, _ = oracle.tcp_ext_batch(golden["blob"], golden["off"], 0, golden["rec"].view(np.uint8))
    exp = golden["tcpx"]
    bad = np.nonzero((ext != exp).any(axis=1))[0]
    assert bad.size == 0, f"{golden['name']}: {bad.size} ext records differ, first {bad[:8]}: " \
                          f"{ext[bad[0]].tolist()} vs {exp[bad[0]].tolist()}"
    v = golden["rec"][:, 2]
    tcp = (v == TCP) | (v == TCP6)
    assert (exp[~tcp] == 0).all()
    assert tcp.sum() > 0


def test_oracle_inplace_matches_reference(golden):
    _, b = oracle.tcp_ext_batch(golden["blob"], golden["off"], 0, golden["rec"].view(np.uint8), flags=INPLACE)
    l4, v = _l4(golden)
    off = golden["off"].astype(np.int64)
    tcp = np.nonzero((v == TCP) | (v == TCP6))[0]
    for i in tcp:
        s = int(off[i] + l4[i])
        assert bytes(b[s:s + 16]) == bytes(golden["tcpx_hdr"][i]), f"{golden['name']} frame {i}"
    # nothing else changed
    mask = np.ones(b.size, bool)
    for i in tcp:
        s = int(off[i] + l4[i])
        mask[s:s + 16] = False
    assert (b[mask] == golden["blob"][mask]).all()


def test_reference_ext_fields_are_the_head(golden):
    """Cross-check of the fixture itself: the ports and tcplen agree with the
    RX record (the reference's tcp_to_idx bucket and doff strip)."""
    v = golden["rec"][:, 2]
    tcp = (v == TCP) | (v == TCP6)
    x = golden["tcpx"][tcp].view(oracle.TCPX_DTYPE).reshape(-1)
    r = golden["rec"][tcp]
    l4len = r[:, 6].astype(np.int64) | (r[:, 7].astype(np.int64) << 8)
    fin_syn = (r[:, 14] & 3) != 0
    assert ((l4len + fin_syn) & 0xffff == x["tcplen"]).all()


def test_oracle_ext_synthetic_traces():
    """Strided C2-shaped frames: the ext of every frame equals the header
    fields read directly."""
    tr = traces.make_trace("tcp64", 512, seed=7)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY, 128, 0, 0)
    ext, _ = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, rec)
    x = ext.view(oracle.TCPX_DTYPE).reshape(-1)
    assert (rec[:, 2] == TCP).all()
    for i in range(0, tr.n, 37):
        f = tr.blob[i * tr.stride:]
        assert x["seqno"][i] == int.from_bytes(bytes(f[38:42]), "big")
        assert x["ackno"][i] == int.from_bytes(bytes(f[42:46]), "big")
        assert x["wnd"][i] == int.from_bytes(bytes(f[48:50]), "big")
        assert x["src_port"][i] == int.from_bytes(bytes(f[34:36]), "big")


@pytest.mark.parametrize("n", [0, 1])
def test_oracle_ext_empty_and_single(n):
    tr = traces.make_trace("tcp64", max(n, 1), seed=3)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY, 128, 0, 0)
    ext, _ = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, rec[:n])
    assert ext.shape == (n, 16)


# ---------------------------------------------------------------- GPU

def _dev_run(eng, blob, off, stride, rec_u8, flags=0):
    """Upload frames and records, run ixg_tcp_ext_batch_dev, return (ext, frames after)."""
    import torch
    from ix_amd import tcpx
    dev = torch.device("cuda", 0)
    n = int(rec_u8.shape[0])
    b = torch.from_numpy(np.ascontiguousarray(blob, dtype=np.uint8).copy()).to(dev)
    o = None if off is None else torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).to(dev)
    r = torch.from_numpy(np.ascontiguousarray(rec_u8, dtype=np.uint8).reshape(-1)).to(dev)
    ext = torch.full((max(n, 1), 16), 0xA5, dtype=torch.uint8, device=dev)
    tcpx.batch_dev(eng, b.data_ptr(), None if o is None else o.data_ptr(), stride, r.data_ptr(), n,
                   ext.data_ptr(), flags, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return ext[:n].cpu().numpy(), b.cpu().numpy()


@pytest.fixture(scope="module")
def gpu_engine():
    from ix_amd import ixgrx
    e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, 0))
    yield e
    e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, INPLACE])
def test_gpu_ext_matches_reference(golden, gpu_engine, flags):
    ext, b = _dev_run(gpu_engine, golden["blob"], golden["off"], 0, golden["rec"], flags)
    bad = np.nonzero((ext != golden["tcpx"]).any(axis=1))[0]
    assert bad.size == 0, f"{golden['name']}: {bad.size} differ, first {bad[:6].tolist()}: " \
                          f"{ext[bad[0]].tolist()} vs {golden['tcpx'][bad[0]].tolist()}"
    _, eb = oracle.tcp_ext_batch(golden["blob"], golden["off"], 0, golden["rec"], flags)
    assert (b[:eb.size] == eb).all(), "frames after the kernel differ from the reference's in-place conversion"


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,flags", [("tcp64", 100000, 0), ("imix", 40000, 0), ("mixed", 40000, 2),
                                          ("tcp64opt", 30000, 0), ("tcp1514", 4000, 0)])
def test_gpu_ext_after_gpu_rx(kind, n, flags, gpu_engine):
    """RX on the device, then the head's rest on the device, vs the oracle
    (both steps), IPv4 options and the IPv6 extension included."""
    from ix_amd import ixgrx
    tr = traces.make_trace(kind, n, seed=0x7C0 + n, bad_ip=0.01, bad_l4=0.01)
    eng = gpu_engine if flags == 0 else ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, 128, 0, flags))
    try:
        rec = eng.batch_trace(tr).view(np.uint8).reshape(-1, 16)
        er, _ = oracle.rx_trace(tr, traces.RSS_KEY, flags=flags, threads=8)
        assert (rec == er).all()
        for fl in (0, INPLACE):
            ext, b = _dev_run(eng, tr.blob, tr.off, tr.stride, rec, fl)
            eext, eb = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, er, fl)
            assert (ext == eext).all(), kind
            assert (b == eb).all(), kind
            v = rec[:, 2]
            assert ((ext != 0).any(1) == ((v == TCP) | (v == TCP6))).all()
    finally:
        if eng is not gpu_engine:
            eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 65, 257])
def test_gpu_ext_ragged(n, gpu_engine):
    tr = traces.make_trace("imix", max(n, 1), seed=0x7D0 + n)
    er, _ = oracle.rx_trace(tr, traces.RSS_KEY)
    ext, _ = _dev_run(gpu_engine, tr.blob, tr.off, tr.stride, er[:n])
    eext, _ = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, er[:n])
    assert ext.shape == (n, 16) and (ext == eext).all()


@pytest.mark.gpu
def test_gpu_ext_rejects_bad_arguments(gpu_engine):
    import ctypes
    from ix_amd import ixgrx, tcpx
    lib = tcpx._bind(gpu_engine._lib)
    fr = ixgrx.RxFrames(16, None, 0, 60, 0)
    assert lib.ixg_tcp_ext_batch_dev(gpu_engine._ctx, ctypes.byref(fr), 16, 4, 16, 2, None) == -22  # bad flag
    fr = ixgrx.RxFrames(18, None, 0, 60, 0)
    assert lib.ixg_tcp_ext_batch_dev(gpu_engine._ctx, ctypes.byref(fr), 16, 4, 16, 0, None) == -22  # base align
    fr = ixgrx.RxFrames(16, None, 0, 62, 0)
    assert lib.ixg_tcp_ext_batch_dev(gpu_engine._ctx, ctypes.byref(fr), 16, 4, 16, 0, None) == -22  # stride


def test_oracle_ext_vs_reference_fresh_fuzz():
    """Fresh fuzz frames (mutated seq/ack/flags/doff fields) through the
    reference's own tcp_input head, where the harness is built (this
    container; make -C oracle ref): the oracle agrees on every frame, and
    the harness's own cross-checks (pass/drop, tcp_rst arguments) hold."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "golden"))
    import make_golden as mg
    if not os.path.exists(mg.HARNESS):
        pytest.skip("reference harness not built")
    rng = np.random.default_rng(0x7C5)
    frames = mg.fuzz_frames(rng, 2000) + mg.edge_frames()
    for flags in (0, 1):  # NO_CSUM_DROP: bad-checksum TCP frames reach tcp_input too
        rec, _, tcpx, hdr = mg.run_ref(frames, traces.RSS_KEY, 128, 0, flags, full=True)
        tr = traces.pack(frames)
        ext, b = oracle.tcp_ext_batch(tr.blob, tr.off, 0, rec, INPLACE)
        assert (ext == tcpx).all()
        v = rec[:, 2]
        tcp = np.nonzero(v == TCP)[0]
        assert tcp.size > 200
        ihl = tr.blob[tr.off.astype(np.int64) + 14] & 15
        for i in tcp:
            s = int(tr.off[i]) + 14 + 4 * int(ihl[i])
            assert bytes(b[s:s + 16]) == bytes(hdr[i])


# ---------------------------------------------------------------- fused RX + head (ixg_rx_tcpx_batch_dev)

def _fused_run(eng, blob, off, lens, stride, flags=0):
    """Upload a batch, run ixg_rx_tcpx_batch_dev, return (records, ext, frames after)."""
    import torch
    from ix_amd import ixgrx, tcpx
    dev = torch.device("cuda", 0)
    n = int(lens.shape[0])
    b = torch.from_numpy(np.concatenate([np.ascontiguousarray(blob, dtype=np.uint8),
                                         np.zeros(ixgrx.IXG_TAIL_PAD, np.uint8)])).to(dev)
    o = None if off is None else torch.from_numpy(np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)).to(dev)
    ln = torch.from_numpy(np.ascontiguousarray(lens, dtype=np.uint16).view(np.int16)).to(dev)
    rec = torch.full((max(n, 1), 16), 0x5A, dtype=torch.uint8, device=dev)
    ext = torch.full((max(n, 1), 16), 0xA5, dtype=torch.uint8, device=dev)
    tcpx.rx_batch_dev(eng, b.data_ptr(), None if o is None else o.data_ptr(), ln.data_ptr(), stride, n,
                      rec.data_ptr(), ext.data_ptr(), flags, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return rec[:n].cpu().numpy(), ext[:n].cpu().numpy(), b.cpu().numpy()[:blob.size]


def _golden_engine(g):
    from ix_amd import ixgrx
    eng = ixgrx.RxEngine(ixgrx.Config(bytes(g["key"]), int(g["nb_rx_fgs"]), int(g["dev_idx"]), int(g["flags"])))
    if "fdir" in g:
        eng.set_fdir(np.ascontiguousarray(g["fdir"]).view(ixgrx.FDIR_DTYPE).reshape(-1), int(g["fdir_cpu"]))
    return eng


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [60, 64])
@pytest.mark.parametrize("flags", [0, INPLACE])
def test_gpu_fused_golden_fixed_stride(golden, stride, flags):
    """the golden frames of at most `stride` bytes (every
    edge case of the fixture that fits a 64-byte slot: bad checksums, IP
    options, short segments, drops) in one coalesced fixed-stride batch, so
    the fused coalesced kernel takes them (its lean, fixed-shape and
    general-parse chunks): records against the reference's, ext against its
    tcp_input's LWIP_Context fields (`tcpx`), frames after against its
    in-place conversion (`tcpx_hdr`)."""
    sel = np.nonzero(golden["len"].astype(np.int64) <= stride)[0]
    if sel.size == 0:
        pytest.skip("no frame fits the stride")
    # repeated so the batch spans many chunks and waves, with a ragged end
    reps = max(1, 5000 // sel.size)
    idx = np.tile(sel, reps)[:max(sel.size, min(5000, sel.size * reps) - 17)]
    n = idx.size
    blob = np.zeros(n * stride + 64, np.uint8)
    offs = golden["off"].astype(np.int64)
    lens = golden["len"].astype(np.int64)
    for k, i in enumerate(idx):
        blob[k * stride:k * stride + lens[i]] = golden["blob"][offs[i]:offs[i] + lens[i]]
    eng = _golden_engine(golden)
    try:
        rec, ext, after = _fused_run(eng, blob, None, lens[idx].astype(np.uint16), stride, flags)
    finally:
        eng.close()
    bad = np.nonzero((rec != golden["rec"][idx]).any(axis=1))[0]
    assert bad.size == 0, f"{golden['name']}: {bad.size} records differ, first {bad[:6].tolist()}"
    bad = np.nonzero((ext != golden["tcpx"][idx]).any(axis=1))[0]
    assert bad.size == 0, f"{golden['name']}: {bad.size} ext differ, first {bad[:6].tolist()}: " \
                          f"{ext[bad[0]].tolist()} vs {golden['tcpx'][idx[bad[0]]].tolist()}"
    _, eb = oracle.tcp_ext_batch(blob, None, stride, golden["rec"][idx], flags)
    assert (after == eb[:after.size]).all(), "frames after the fused kernel differ from the in-place conversion"
    if flags:
        l4, v = _l4(golden)
        for k, i in enumerate(idx[:2000]):
            if v[i] in (TCP, TCP6):
                s = k * stride + int(l4[i])
                assert bytes(after[s:s + 16]) == bytes(golden["tcpx_hdr"][i]), (golden["name"], k)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,stride", [("tcp64", 300000, 60), ("tcp64", 70000, 64), ("tcp64opt", 30000, 64),
                                           ("imix", 40000, 0), ("mixed", 20000, 0), ("tcp1514", 3000, 0)])
@pytest.mark.parametrize("flags", [0, INPLACE])
def test_gpu_fused_vs_oracle(kind, n, stride, flags):
    """Synthetic traces, 1 % bad checksums: C2's shape (stride 60, the fused
    kernel's lean path), stride 64, IP options in 64-byte slots (the fused
    kernel's general-parse chunks), and the layouts the fused kernel does not
    take (u64 offsets: RX, then the separate pass): records, ext and frames
    bit-exact against the oracle."""
    from ix_amd import ixgrx
    tr = traces.make_trace(kind, n, seed=0x7E0 + n, bad_ip=0.01, bad_l4=0.01)
    if stride and tr.stride != stride:
        frames = [tr.frame(i) for i in range(tr.n)]
        assert max(len(f) for f in frames) <= stride
        tr = traces.pack(frames, stride=stride)
    er, _ = oracle.rx_trace(tr, traces.RSS_KEY, threads=8)
    eext, eb = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, er, flags)
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY))
    try:
        rec, ext, after = _fused_run(eng, tr.blob, None if tr.stride else tr.off, tr.len, tr.stride, flags)
    finally:
        eng.close()
    assert (rec == er).all(), kind
    bad = np.nonzero((ext != eext).any(axis=1))[0]
    assert bad.size == 0, f"{kind}: {bad.size} ext differ, first {bad[:6].tolist()}"
    assert (after == eb[:after.size]).all(), kind


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 257, 4097])
def test_gpu_fused_ragged(n):
    from ix_amd import ixgrx
    tr = traces.make_trace("tcp64", n, seed=0x7F0 + n, bad_ip=0.05, bad_l4=0.05)
    er, _ = oracle.rx_trace(tr, traces.RSS_KEY)
    eext, _ = oracle.tcp_ext_batch(tr.blob, tr.off, tr.stride, er)
    eng = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY))
    try:
        rec, ext, _ = _fused_run(eng, tr.blob, None, tr.len, tr.stride)
    finally:
        eng.close()
    assert (rec == er).all() and (ext == eext).all()
