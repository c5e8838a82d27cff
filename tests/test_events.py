"""Event records: the usys descriptors of udp_input and
recv_a_pbuf for a batch.

CPU: the oracle (oracle/ixgrx_oracle.c ixgo_ev_batch) against the golden
descriptors written by the reference's own usys_udp_recv / usys_tcp_recv and
mempool_pagemem_to_iomap (tests/golden/ev.npz, make_golden_ev.py), including
udp_input's ip_tuple writes.
GPU: ixg_ev_batch_dev (through the C ABI) against the same fixtures, and
against the oracle on a full RX -> demux -> events pipeline over IMIX
traffic (TCP with payloads and UDP), ragged sizes and stride layouts.
"""
import os

import numpy as np
import pytest

from ix_amd import demux, events, ixgrx, traces
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
CASES = [("rx", "default", False), ("dmx", "demux_default", True)]


def _case(tag, name, with_dmx):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    e = np.load(os.path.join(GOLD, "ev.npz"), allow_pickle=False)
    dmx = z["demux"] if with_dmx else None
    pcbs = e[tag + "_pcbs"]
    exp_blob = z["blob"].copy()
    exp_blob[e[tag + "_tuple_pos"]] = e[tag + "_tuple_val"]
    return z, dmx, pcbs, int(e[tag + "_iomap"]), e[tag + "_ev"], e[tag + "_idx"], exp_blob


@pytest.mark.parametrize("tag,name,with_dmx", CASES)
def test_oracle_matches_reference(tag, name, with_dmx):
    z, dmx, pcbs, io, exp_ev, exp_idx, exp_blob = _case(tag, name, with_dmx)
    ev, idx, blob = oracle.ev_batch(z["blob"], z["off"], 0, z["rec"], dmx, pcbs, io, events.IXG_EV_UDP_TUPLE)
    assert ev.dtype.itemsize == 40 and len(ev) == len(exp_ev)
    assert (ev.view(np.uint8) == exp_ev.view(np.uint8)).all()
    assert (idx == exp_idx).all()
    assert (blob == exp_blob).all()


def test_fixture_covers_both_kinds():
    e = np.load(os.path.join(GOLD, "ev.npz"), allow_pickle=False)
    assert (e["rx_ev"]["sysnr"] == events.USYS_UDP_RECV).sum() > 100
    assert (e["dmx_ev"]["sysnr"] == events.USYS_TCP_RECV).sum() > 10


# ---- GPU ------------------------------------------------------------------

@pytest.fixture(scope="module")
def eng():
    e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY))
    yield e
    e.close()


def _run_dev(eng, blob, off, stride, rec, dmx, pcbs, n, io, flags):
    import torch
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
    to = None if off is None else torch.from_numpy(np.ascontiguousarray(off).view(np.int64)).to(dev)
    tr = torch.from_numpy(np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)).to(dev)
    td = None if dmx is None else torch.from_numpy(np.ascontiguousarray(dmx).view(np.uint8).reshape(n, 8)).to(dev)
    tp = None if pcbs is None or len(pcbs) == 0 else torch.from_numpy(pcbs.view(np.uint8)).to(dev)
    ev = torch.zeros((max(n, 1), 40), dtype=torch.uint8, device=dev)
    fi = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    events.batch_dev(eng, tb.data_ptr(), None if to is None else to.data_ptr(), stride, tr.data_ptr(),
                     None if td is None else td.data_ptr(), None if tp is None else tp.data_ptr(),
                     0 if pcbs is None else len(pcbs), n, io, flags, ev.data_ptr(), fi.data_ptr(), cnt.data_ptr(),
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    k = int(cnt.item())
    return (ev[:k].cpu().numpy().reshape(-1).view(events.EV_DTYPE), fi[:k].cpu().numpy().astype(np.uint32),
            tb.cpu().numpy()[:blob.size])


@pytest.mark.gpu
@pytest.mark.parametrize("tag,name,with_dmx", CASES)
def test_gpu_golden(eng, tag, name, with_dmx):
    z, dmx, pcbs, io, exp_ev, exp_idx, exp_blob = _case(tag, name, with_dmx)
    ev, idx, blob = _run_dev(eng, z["blob"], z["off"], 0, z["rec"], dmx, pcbs, len(z["len"]), io,
                             events.IXG_EV_UDP_TUPLE)
    assert len(ev) == len(exp_ev)
    assert (ev.view(np.uint8) == exp_ev.view(np.uint8)).all()
    assert (idx == exp_idx).all()
    assert (blob == exp_blob).all()


def _imix_pipeline(n, seed):
    """IMIX traffic with every TCP flow an ESTABLISHED PCB (ids 0..), the RX
    records and demux records from the oracle."""
    tr = traces.make_trace("imix", n, seed=seed)
    cfg = ixgrx.Config(traces.RSS_KEY)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY)
    r = rec.view(ixgrx.REC_DTYPE).reshape(-1)
    tcp = np.nonzero(r["verdict"] == ixgrx.V["TCP"])[0]
    keys = demux.tcp_keys(tr.blob, tr.offsets()[tcp])
    keys["id"] = np.arange(len(tcp), dtype=np.uint32)
    tabs = demux.DemuxTables.build(cfg, keys[::2], keys[1::2][:10], np.zeros(0, demux.LISTEN_DTYPE))
    dmx = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen, 0,
                             tr.blob, tr.off, tr.len, tr.stride, rec)
    pcbs = np.zeros(len(tcp), dtype=events.PCB_DTYPE)
    rng = np.random.default_rng(seed)
    pcbs["pcb_idx"] = rng.integers(0, 1 << 48, size=len(tcp), dtype=np.uint64)
    pcbs["cookie"] = rng.integers(0, 1 << 63, size=len(tcp), dtype=np.uint64)
    return tr, rec, dmx, pcbs


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 200000])
def test_gpu_pipeline_vs_oracle(eng, n):
    tr, rec, dmx, pcbs = _imix_pipeline(n, 0x7E0100 + n)
    io = 0x7F0000000000
    ev, idx, blob = _run_dev(eng, tr.blob, tr.off, 0, rec, dmx, pcbs, n, io, events.IXG_EV_UDP_TUPLE)
    eev, eidx, eblob = oracle.ev_batch(tr.blob, tr.off, 0, rec, dmx, pcbs, io, events.IXG_EV_UDP_TUPLE)
    assert len(ev) == len(eev)
    assert (ev.view(np.uint8) == eev.view(np.uint8)).all()
    assert (idx == eidx).all()
    assert (blob == eblob[:blob.size]).all()
    if n >= 4097:
        assert (ev["sysnr"] == events.USYS_TCP_RECV).sum() > 0 and (ev["sysnr"] == events.USYS_UDP_RECV).sum() > 0


@pytest.mark.gpu
def test_gpu_back_to_back_launches(eng):
    """Launches queued on one stream without a sync in between, over a batch
    of 17K chunks (the per-chunk and per-group scratch counts and bases are
    rewritten by every launch): every launch's output equals the oracle's."""
    import torch
    n = 1_100_003
    tr, rec, dmx, pcbs = _imix_pipeline(n, 0x7E0300)
    io = 0x7F0000000000
    eev, eidx, _ = oracle.ev_batch(tr.blob, tr.off, 0, rec, dmx, pcbs, io, 0)
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(np.concatenate([tr.blob, np.zeros(64, np.uint8)])).to(dev)
    to = torch.from_numpy(np.ascontiguousarray(tr.off).view(np.int64)).to(dev)
    trr = torch.from_numpy(np.ascontiguousarray(rec).view(np.uint8).reshape(n, 16)).to(dev)
    td = torch.from_numpy(np.ascontiguousarray(dmx).view(np.uint8).reshape(n, 8)).to(dev)
    tp = torch.from_numpy(pcbs.view(np.uint8)).to(dev)
    outs = []
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        ev = torch.zeros((n, 40), dtype=torch.uint8, device=dev)
        fi = torch.zeros(n, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        events.batch_dev(eng, tb.data_ptr(), to.data_ptr(), 0, trr.data_ptr(), td.data_ptr(), tp.data_ptr(),
                         len(pcbs), n, io, 0, ev.data_ptr(), fi.data_ptr(), cnt.data_ptr(), s)
        outs.append((ev, fi, cnt))
    torch.cuda.synchronize()
    for ev, fi, cnt in outs:
        k = int(cnt.item())
        assert k == len(eev)
        assert (ev[:k].cpu().numpy().reshape(-1).view(events.EV_DTYPE).view(np.uint8) == eev.view(np.uint8)).all()
        assert (fi[:k].cpu().numpy().astype(np.uint32) == eidx).all()


@pytest.mark.gpu
def test_gpu_stride_layout_no_demux(eng):
    tr = traces.make_trace("tcp64", 3000, seed=0x7E0200)
    rec, _ = oracle.rx_trace(tr, traces.RSS_KEY)
    # no UDP, no demux: no events at all
    ev, idx, _ = _run_dev(eng, tr.blob, None, tr.stride, rec, None, None, tr.n, 0, 0)
    assert len(ev) == 0
    # turn a third of the records into UDP ones: iomap from the stride layout
    r = rec.view(ixgrx.REC_DTYPE).reshape(-1).copy()
    r["verdict"][::3] = ixgrx.V["UDP"]
    ev, idx, _ = _run_dev(eng, tr.blob, None, tr.stride, r, None, None, tr.n, 1 << 40, 0)
    eev, eidx, _ = oracle.ev_batch(tr.blob, None, tr.stride, r, None, None, 1 << 40, 0)
    assert len(ev) == 1000 and (ev.view(np.uint8) == eev.view(np.uint8)).all() and (idx == eidx).all()
