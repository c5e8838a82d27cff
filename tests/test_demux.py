"""PCB demux (dp/net/tcp_in.c:233-323, 500-510).

CPU: the oracle against the golden vectors the reference's own
tcp_input_find_list produced (tests/golden/demux_*.npz,
make_golden_demux.py); the host-side table builder (CSR list order, and
flow-group/bucket placement against the reference's records).
GPU: the HIP demux kernel against the golden vectors and against the oracle
on larger synthetic batches, fed by the GPU's own RX records.
"""
import numpy as np
import pytest

from ix_amd import demux, ixgrx, traces
from oracle import oracle

KEY = traces.RSS_KEY


def _n_out(g):
    return int(g["n_out"]) if "n_out" in g else 0


def _oracle(g, rec=None):
    return oracle.demux_batch(int(g["nfg"]), g["active_start"], g["active"], g["tw_start"], g["tw"], g["listen"],
                              int(g["dev_idx"]) * 512, g["blob"], g["off"], g["len"], 0,
                              g["rec"] if rec is None else rec, n_out=_n_out(g))


def _tables(g):
    return demux.DemuxTables(int(g["nfg"]), g["active_start"], g["active"].view(demux.PCB_DTYPE),
                             g["tw_start"], g["tw"].view(demux.PCB_DTYPE), g["listen"].view(demux.LISTEN_DTYPE),
                             _n_out(g))


def _set_fdir(eng, g):
    """The golden's flow-director filters (the fdir fixture), on the engine
    that recomputes its RX records."""
    if "fdir" in g:
        eng.set_fdir(np.ascontiguousarray(g["fdir"]).view(ixgrx.FDIR_DTYPE).reshape(-1), int(g["fdir_cpu"]))


def _diff(got, exp, what):
    got = np.ascontiguousarray(got).view(np.uint8).reshape(-1, 8)
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} demux records differ; first {bad[:6].tolist()}: " \
                          f"got {got[bad[0]].tolist()} vs exp {exp[bad[0]].tolist()}"


def test_oracle_matches_reference_golden(golden_demux):
    _diff(_oracle(golden_demux), golden_demux["demux"], golden_demux["name"])


def test_golden_covers_every_outcome():
    from conftest import load_golden
    kinds = set()
    for name in ("demux_default", "demux_nolisten_nfg64"):
        kinds |= set(np.unique(load_golden(name)["demux"][:, 4]).tolist())
    assert kinds == {demux.D_NONE, demux.D_ACTIVE, demux.D_TIMEWAIT, demux.D_LISTEN, demux.D_RESET, demux.D_DROP}
    # flow-director frames (outbound groups) reach ACTIVE and TIME-WAIT PCBs
    g = load_golden("demux_fdir_outbound")
    fg = g["rec"][:, 0].astype(np.int64) | (g["rec"][:, 1].astype(np.int64) << 8)
    out = set(np.unique(g["demux"][fg >= ixgrx.IXG_ETH_MAX_TOTAL_FG, 4]).tolist())
    assert {demux.D_ACTIVE, demux.D_TIMEWAIT} <= out


def test_listen_last_entry_quirk():
    """A non-empty listen list with no match yields its last entry
    (tcp_in.c:273-317: the hlist loop variable keeps the last node)."""
    g = traces.pack([bytes(f) for f in traces.build_ipv4(np.random.default_rng(5), 4, 60, 6)])
    rec, _ = oracle.rx_trace(g, KEY)
    listen = np.array([(0, 1, 0, 11, 0), (0, 2, 0, 22, 0), (0, 3, 0, 33, 0)], dtype=demux.LISTEN_DTYPE)
    t = demux.DemuxTables.from_lists(1, [], [], np.zeros(0, demux.PCB_DTYPE), [], np.zeros(0, demux.PCB_DTYPE),
                                     listen)
    out = oracle.demux_batch(1, t.active_start, t.active, t.tw_start, t.tw, t.listen, 0, g.blob, g.off, g.len, 0,
                             rec).view(demux.DEMUX_DTYPE).ravel()
    assert (out["kind"] == demux.D_LISTEN).all() and (out["id"] == 33).all()


def test_table_builder_keeps_list_order():
    rng = np.random.default_rng(7)
    n = 2000
    keys = np.zeros(n, demux.PCB_DTYPE)
    keys["id"] = np.arange(n)
    fg = rng.integers(0, 4, n)
    bk = rng.integers(0, 8, n)
    t = demux.DemuxTables.from_lists(4, fg, bk, keys, fg, keys, np.zeros(0, demux.LISTEN_DTYPE))
    assert t.active_start[0] == 0 and t.active_start[-1] == n and (np.diff(t.active_start.astype(np.int64)) >= 0).all()
    for g in range(4):
        for b in range(8):
            s, e = t.active_start[g * 512 + b], t.active_start[g * 512 + b + 1]
            ids = t.active["id"][s:e]
            assert (ids == np.nonzero((fg == g) & (bk == b))[0]).all()
        assert (t.tw["id"][t.tw_start[g]:t.tw_start[g + 1]] == np.nonzero(fg == g)[0]).all()


def test_flow_placement_matches_reference_records(golden_demux):
    """DemuxTables.build puts a connection where the reference's record for
    its packets points: fg_id (RSS) and pcb_bucket (tcp_to_idx)."""
    g = golden_demux
    cfg = ixgrx.Config(bytes(g["key"]), int(g["nb_rx_fgs"]), int(g["dev_idx"]), 0)
    rec = g["rec"]
    tcp = np.nonzero(rec[:, 2] == 0x01)[0]
    offs, blob = g["off"].astype(np.int64), g["blob"]
    rip = np.array([int(np.frombuffer(blob[o + 26:o + 30].tobytes(), "<u4")[0]) for o in offs[tcp]], np.uint32)
    lip = np.array([int(np.frombuffer(blob[o + 30:o + 34].tobytes(), "<u4")[0]) for o in offs[tcp]], np.uint32)
    l4 = 14 + 4 * (blob[offs[tcp] + 14] & 15).astype(np.int64)
    rp = (blob[offs[tcp] + l4].astype(np.uint32) << 8) | blob[offs[tcp] + l4 + 1]
    lp = (blob[offs[tcp] + l4 + 2].astype(np.uint32) << 8) | blob[offs[tcp] + l4 + 3]
    fg, bucket = demux.flow_of(cfg, rip, lip, rp, lp)
    fg_ref = (rec[tcp, 0].astype(np.int64) | (rec[tcp, 1].astype(np.int64) << 8)) - 512 * int(g["dev_idx"])
    bk_ref = rec[tcp, 12].astype(np.int64) | (rec[tcp, 13].astype(np.int64) << 8)
    rss = (rec[tcp, 3] & ixgrx.RF_FDIR) == 0
    assert (fg[rss] == fg_ref[rss]).all() and (bucket == bk_ref).all()


# ---- GPU ------------------------------------------------------------------


@pytest.mark.gpu
def test_gpu_golden(golden_demux):
    g = golden_demux
    eng = ixgrx.RxEngine(ixgrx.Config(bytes(g["key"]), int(g["nb_rx_fgs"]), int(g["dev_idx"]), 0))
    try:
        demux.load(eng, _tables(g))
        out = demux.batch_host(eng, g["blob"], g["off"], g["len"], 0, g["rec"])
        _diff(out, g["demux"], g["name"])
    finally:
        eng.close()


def _synthetic_tables(cfg, tr, rec, rng, active_frac=0.6, tw_frac=0.1, listen=True):
    """Connections for a share of a trace's TCP tuples, plus noise."""
    tcp = np.nonzero(rec[:, 2] == 0x01)[0]
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    o = offs[tcp]
    l4 = o + 14 + 4 * (b[o + 14] & 15).astype(np.int64)
    keys = np.zeros(tcp.size, demux.PCB_DTYPE)
    keys["remote_ip"] = b[o + 26] | (b[o + 27].astype(np.uint32) << 8) | (b[o + 28].astype(np.uint32) << 16) | \
        (b[o + 29].astype(np.uint32) << 24)
    keys["local_ip"] = b[o + 30] | (b[o + 31].astype(np.uint32) << 8) | (b[o + 32].astype(np.uint32) << 16) | \
        (b[o + 33].astype(np.uint32) << 24)
    keys["remote_port"] = (b[l4].astype(np.uint32) << 8) | b[l4 + 1]
    keys["local_port"] = (b[l4 + 2].astype(np.uint32) << 8) | b[l4 + 3]
    keys["id"] = np.arange(tcp.size) + 1
    u = rng.random(tcp.size)
    act = keys[u < active_frac]
    tw = keys[(u >= active_frac) & (u < active_frac + tw_frac)]
    noise = np.zeros(5000, demux.PCB_DTYPE)
    for f in ("remote_ip", "local_ip"):
        noise[f] = rng.integers(0, 2**32, noise.size, dtype=np.uint64)
    for f in ("remote_port", "local_port"):
        noise[f] = rng.integers(0, 2**16, noise.size)
    noise["id"] = 10**7 + np.arange(noise.size)
    lis = np.zeros(0, demux.LISTEN_DTYPE)
    if listen:
        lis = np.array([(0, int(keys["local_port"][k]), 0, 900 + k, 0) for k in range(0, min(40, tcp.size), 3)],
                       dtype=demux.LISTEN_DTYPE)
    return demux.DemuxTables.build(cfg, np.concatenate([act, noise]), tw, lis)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,listen", [("tcp64", 200000, True), ("imix", 100000, False),
                                           ("mixed", 60000, True)])
def test_gpu_device_pipeline_vs_oracle(kind, n, listen):
    """RX records made on the GPU feed the device demux; checked against
    the oracle's demux of the oracle's records."""
    import torch
    rng = np.random.default_rng(n)
    tr = traces.make_trace(kind, n, seed=0x1BD000 + n, bad_ip=0.01, bad_l4=0.01)
    cfg = ixgrx.Config(KEY, 128, 1, 0)
    er, _ = oracle.rx_trace(tr, KEY, 128, 1, 0, threads=8, hash_mode=oracle.HASH_TABLE)
    tabs = _synthetic_tables(cfg, tr, er, rng, listen=listen)
    eng = ixgrx.RxEngine(cfg)
    try:
        demux.load(eng, tabs)
        dev = torch.device("cuda:0")
        blob = torch.from_numpy(np.concatenate([tr.blob, np.zeros(64, np.uint8)])).to(dev)
        lens = torch.from_numpy(tr.len.view(np.int16)).to(dev)
        off = None if tr.off is None else torch.from_numpy(tr.off.view(np.int64)).to(dev)
        rec = torch.empty((tr.n, 16), dtype=torch.uint8, device=dev)
        out = torch.empty((tr.n, 8), dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream().cuda_stream
        eng.batch_dev(blob.data_ptr(), None if off is None else off.data_ptr(), lens.data_ptr(), tr.stride, tr.n,
                      rec.data_ptr(), None, s)
        demux.batch_dev(eng, blob.data_ptr(), None if off is None else off.data_ptr(), tr.stride, tr.n,
                        rec.data_ptr(), out.data_ptr(), s)
        torch.cuda.synchronize()
        assert (rec.cpu().numpy() == er).all()
        exp = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen,
                                 512, tr.blob, tr.off, tr.len, tr.stride, er)
        _diff(out.cpu().numpy(), exp, kind)
        kinds = np.unique(exp[:, 4])
        assert demux.D_ACTIVE in kinds and demux.D_TIMEWAIT in kinds
    finally:
        eng.close()


@pytest.mark.gpu
def test_gpu_demux_requires_tables():
    eng = ixgrx.RxEngine(ixgrx.Config(KEY))
    try:
        with pytest.raises(RuntimeError, match="no demux tables"):
            demux.batch_host(eng, np.zeros(64, np.uint8), None, np.array([60], np.uint16), 64,
                             np.zeros(1, ixgrx.REC_DTYPE))
    finally:
        eng.close()


def _engine_in_mode(cfg, mode):
    """An engine with the launch split forced (ixg_rx_set_split)."""
    return ixgrx.RxEngine(cfg, split=mode)


def _fused_dev(eng, blob, off, lens, stride, n):
    import torch
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(np.concatenate([blob, np.zeros(64, np.uint8)])).to(dev)
    tl = torch.from_numpy(np.ascontiguousarray(lens).view(np.int16)).to(dev)
    to = None if off is None else torch.from_numpy(np.ascontiguousarray(off).view(np.int64)).to(dev)
    rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    demux.rx_demux_dev(eng, tb.data_ptr(), None if to is None else to.data_ptr(), tl.data_ptr(), stride, n,
                       rec.data_ptr(), out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return rec.cpu().numpy(), out.cpu().numpy()


MODES = ["auto", "general", "fast", "short", "long"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_fused_golden(golden_demux, mode):
    """RX + demux in one pass (ixg_rx_demux_batch_dev) on the reference's
    demux fixtures, every launch split."""
    g = golden_demux
    eng = _engine_in_mode(ixgrx.Config(bytes(g["key"]), int(g["nb_rx_fgs"]), int(g["dev_idx"]), 0), mode)
    try:
        demux.load(eng, _tables(g))
        _set_fdir(eng, g)
        rec, out = _fused_dev(eng, g["blob"], g["off"], g["len"], 0, len(g["len"]))
        assert (rec == g["rec"]).all()
        _diff(out, g["demux"], g["name"] + " fused " + mode)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kind,n,listen", [("tcp64", 200000, True), ("imix", 100000, False),
                                           ("mixed", 60000, True), ("tcp1514", 20000, True)])
def test_gpu_fused_vs_oracle(kind, n, listen, mode):
    rng = np.random.default_rng(n + 7)
    tr = traces.make_trace(kind, n, seed=0x1BD100 + n, bad_ip=0.01, bad_l4=0.01)
    cfg = ixgrx.Config(KEY, 128, 1, 0)
    er, _ = oracle.rx_trace(tr, KEY, 128, 1, 0, threads=8, hash_mode=oracle.HASH_TABLE)
    tabs = _synthetic_tables(cfg, tr, er, rng, listen=listen)
    eng = _engine_in_mode(cfg, mode)
    try:
        demux.load(eng, tabs)
        rec, out = _fused_dev(eng, tr.blob, tr.off, tr.len, tr.stride, tr.n)
        assert (rec == er).all()
        exp = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen,
                                 512, tr.blob, tr.off, tr.len, tr.stride, er)
        _diff(out, exp, f"{kind} fused {mode}")
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["auto", "general"])
@pytest.mark.parametrize("kind", ["tcp64", "imix"])
def test_gpu_fdir_outbound_groups(kind, mode):
    """Frames the flow director steers (ixg_rx_set_fdir) carry the CPU's
    outbound group ETH_MAX_TOTAL_FG + cpu; their PCB lookup must use that
    group's active and TIME-WAIT lists (tcp_in.c:249,260 on cur_fg =
    fgs[pkt->fg_id]), which the snapshot holds after the local groups. Fused
    and separate demux against the oracle, with matching outbound PCBs."""
    import torch
    rng = np.random.default_rng(0xFD1)
    tr = traces.make_trace(kind, 100000, seed=0x1BD200)
    cfg = ixgrx.Config(KEY, 128, 1, 0)
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    tcp = np.nonzero(b[offs + 23] == 6)[0]
    keys = demux.tcp_keys(b, offs[tcp])
    keys["id"] = np.arange(tcp.size) + 1
    pick = rng.random(tcp.size) < 0.25
    filt = np.zeros(int(pick.sum()), ixgrx.FDIR_DTYPE)
    filt["src_ip"], filt["dst_ip"] = keys["remote_ip"][pick], keys["local_ip"][pick]
    filt["src_port"], filt["dst_port"] = keys["remote_port"][pick], keys["local_port"][pick]
    cpu, n_out = 2, 4
    out_keys = keys[pick]
    u = rng.random(out_keys.size)
    oa, ot = out_keys[u < 0.7], out_keys[(u >= 0.7) & (u < 0.85)]
    local = keys[~pick][:5000]
    lis = np.array([(0, int(keys["local_port"][0]), 0, 77, 0)], dtype=demux.LISTEN_DTYPE)
    tabs = demux.DemuxTables.build(cfg, local, np.zeros(0, demux.PCB_DTYPE), lis,
                                   outbound=(oa, ot, np.full(oa.size, cpu), np.full(ot.size, cpu)), n_out=n_out)
    er, _ = oracle.rx_batch(KEY, 128, 1, 0, tr.blob, tr.off, tr.len, tr.stride, threads=8, fdir=filt, cpu_id=cpu)
    exp = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen, 512,
                             tr.blob, tr.off, tr.len, tr.stride, er, n_out=n_out)
    kinds = exp[(er[:, 0].astype(np.int64) | (er[:, 1].astype(np.int64) << 8)) >= 8192, 4]
    assert (kinds == demux.D_ACTIVE).sum() > 1000 and (kinds == demux.D_TIMEWAIT).sum() > 100
    eng = _engine_in_mode(cfg, mode)
    try:
        demux.load(eng, tabs)
        eng.set_fdir(filt, cpu)
        rec, out = _fused_dev(eng, tr.blob, tr.off, tr.len, tr.stride, tr.n)
        assert (rec == er).all()
        _diff(out, exp, f"{kind} fdir fused {mode}")
        out2 = demux.batch_host(eng, tr.blob, tr.off, tr.len, tr.stride, er)
        _diff(out2, exp, f"{kind} fdir separate {mode}")
    finally:
        eng.close()
