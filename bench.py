#!/usr/bin/env python3
"""Benchmark: device-resident RX parse + checksum + flow-hash on MI355X.

A step = one pass of the hot path (one ixg_rx_batch_dev launch) over one
batch of synthetic frames already resident in HBM. Default workload = the
configuration BASELINE.json's metric is quoted on: configs[1], 16,777,216
64-byte Eth/IPv4/TCP frames on one GPU. A 1514-byte shard (C4's per-GPU
shape) is measured as the secondary line. N>1: one process per GPU, each
with its own batch (weak scaling), no collective on the data path; the
timed region is bracketed by barrier + synchronize and the max over ranks
is taken.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkt/s + GB/s device-resident RX parse+cksum+flow-hash, 64B & 1500B frames"
PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

# one ixg_rx_batch_dev launch = the fixed-shape kernel + the general kernel
# (which, when no chunk was deferred, only scans the per-chunk flags); the
# HIP events bracket both on the launch stream
def kernels(wl) -> str:
    """The dispatches one launch makes (ixgrx_launch): for fixed strides <=
    64 B the coalesced fixed-shape kernel, else the sampler and the lane-load
    one; then the short and the long general kernels (each exits at once
    when its class has nothing deferred), or behind the coalesced kernel one
    general kernel taking both classes (ixg_rx_any_s). The long class runs
    the flat walk's build (ixg_rx_glong_*) unless the IPv6 tables are staged
    (IXG_F_IPV6) or a fixed stride can never give a flat chunk."""
    v6 = bool(getattr(wl, "flags", 0) & 2)
    if wl.off is not None:
        return "ixg_rx_short_sp_o (samples the launch mode itself) + " + ("ixg_rx_general_o" if v6 else "ixg_rx_glong_o")
    if wl.stride <= 64:
        return "ixg_rx_fastc_s (deferred chunks finished in the same dispatch)"
    flat = not v6 and 63 * wl.stride < 30 * 1024
    return "ixg_rx_short_sp_s (samples the launch mode itself) + " + ("ixg_rx_glong_s" if flat else "ixg_rx_general_s")


# untimed launches before each secondary line (demux, events, TX) is timed
LINE_WARMUP = 20

WORKLOADS = {
    # name: (trace kind, frames per GPU, distinct frames in the pool, description)
    "c2": ("tcp64", 16 * 1024 * 1024, 1 << 20, "C2: 16M x 64B Eth/IPv4/TCP frames (L=60, stride 60), 1 GPU"),
    "c4": ("tcp1514", 8 * 1024 * 1024, 1 << 13, "C4 per-GPU shard: 8M x 1514B IPv4/TCP frames (stride 1516)"),
    "c3": ("imix", 16 * 1024 * 1024, 1 << 18, "C3: 16M IMIX 7:4:1 (60/590/1514B) TCP+UDP, packed, u64 offsets"),
    "c5": ("mixed", 16 * 1024 * 1024, 1 << 18, "C5: 16M mixed IPv4 ihl 5..15 + 50% IPv6 (IXG_F_IPV6 extension: IPv6 "
                                                "parsed), packed"),
    # C5 in the reference's semantics: IPv6 frames are dropped by eth_input
    # (dp/net/ip.c:132-137), IPv4 with options parsed
    "c5r": ("mixed", 16 * 1024 * 1024, 1 << 18, "C5 (reference semantics: IPv6 -> DROP_ETHERTYPE): 16M mixed IPv4 "
                                                 "ihl 5..15 + 50% IPv6, packed"),
    # A/B only (not configs): C5's families alone or in 128-frame runs
    "c5v4": ("mixed_v4", 16 * 1024 * 1024, 1 << 18, "C5 IPv4 part only (A/B only)"),
    "c5v6": ("mixed_v6", 16 * 1024 * 1024, 1 << 18, "C5 IPv6 part only (A/B only)"),
    "c5s": ("mixed_sorted", 16 * 1024 * 1024, 1 << 18, "C5 in 128-frame single-family runs (A/B only)"),
    # C2 with 1% bad IP and 1% bad TCP checksums (flag paths)
    "c2b": ("tcp64", 16 * 1024 * 1024, 1 << 20, "C2 with 1% bad IP + 1% bad TCP checksums (L=60, stride 60)"),
    # A/B only (not a config): C2's slots, IPv4 with one option word (all deferred)
    "c2opt": ("tcp64opt", 16 * 1024 * 1024, 1 << 20, "C2 slots, IPv4 ihl 6 (A/B only)"),
    # A/B only (not a config): C2's frames in the packed u64-offset layout
    "c2o": ("tcp64", 16 * 1024 * 1024, 1 << 20, "C2 frames, u64-offset layout (A/B only)"),
}


def alg_bytes(tr, flags: int = 0) -> np.ndarray:
    """Algorithmic bytes read per frame: 14 + ip_len for
    IPv4 (the Ethernet header plus the IP datagram; padding excluded), 54 +
    payload for IPv6 under IXG_F_IPV6 (else 14: eth_input drops it on the
    ethertype), plus the descriptor and the 16-byte record."""
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    et = (b[offs + 12].astype(np.int64) << 8) | b[offs + 13]
    v4 = (b[offs + 16].astype(np.int64) << 8) | b[offs + 17]
    v6 = (b[offs + 18].astype(np.int64) << 8) | b[offs + 19]
    rd = np.where(et == 0x86DD, 54 + v6 if flags & 2 else 14, 14 + v4)
    rd = np.minimum(rd, tr.len.astype(np.int64))
    desc = 2 + (8 if tr.off is not None else 0)
    return rd + desc + 16


def lines_touched(lo: np.ndarray, hi: np.ndarray, line: int = 128) -> int:
    """The distinct `line`-byte lines holding a byte of any range [lo, hi)."""
    keep = hi > lo
    lo, hi = lo[keep] // line, (hi[keep] - 1) // line
    mark = np.zeros(int(hi.max()) + 2, dtype=np.int64)
    np.add.at(mark, lo, 1)
    np.add.at(mark, hi + 1, -1)
    return int((np.cumsum(mark) > 0).sum())


def line_floor_bytes(tr, flags: int = 0, line: int = 128) -> float:
    """The bytes per frame a memory system that fetches whole `line`-byte
    lines must move: the distinct lines of the batch that hold a byte the
    path reads (frame bytes [12, alg_bytes' read end), as in alg_bytes),
    plus the descriptor and the record. For packed batches whose frames the
    reference reads only in part (C5 in reference semantics: IPv6 frames
    dropped on the Ethernet type) this is the reachable floor; the 8(d)
    bytes count only the bytes read."""
    offs = tr.offsets().astype(np.int64)
    b = tr.blob
    et = (b[offs + 12].astype(np.int64) << 8) | b[offs + 13]
    v4 = (b[offs + 16].astype(np.int64) << 8) | b[offs + 17]
    v6 = (b[offs + 18].astype(np.int64) << 8) | b[offs + 19]
    rd = np.minimum(np.where(et == 0x86DD, 54 + v6 if flags & 2 else 14, 14 + v4), tr.len.astype(np.int64))
    lines = lines_touched(offs + 12, offs + np.maximum(rd, 13), line)
    desc = 2 + (8 if tr.off is not None else 0)
    return lines * line / tr.n + desc + 16


class Workload:
    """A batch of n frames on `dev`, tiled from `pool` distinct frames."""

    def __init__(self, name: str, seed: int, dev, n: int | None = None, pool: int | None = None):
        import torch
        from ix_amd import traces
        kind, n_def, pool_def, self.desc = WORKLOADS[name]
        self.name = name
        self.n = n or n_def
        pool = min(pool or pool_def, self.n)
        assert self.n % pool == 0
        self.reps = self.n // pool
        bad = 0.01 if name == "c2b" else 0.0
        self.pool = traces.make_trace(kind, pool, seed=seed, bad_ip=bad, bad_l4=bad)
        if name == "c2o":
            tr = self.pool
            self.pool = traces.Trace(tr.blob, tr.offsets().copy(), tr.len, 0)
        self.flags = 2 if kind.startswith("mixed") and name != "c5r" else 0
        tr = self.pool
        self.bytes_per_pkt = float(alg_bytes(tr, self.flags).mean())
        self.wire_bytes = float(tr.len.astype(np.int64).mean())
        if tr.off is None:
            S = tr.stride
            self.stride = S
            src = torch.from_numpy(tr.blob[:pool * S]).to(dev)
            self.blob = torch.zeros(self.n * S + traces.TAIL_PAD, dtype=torch.uint8, device=dev)
            self.blob[:self.n * S].view(self.reps, pool * S).copy_(src.unsqueeze(0).expand(self.reps, -1))
            self.off = None
        else:
            self.stride = 0
            span = int(tr.off[-1]) + ((int(tr.len[-1]) + 3) // 4) * 4
            src = torch.from_numpy(tr.blob[:span]).to(dev)
            self.blob = torch.zeros(self.reps * span + traces.TAIL_PAD, dtype=torch.uint8, device=dev)
            self.blob[:self.reps * span].view(self.reps, span).copy_(src.unsqueeze(0).expand(self.reps, -1))
            o = torch.from_numpy(tr.off.view(np.int64)).to(dev)
            k = torch.arange(self.reps, device=dev, dtype=torch.int64).unsqueeze(1) * span
            self.off = (o.unsqueeze(0) + k).reshape(-1).contiguous()
        ln = torch.from_numpy(tr.len.view(np.int16)).to(dev)
        self.len = ln.repeat(self.reps).contiguous()
        self.out = torch.empty((self.n, 16), dtype=torch.uint8, device=dev)

    def launch(self, eng, stream) -> None:
        eng.batch_dev(self.blob.data_ptr(), None if self.off is None else self.off.data_ptr(),
                      self.len.data_ptr(), self.stride, self.n, self.out.data_ptr(), None, stream)

    def snapshot(self):
        """Device-side tiling check (every repetition of the pool produced
        the same records as the first) and the first repetition's records,
        for the cpu_baseline leg to compare with the oracle."""
        import torch
        v = self.out.view(self.reps, -1, 16)
        tiled = bool(torch.equal(v, v[:1].expand(self.reps, -1, -1)))
        return tiled, v[0].cpu().numpy()


def time_steps(wl, eng, steps, warmup, dist, world):
    """W warm-up launches, then exactly K timed launches back to back
    (barrier + synchronize on both sides; the wall time, max over ranks, is
    the line's value), then the same K launches again, each between HIP
    events on the launch stream, for the per-launch kernel time the
    roofline uses (events between launches would add their own gaps to the
    value loop)."""
    import torch
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for _ in range(warmup):
        wl.launch(eng, sp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        wl.launch(eng, sp)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for a, b in ev:
        a.record(stream)
        wl.launch(eng, sp)
        b.record(stream)
    torch.cuda.synchronize()
    kern = [a.elapsed_time(b) * 1e-3 for a, b in ev]
    if world > 1:
        from ix_amd.shard import max_over_ranks
        el = max_over_ranks(el, dist, device="cuda" if dist.get_backend() == "nccl" else "cpu")
    return el, float(np.mean(kern)), float(np.min(kern))


def mbuf_arena(tr, n: int):
    """The first n frames of `tr` laid out as IX mbufs (2112-B elements, len
    @0, data @+64; inc/ix/mbuf.h:73-90). Returns (arena, pointers)."""
    S = 2112
    arena = np.zeros(n * S + 64, dtype=np.uint8)
    base = (-arena.ctypes.data) % 64
    rows = arena[base:base + n * S].reshape(n, S)
    offs = tr.offsets()[:n].astype(np.int64)
    lens = tr.len[:n].astype(np.int64)
    rows[:, :8] = lens.astype("<u8").view(np.uint8).reshape(n, 8)
    for L in np.unique(lens):
        idx = np.nonzero(lens == L)[0]
        src = offs[idx, None] + np.arange(L, dtype=np.int64)[None, :]
        rows[idx, 64:64 + L] = tr.blob[src]
    ptrs = arena.ctypes.data + base + np.arange(n, dtype=np.uint64) * S
    return arena, ptrs


def cpu_rate(ptrs, flags, key, seconds, threads, hash_mode, work):
    from oracle import oracle
    done, t0 = 0, time.perf_counter()
    while True:
        oracle.rx_mbufs(key, 128, 0, flags, ptrs, threads=threads, hash_mode=hash_mode, work=work)
        done += len(ptrs)
        el = time.perf_counter() - t0
        if el >= seconds:
            return done / el / 1e6, done, el


def cpu_baseline(tr, flags, key, seconds: float, threads: int, name: str):
    """dp/ix's own RX path on the GPU box's host cores:
    oracle/_ref/ixref_bench, built from the reference's dp/net + dp/lwip
    sources (oracle/ref_harness/harness_bench.c), one process per core, each
    over its own arena of pre-filled 2112-B IX mbufs larger than the LLC.
    `value` = IX's per-packet software work as deployed (eth_input -> ip_input
    -> tcp_input_tmp -> tcp_input head with tcp_to_idx; checksums and RSS are
    the NIC's); "full_software" adds the reference's checksum and Toeplitz
    functions (the work the GPU kernels do). The oracle (C restatement, the
    "port") is timed beside it. Falls back to the port when the reference
    binary was not built."""
    from oracle import oracle
    procs = threads
    mb = 1 << 18  # 553 MB of mbufs per core: beyond the LLC, as fresh DMA'd packets
    ix = oracle.ref_bench(tr, key, "ix", procs, seconds, mb) if flags == 0 else None
    res = {}
    if ix is not None:
        full = oracle.ref_bench(tr, key, "full", procs, max(2.0, seconds / 2), mb)
        one = oracle.ref_bench(tr, key, "ix", 1, max(2.0, seconds / 4), mb)
        res = {"value": round(ix["mpps"], 2), "unit": "Mpkt/s", "cores": procs, "kind": "reference",
               "sample": f"oracle/_ref/ixref_bench ix: the reference's eth_input -> ip_input -> tcp_input_tmp -> "
                         f"tcp_input head + tcp_to_idx (NIC checksum/RSS offload as in IX) over {ix['frames']} "
                         f"distinct {name} frames in {mb} pre-filled 2112-B IX mbufs per core, {ix['pkts']:.0f} "
                         f"frames in {ix['seconds']:.1f}s on {procs} processes",
               "ns_per_pkt_core": ix["ns_per_pkt_core"],
               "full_software": {"mpps": round(full["mpps"], 2), "cores": procs,
                                 "ns_per_pkt_core": full["ns_per_pkt_core"],
                                 "what": "+ the reference's chksum_internet, inet_chksum_pseudo_partial and "
                                         "compute_toeplitz_hash per frame (the NIC's work in software)"},
               "reference_1core": {"mpps": round(one["mpps"], 2), "ns_per_pkt": one["ns_per_pkt_core"]}}
    n = min(tr.n, 1 << 20)
    arena, ptrs = mbuf_arena(tr, n)
    v, done, secs = cpu_rate(ptrs, flags, key, max(2.0, seconds / 2), threads, oracle.HASH_TABLE, oracle.WORK_FULL)
    side = max(1.0, seconds / 8)
    one = {}
    for label, hm, wk in (("full_table", oracle.HASH_TABLE, oracle.WORK_FULL),
                          ("full_bitserial", oracle.HASH_BITSERIAL, oracle.WORK_FULL),
                          ("ix_equivalent", oracle.HASH_TABLE, oracle.WORK_IX)):
        one[label] = round(cpu_rate(ptrs[:1 << 16], flags, key, side, 1, hm, wk)[0], 2)
    del arena
    port = {"mpps": round(v, 2), "cores": threads,
            "sample": f"oracle/ixgrx_oracle.c full software (table-driven Toeplitz/CRC) over {n} {name} frames "
                      f"in 2112-B IX mbufs, {done} frames in {secs:.1f}s on {threads} threads",
            "modes_1core_mpps": one}
    if not res:
        res = {"value": port["mpps"], "unit": "Mpkt/s", "cores": threads, "kind": "port", "sample": port["sample"],
               "modes_1core_mpps": one,
               "note": "oracle/_ref/ixref_bench not built (or not an IPv4-only workload): the port is the baseline"}
    else:
        res["port"] = port
    return res


def parity_leg(checks, key) -> dict:
    """The oracle checks the device results of every line (part of the
    cpu_baseline leg: the oracle is only ever the checker). A line passes
    when its tiled batch is self-consistent on the device and its first
    repetition equals the oracle's records for the distinct frames."""
    from ix_amd import demux
    from oracle import oracle
    res = {}
    for c in checks:
        if c[0] == "rx":
            _, name, pool, flags, rec, tiled = c
            er, _ = oracle.rx_trace(pool, key, flags=flags, threads=8, hash_mode=oracle.HASH_TABLE)
            res[name] = "ok" if tiled and np.array_equal(rec, er) else "MISMATCH"
        elif c[0] == "hostpath":
            _, pool, recs, name = c
            er, _ = oracle.rx_trace(pool, key, threads=8, hash_mode=oracle.HASH_TABLE)
            res[name] = "ok" if np.array_equal(recs, er) else "MISMATCH"
        elif c[0] == "mbufs":
            _, tr, ptrs, arena, rec = c
            er = oracle.rx_mbufs(key, 128, 0, 0, ptrs[:1 << 16], threads=8, hash_mode=oracle.HASH_TABLE)
            res["mbufs"] = "ok" if np.array_equal(rec.view(np.uint8).reshape(-1, 16)[:1 << 16], er) else "MISMATCH"
        elif c[0] == "events":
            _, pool, tabs, pcbs, io, ev0, f0, tiled = c
            er, _ = oracle.rx_trace(pool, key, threads=8, hash_mode=oracle.HASH_TABLE)
            dx = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen,
                                    0, pool.blob, pool.off, pool.len, pool.stride, er)
            eev, eidx, _ = oracle.ev_batch(pool.blob, pool.off, 0, er, dx, pcbs, io, 0)
            ok = ev0 is not None and len(ev0) == len(eev) and \
                np.array_equal(ev0.view(np.uint8), eev.view(np.uint8)) and np.array_equal(f0, eidx.astype(np.int64))
            res["events"] = "ok" if ok and tiled else ("MISMATCH" if not ok else "MISMATCH (tiling)")
        elif c[0] == "tcpx":
            _, pool, rec, ext0, tiled = c
            er, _ = oracle.rx_trace(pool, key, threads=8, hash_mode=oracle.HASH_TABLE)
            eext, _ = oracle.tcp_ext_batch(pool.blob, pool.off, pool.stride, er)
            ok = np.array_equal(rec, er) and np.array_equal(ext0, eext)
            res["tcpx"] = "ok" if ok and tiled else ("MISMATCH" if not ok else "MISMATCH (tiling)")
        elif c[0] == "icmp":
            _, pool, rec, out, mac, host, tiled = c
            er, _ = oracle.rx_trace(pool, key, threads=8, hash_mode=oracle.HASH_TABLE)
            eo, k = oracle.icmp_reflect_batch(pool.blob, pool.off, 0, er, mac, host)
            ok = np.array_equal(rec, er) and k == pool.n and np.array_equal(out[:eo.size], eo)
            res["icmp"] = "ok" if ok and tiled else ("MISMATCH" if not ok else "MISMATCH (tiling)")
        elif c[0] == "tx":
            _, kind, (buf, segs, smac, dmacs, out, out_len), tiled = c
            size = int(segs["out_off"][-1]) + 2048
            eo, el = oracle.tx_batch(buf, segs, smac, dmacs, size, 0)
            ok = np.array_equal(el, out_len) and all(
                np.array_equal(out[o:o + L], eo[o:o + L]) for o, L in zip(segs["out_off"].astype(np.int64), el))
            res["tx_" + kind] = "ok" if ok and tiled else ("MISMATCH" if not ok else "MISMATCH (tiling)")
        else:
            _, name, pool, tabs, rec, dmx, tiled = c
            er, _ = oracle.rx_trace(pool, key, threads=8, hash_mode=oracle.HASH_TABLE)
            exp = oracle.demux_batch(tabs.nfg, tabs.active_start, tabs.active, tabs.tw_start, tabs.tw, tabs.listen,
                                     0, pool.blob, pool.off, pool.len, pool.stride, er)
            ok = tiled and np.array_equal(rec, er) and np.array_equal(dmx, exp)
            res[name] = "ok" if ok else "MISMATCH"
            res[name + "_kinds"] = {demux.KINDS[int(v)]: int(n) for v, n in zip(*np.unique(exp[:, 4], return_counts=True))}
    return res


def copy_inclusive(wl, eng, key, reps=3):
    """Host-resident batch: H2D frames (pinned) + kernel + D2H records."""
    import torch
    n = wl.n
    h_blob = wl.blob.cpu().pin_memory()
    h_len = wl.len.cpu().pin_memory()
    h_off = None if wl.off is None else wl.off.cpu().pin_memory()
    h_out = torch.empty((n, 16), dtype=torch.uint8).pin_memory()
    s = torch.cuda.current_stream()
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wl.blob.copy_(h_blob, non_blocking=True)
        wl.len.copy_(h_len, non_blocking=True)
        if h_off is not None:
            wl.off.copy_(h_off, non_blocking=True)
        wl.launch(eng, s.cuda_stream)
        h_out.copy_(wl.out, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    h2d = h_blob.numel() + h_len.numel() * 2 + (0 if h_off is None else h_off.numel() * 8)
    return {"mpps": n / best / 1e6, "seconds": best, "h2d_bytes": int(h2d), "d2h_bytes": int(n * 16),
            "link_gbps": (h2d + n * 16) / best / 1e9}


def copy_overlapped(wl, engs, pieces=16, reps=3):
    """Host-resident batch, pipelined: the batch in `pieces` slices on two
    streams (one context each, IX's per-CPU model), so slice k+1's H2D copy
    overlaps slice k's kernels and D2H copy of records. Fixed-stride
    workloads only."""
    import torch
    n, S = wl.n, wl.stride
    assert wl.off is None and n % pieces == 0
    C = n // pieces
    h_blob = wl.blob.cpu().pin_memory()
    h_len = wl.len.cpu().pin_memory()
    h_out = torch.empty((n, 16), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(pieces):
            st = streams[k % 2]
            a, b = k * C, (k + 1) * C
            with torch.cuda.stream(st):
                wl.blob[a * S:b * S].copy_(h_blob[a * S:b * S], non_blocking=True)
                wl.len[a:b].copy_(h_len[a:b], non_blocking=True)
                engs[k % 2].batch_dev(wl.blob.data_ptr() + a * S, None, wl.len.data_ptr() + 2 * a, S, C,
                                      wl.out.data_ptr() + 16 * a, None, st.cuda_stream)
                h_out[a:b].copy_(wl.out[a:b], non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    tiled = bool(torch.equal(h_out.view(wl.reps, -1, 16), h_out.view(wl.reps, -1, 16)[:1].expand(wl.reps, -1, -1)))
    h2d = n * S + n * 2
    return {"mpps": round(n / best / 1e6, 2), "seconds": round(best, 5), "pieces": pieces, "streams": 2,
            "h2d_bytes": int(h2d), "d2h_bytes": int(n * 16), "link_gbps": round((h2d + n * 16) / best / 1e9, 2),
            "parity": "tiled-consistent" if tiled else "MISMATCH"}


def demux_line(dev, key, steps: int, rank: int, eng_for):
    """PCB demux over C2's shape: 16M 64-B TCP frames tiled
    from 2^16 distinct connections. Two forms, each a step = one launch: the
    fused RX + demux (ixg_rx_demux_batch_dev: the lookup runs in the RX
    kernels from the parse state) and the separate demux pass over frames +
    records already in HBM (ixg_demux_batch_dev). Three table sets:
    `established` (every connection ESTABLISHED, the echoserver case; 1 %
    extra TIME-WAIT entries of other connections and one listener, which no
    frame reaches), `mixed` (90 % of the connections active, 5 % in
    TIME-WAIT with their own tuple, 5 % unknown, which the listen list takes:
    a non-empty list hands an unmatched segment to its last entry,
    tcp_in.c:317-323) and `mixed_nolisten` (the same without listeners: the
    unknown 5 % get RESET, tcp_in.c:500-510). Every outcome of the lookup
    occurs in one of them, each checked against the oracle."""
    import torch
    from ix_amd import demux
    wl = Workload("c2", seed=0x1BD000 + 97 * rank, dev=dev, pool=1 << 16)
    eng = eng_for(0)
    stream = torch.cuda.current_stream()
    wl.launch(eng, stream.cuda_stream)
    pool = wl.pool
    keys = demux.tcp_keys(pool.blob, pool.offsets())
    cfg = eng.cfg
    rng = np.random.default_rng(1)
    tw = keys[rng.random(keys.size) < 0.01].copy()
    tw["id"] += 1 << 20
    tw["remote_port"] ^= 1  # TIME-WAIT entries of other (closed) connections
    lis = np.array([(0, 80, 0, 7, 0)], dtype=demux.LISTEN_DTYPE)
    u = np.random.default_rng(2).random(keys.size)
    tabsets = {"established": demux.DemuxTables.build(cfg, keys, tw, lis),
               "mixed": demux.DemuxTables.build(cfg, keys[u < 0.90], keys[(u >= 0.90) & (u < 0.95)], lis),
               "mixed_nolisten": demux.DemuxTables.build(cfg, keys[u < 0.90], keys[(u >= 0.90) & (u < 0.95)],
                                                         np.zeros(0, demux.LISTEN_DTYPE))}
    out = torch.empty((wl.n, 8), dtype=torch.uint8, device=dev)
    out2 = torch.empty((wl.n, 8), dtype=torch.uint8, device=dev)
    rec2 = torch.empty((wl.n, 16), dtype=torch.uint8, device=dev)

    def separate():
        demux.batch_dev(eng, wl.blob.data_ptr(), None, wl.stride, wl.n, wl.out.data_ptr(), out.data_ptr(),
                        stream.cuda_stream)

    def fused():
        demux.rx_demux_dev(eng, wl.blob.data_ptr(), None, wl.len.data_ptr(), wl.stride, wl.n, rec2.data_ptr(),
                           out2.data_ptr(), stream.cuda_stream)

    def timed(fn):
        for _ in range(LINE_WARMUP):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(stream)
            fn()
            b.record(stream)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, float(np.mean([a.elapsed_time(b) * 1e-3 for a, b in ev]))
    # separate pass, algorithmic bytes per frame: the record (16), the header
    # bytes the lookup reads (byte 14 + the 12 tuple bytes), the bucket bounds
    # (8), the entries compared up to the match (16 each, here ~1 per bucket)
    # and the 8-byte result. Fused: RX's 72 B + the 8-byte result (the table
    # reads are L2 / Infinity-Cache resident: 64K connections = 1 MiB).
    alg = 16 + 13 + 8 + 16 * 1.0 + 8
    algf = 72 + 8
    # the separate pass's 128-B line floor: the lines holding byte 14 and the
    # tuple bytes 26..37 of each frame (at C2's 60-B stride every line of the
    # frames), the record read, the 8-B result; the bucket lines (64 KiB of
    # connections: 4 MiB of lines) stay in L2 / Infinity Cache
    offs = pool.offsets().astype(np.int64)
    floor = lines_touched(np.concatenate([offs + 14, offs + 26]), np.concatenate([offs + 15, offs + 38])) * 128 \
        / pool.n + 16 + 8
    res, checks = {"workload": "PCB demux over C2: 16M x 64B TCP frames, 65536 connections; table sets "
                               "established (all ESTABLISHED, 1% other TIME-WAIT entries, 1 listener), mixed "
                               "(90% active, 5% TIME-WAIT, 5% unknown -> listen list), mixed_nolisten (unknown "
                               "-> RESET)"}, []
    for name, tabs in tabsets.items():
        demux.load(eng, tabs)
        el, k = timed(separate)
        elf, kf = timed(fused)
        v = out.view(wl.reps, -1, 8)
        tiled = bool(torch.equal(v, v[:1].expand(wl.reps, -1, -1))) and bool(torch.equal(out, out2)) and \
            bool(torch.equal(rec2, wl.out))
        checks.append(("demux", "demux" if name == "established" else "demux_" + name, pool, tabs,
                       wl.out.view(wl.reps, -1, 16)[0].cpu().numpy(), v[0].cpu().numpy(), tiled))
        line = {"fused": {"kernel": "RX kernels with the lookup fused (ixg_rx_demux_batch_dev)",
                          "mpps": round(wl.n * steps / elf / 1e6, 2), "kernel_ms_avg": round(kf * 1e3, 4),
                          "alg_bytes_per_pkt": algf,
                          "roofline_frac": round(algf * wl.n / kf / 1e9 / PEAK_HBM_GBPS, 4)},
                "separate": {"kernel": "ixg_demux_s over RX records in HBM (ixg_demux_batch_dev)",
                             "mpps": round(wl.n * steps / el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
                             "alg_bytes_per_pkt": alg,
                             "roofline_frac": round(alg * wl.n / k / 1e9 / PEAK_HBM_GBPS, 4),
                             "line_floor_bytes_per_pkt": round(floor, 1),
                             "frac_vs_line_floor": round(floor * wl.n / k / 1e9 / PEAK_HBM_GBPS, 4)},
                "parity": "tiled-consistent" if tiled else "MISMATCH"}
        if name == "established":
            res.update(line)
        else:
            res[name] = line
    return res, checks


def events_line(dev, key, steps: int, rank: int, eng_for):
    """Event records over C3's IMIX shape: 16M frames tiled
    from 2^16 distinct ones, TCP (with payloads) and UDP half and half, every
    TCP flow an ESTABLISHED PCB. The RX and demux records come from the fused
    RX + demux launch (untimed); a step = one ixg_ev_batch_dev launch (count,
    group, scan, emit): the usys_tcp_recv / usys_udp_recv descriptors, dense and in
    frame order."""
    import torch
    from ix_amd import demux, events, ixgrx
    wl = Workload("c3", seed=0x1BC000 + 97 * rank, dev=dev, pool=1 << 16)
    eng = eng_for(0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    pool, P = wl.pool, wl.pool.n
    wl.launch(eng, sp)
    torch.cuda.synchronize()
    r0 = wl.out[:P].cpu().numpy().reshape(-1).view(ixgrx.REC_DTYPE)
    tcp = np.nonzero(r0["verdict"] == ixgrx.V["TCP"])[0]
    keys = demux.tcp_keys(pool.blob, pool.offsets()[tcp])
    keys["id"] = np.arange(tcp.size, dtype=np.uint32)
    tabs = demux.DemuxTables.build(eng.cfg, keys, np.zeros(0, demux.PCB_DTYPE), np.zeros(0, demux.LISTEN_DTYPE))
    demux.load(eng, tabs)
    n = wl.n
    rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    dmx = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    demux.rx_demux_dev(eng, wl.blob.data_ptr(), wl.off.data_ptr(), wl.len.data_ptr(), 0, n, rec.data_ptr(),
                       dmx.data_ptr(), sp)
    rng = np.random.default_rng(3)
    pcbs = np.zeros(tcp.size, dtype=events.PCB_DTYPE)
    pcbs["pcb_idx"] = rng.integers(0, 1 << 48, size=tcp.size, dtype=np.uint64)
    pcbs["cookie"] = rng.integers(0, 1 << 63, size=tcp.size, dtype=np.uint64)
    tp = torch.from_numpy(pcbs.view(np.uint8)).to(dev)
    ev = torch.empty((n, 40), dtype=torch.uint8, device=dev)
    fi = torch.empty(n, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    io = 0x7F0000000000

    def launch():
        events.batch_dev(eng, wl.blob.data_ptr(), wl.off.data_ptr(), 0, rec.data_ptr(), dmx.data_ptr(), tp.data_ptr(),
                         tcp.size, n, io, 0, ev.data_ptr(), fi.data_ptr(), cnt.data_ptr(), sp)
    for _ in range(LINE_WARMUP):
        launch()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, c in evs:
        a.record(stream)
        launch()
        c.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = float(np.mean([a.elapsed_time(c) * 1e-3 for a, c in evs]))
    m = int(cnt.item())
    # tiling: each repetition's events are the first one's, frame indices
    # shifted by the pool size and iomap addresses by the repetition's span
    reps = wl.reps
    cp = m // reps
    e = ev[:m].cpu().numpy().reshape(-1).view(events.EV_DTYPE).reshape(reps, cp) if m % reps == 0 else None
    f = fi[:m].cpu().numpy().astype(np.int64).reshape(reps, cp) if e is not None else None
    tiled = e is not None
    if tiled:
        span = int(wl.off[P].item())
        sh = (np.arange(reps, dtype=np.uint64) * np.uint64(span))[:, None]
        udp = e["sysnr"] == events.USYS_UDP_RECV
        tiled = bool((f - f[:1] == np.arange(reps)[:, None] * P).all()
                     and (e["sysnr"] == e[:1]["sysnr"]).all() and (e["argb"] == e[:1]["argb"]).all()
                     and (e["argd"] == e[:1]["argd"]).all()
                     and (np.where(udp, e["arga"] - sh, e["arga"]) == e[:1]["arga"]).all()
                     and (e["argc"] - sh == e[:1]["argc"]).all())
    n_tcp = int((e[0]["sysnr"] == events.USYS_TCP_RECV).sum()) * reps if e is not None else 0
    # algorithmic bytes: count pass reads the record and demux record (24 B
    # per frame), emit pass reads them again, then per event the 40-byte
    # descriptor + 4-byte frame index written, + the 16-byte PCB entry read
    # for a TCP event
    alg = 48 * n + 44 * m + 16 * n_tcp
    check = ("events", pool, tabs, pcbs, io, e[0] if e is not None else None,
             f[0] if f is not None else None, tiled)
    return {"workload": "event records over C3's shape: 16M IMIX frames (TCP with payload + UDP), "
                        f"{tcp.size} established connections; kernels ixg_ev_count + ixg_ev_group + ixg_ev_scan + ixg_ev_emit",
            "events_per_launch": m, "tcp_events": n_tcp,
            "mevents_per_s": round(m * steps / el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
            "alg_bytes_per_frame": round(alg / n, 1), "roofline_frac": round(alg / k / 1e9 / PEAK_HBM_GBPS, 4),
            "parity": "tiled-consistent" if check[-1] else "MISMATCH"}, check


def tcpx_line(dev, steps: int, rank: int, eng_for):
    """The rest of the tcp_input head (tcp_in.c:230-241) over
    C2's shape: 16M 64-B TCP frames tiled from 2^16 distinct ones; the RX
    records come from one untimed RX launch, a step = one
    ixg_tcp_ext_batch_dev launch (struct ixg_tcp_ext per frame)."""
    import torch
    from ix_amd import tcpx
    wl = Workload("c2", seed=0x1BF100 + 97 * rank, dev=dev, pool=1 << 16)
    eng = eng_for(0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    wl.launch(eng, sp)
    ext = torch.empty((wl.n, 16), dtype=torch.uint8, device=dev)

    def launch():
        tcpx.batch_dev(eng, wl.blob.data_ptr(), None, wl.stride, wl.out.data_ptr(), wl.n, ext.data_ptr(), 0, sp)
    for _ in range(LINE_WARMUP):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, c in ev:
        a.record(stream)
        launch()
        c.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = float(np.mean([a.elapsed_time(c) * 1e-3 for a, c in ev]))
    v = ext.view(wl.reps, -1, 16)
    tiled = bool(torch.equal(v, v[:1].expand(wl.reps, -1, -1)))
    # algorithmic bytes per frame: the record (16), the IHL byte, the 14 header
    # bytes the head converts (ports, seqno, ackno, wnd) and the 16-byte ext
    # written; the frame lines they sit in are the frame itself at C2's size
    alg = 16 + 1 + 14 + 16
    # what a memory system fetching whole 128-B lines must move: the lines
    # holding the IHL dword (bytes 12..15) and the 20 header bytes from 2
    # before the TCP header, + the record and the ext (at C2's 60-B stride
    # every line of the frames holds such a byte)
    offs = wl.pool.offsets().astype(np.int64)
    t = offs + 14 + 4 * (wl.pool.blob[offs + 14].astype(np.int64) & 15)
    nl = lines_touched(np.concatenate([offs + 12, t - 2]), np.concatenate([offs + 16, t + 18]))
    floor = nl * 128 / wl.pool.n + 32
    check = ("tcpx", wl.pool, wl.out.view(wl.reps, -1, 16)[0].cpu().numpy(), v[0].cpu().numpy(), tiled)
    fused = tcpx_fused(wl, eng, ext, steps, sp, stream)
    return {"workload": "tcp_input head rest (seqno/ackno/wnd/tcplen) over C2: 16M x 64B TCP frames; kernel ixg_tcpx_s",
            "fused": fused,
            "mpps": round(wl.n * steps / el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
            "alg_bytes_per_pkt": alg, "roofline_frac": round(alg * wl.n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "line_floor_bytes_per_pkt": round(floor, 1),
            "frac_vs_line_floor": round(floor * wl.n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "gbps_frame_bytes": round((16 + wl.stride + 16) * wl.n / k / 1e9, 1),
            "parity": "tiled-consistent" if tiled else "MISMATCH"}, check


def tcpx_fused(wl, eng, ext, steps, sp, stream):
    """RX and the tcp_input head in one pass (ixg_rx_tcpx_batch_dev, VERDICT
    r05 next #3): over the same C2 batch the coalesced kernel writes each
    frame's ixg_tcp_ext from the header dwords it has just parsed
    (ixg_rx_fastc_tcpx_s), so the frames are read once. Timed against the
    plain RX launch (ixg_rx_fastc_s) interleaved in the same process; the
    ratio is the fused pass's cost over RX alone. Algorithmic bytes per
    frame: C2's 72 + the 16-byte ext written = 88. Parity: the fused records
    and ext are the separate passes' (already checked against the oracle by
    the parity leg) and tiled across the batch."""
    import torch
    from ix_amd import tcpx
    rec2 = torch.empty_like(wl.out)
    ext2 = torch.empty_like(ext)

    def fused():
        tcpx.rx_batch_dev(eng, wl.blob.data_ptr(), None, wl.len.data_ptr(), wl.stride, wl.n, rec2.data_ptr(),
                          ext2.data_ptr(), 0, sp)
    for _ in range(LINE_WARMUP):
        fused()
        wl.launch(eng, sp)
    kf, kr = [], []
    t_el = 0.0
    for _ in range(4):
        for fn, acc in ((fused, kf), (lambda: wl.launch(eng, sp), kr)):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for a, c in ev:
                a.record(stream)
                fn()
                c.record(stream)
            torch.cuda.synchronize()
            if fn is fused:
                t_el += time.perf_counter() - t0
            acc.extend(a.elapsed_time(c) * 1e-3 for a, c in ev)
    k, k_rx = float(np.mean(kf)), float(np.mean(kr))
    same = bool(torch.equal(rec2, wl.out)) and bool(torch.equal(ext2, ext))
    alg = 72 + 16
    return {"workload": "RX + tcp_input head rest in one pass over C2 (16M x 64B TCP frames); kernel ixg_rx_fastc_tcpx_s",
            "mpps": round(wl.n * steps * 4 / t_el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
            "rx_alone_kernel_ms_avg": round(k_rx * 1e3, 4), "ratio_vs_rx_alone": round(k / k_rx, 3),
            "alg_bytes_per_pkt": alg,
            "roofline_frac": round(alg * wl.n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "parity": "same-as-separate-passes" if same else "MISMATCH"}


def icmp_line(dev, steps: int, rank: int, eng_for, n: int = 1 << 24):
    """ICMP echo reflect (dp/net/icmp.c:44-71,88-91) over a
    ping flood: n default pings (56-B payload, 98-B frames, packed at
    100-B offsets) tiled from 2^14 distinct ones in HBM, every frame an echo
    request; the RX records come from one untimed RX launch, a step = one
    ixg_icmp_reflect_dev launch (each lane rewrites its own frame: the lane
    path). The parity copy is reflected once on its own buffer (a step
    rewrites its frames in place, so the timed buffer's frames are replies
    after the first step)."""
    import torch
    from ix_amd import icmp, traces
    rng = np.random.default_rng(0x1BF200 + 97 * rank)
    pool = traces.pack([traces.icmp_echo(rng, 56) for _ in range(1 << 14)])
    reps = n // pool.n
    span = int(pool.off[-1]) + 100
    assert int(pool.len[0]) == 98 and int(pool.off[1]) == 100 and span == 100 * pool.n
    blob = torch.from_numpy(np.ascontiguousarray(pool.blob[:span])).to(dev).repeat(reps)
    blob = torch.cat([blob, torch.zeros(64, dtype=torch.uint8, device=dev)])
    off = torch.arange(n, dtype=torch.int64, device=dev) * 100
    lens = torch.full((n,), 98, dtype=torch.int16, device=dev)
    rec = torch.empty((n, 16), dtype=torch.uint8, device=dev)
    eng = eng_for(0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    eng.batch_dev(blob.data_ptr(), off.data_ptr(), lens.data_ptr(), 0, n, rec.data_ptr(), None, sp)
    mac, host = bytes([2, 9, 8, 7, 6, 5]), 0xc0a80001
    # the parity copy: the pool once, reflected once
    pb = torch.from_numpy(np.ascontiguousarray(pool.blob)).to(dev)
    icmp.reflect_dev(eng, pb.data_ptr(), off[:pool.n].data_ptr(), 0, rec.data_ptr(), pool.n, mac, host, sp)

    def launch():
        icmp.reflect_dev(eng, blob.data_ptr(), off.data_ptr(), 0, rec.data_ptr(), n, mac, host, sp)
    for _ in range(LINE_WARMUP):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, c in ev:
        a.record(stream)
        launch()
        c.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = float(np.mean([a.elapsed_time(c) * 1e-3 for a, c in ev]))
    v = blob[:reps * span].view(reps, span)
    tiled = bool(torch.equal(v, v[:1].expand(reps, -1)))
    # algorithmic bytes per frame: the record (16), the frame bytes the reply
    # is built from (source MAC, source IP, the 64-B message: 74) and the 23
    # header bytes written
    alg = 16 + 6 + 4 + 64 + 23
    # what whole 128-B lines make it move: the record, every line of the
    # frames read, every line holding a rewritten byte written back
    o = pool.off.astype(np.int64)
    rd = lines_touched(o + 6, o + 98)
    wr = lines_touched(np.concatenate([o, o + 26]), np.concatenate([o + 12, o + 38]))
    floor = 16 + (rd + wr) * 128 / pool.n
    check = ("icmp", pool, rec[:pool.n].cpu().numpy(), pb.cpu().numpy(), mac, host, tiled)
    return {"workload": f"ICMP echo reflect over a ping flood: {n} x 98-B echo requests (56-B payload) in HBM; "
                        "kernel ixg_icmp_reflect_o",
            "mpps": round(n * steps / el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
            "alg_bytes_per_pkt": alg, "roofline_frac": round(alg * n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "line_floor_bytes_per_pkt": round(floor, 1),
            "frac_vs_line_floor": round(floor * n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "parity": "tiled-consistent" if tiled else "MISMATCH"}, check


def tx_line(dev, steps: int, eng, kind: str, n: int):
    """TX header build + checksums: n segments tiled from 2^16
    distinct ones, frames packed 16-byte aligned in HBM; a step = one
    ixg_tx_batch_dev launch (full checksums, as the NIC puts them on the
    wire)."""
    import torch
    from ix_amd import tx
    b = tx.make_segments(kind, n, seed=0x1BE000 + n, pool=1 << 16, layout="packed")
    tx.set_macs(eng, b.src_mac, b.dmacs)
    buf = torch.from_numpy(b.buf).to(dev)
    segs = torch.from_numpy(b.segs.view(np.uint8)).to(dev)
    out = torch.empty(b.out_size, dtype=torch.uint8, device=dev)
    out_len = torch.empty(n, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream()

    def launch():
        tx.batch_dev(eng, buf.data_ptr(), segs.data_ptr(), n, out.data_ptr(), out_len.data_ptr(), 0,
                     stream.cuda_stream)
    for _ in range(LINE_WARMUP):
        launch()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, c in ev:
        a.record(stream)
        launch()
        c.record(stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    k = float(np.mean([a.elapsed_time(c) * 1e-3 for a, c in ev]))
    pool = 1 << 16
    reps = n // pool
    span = int(b.segs["out_off"][pool]) if reps > 1 else b.out_size
    rows = out[:reps * span].view(reps, span)
    tiled = bool(torch.equal(rows, rows[:1].expand(reps, -1)))
    L = b.segs["seg_len"].astype(np.float64)
    flen = 34 + L + np.where(b.segs["proto"] == 17, 8, 0)
    alg = float((40 + L + flen + 2).mean())  # descriptor + segment read, frame + length written
    first = (b.buf[:int(b.segs["seg_off"][pool]) if reps > 1 else b.buf.size + 0], b.segs[:pool].copy(),
             b.src_mac, b.dmacs, out[:span].cpu().numpy(), out_len[:pool].cpu().numpy().astype(np.uint16))
    return {"workload": f"TX build over {n} {kind} segments (frames packed in HBM, full checksums; "
                        "kernel ixg_tx_build)",
            "mpps": round(n * steps / el / 1e6, 2), "kernel_ms_avg": round(k * 1e3, 4),
            "alg_bytes_per_pkt": round(alg, 1), "roofline_frac": round(alg * n / k / 1e9 / PEAK_HBM_GBPS, 4),
            "parity": "tiled-consistent" if tiled else "MISMATCH"}, ("tx", kind, first, tiled)


def mbuf_path(eng, n: int, seed: int, reps: int = 3):
    """IX's own layout end to end: n C2 frames in 2112-byte
    mbufs in host memory -> ixg_rx_batch_mbufs (gather into pinned staging,
    H2D, kernels, D2H of records; pipelined in chunks over two stages) ->
    records in host memory."""
    from ix_amd import ixgrx, traces
    tr = traces.make_trace("tcp64", n, seed=seed, pool=1 << 16)
    arena, ptrs = ixgrx.make_mbufs(tr)
    eng.batch_mbufs(ptrs[:1024])
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        rec = eng.batch_mbufs(ptrs)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    tiled = bool((rec.view(np.uint8).reshape(n // (1 << 16), -1) ==
                  rec.view(np.uint8).reshape(n // (1 << 16), -1)[:1]).all())
    return {"mpps": round(n / best / 1e6, 2), "seconds": round(best, 4), "frames": n,
            "note": "host mbufs -> records in host memory, one host thread (IX's per-CPU model)",
            "parity": "tiled-consistent" if tiled else "MISMATCH"}, ("mbufs", tr, ptrs, arena, rec)


LOOP_EXE = os.path.join(ROOT, "examples", "bin", "ix_async_loop")


def write_frames_file(tr, path: str) -> None:
    """The frames file examples/ix_async_loop.c reads: u32 count, u16
    lengths, then the frames back to back."""
    offs = tr.offsets().astype(np.int64)
    with open(path, "wb") as f:
        f.write(np.uint32(tr.n).tobytes())
        f.write(tr.len.astype("<u2").tobytes())
        for o, L in zip(offs, tr.len.astype(np.int64)):
            f.write(tr.blob[o:o + L].tobytes())


def _loop_run(path: str, mode: str, timeout: float, env: dict | None = None, **kw) -> dict:
    import subprocess
    args = [LOOP_EXE, path, mode] + [f"{k}={v}" for k, v in kw.items()]
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout,
                       env=None if env is None else {**os.environ, **env})
    if r.returncode != 0:
        return {"error": f"rc={r.returncode}: {r.stderr.strip()[-300:]}"}
    return json.loads(r.stdout.strip().splitlines()[-1])


def host_path(seconds: float = 3.0, threads=(1, 4, 16)):
    """the path starts and ends in host memory. IX's run loop
    (examples/ix_async_loop.c: per sys_bpoll iteration <= 64 frames off the
    RX queue, dp/core/ethqueue.c:71,117-149) drives libixgrx's asynchronous
    host path, one context per host thread (IX's per-CPU model), over C2's
    64-B frames in 2112-B IX mbufs: aggregate Mpkt/s and submit->poll
    latency at 1/4/16 threads, next to cpu_baseline, with the library's
    per-thread breakdown (ixg_rx_async_stats). Then 1514-B frames at 16
    threads, gathered and read in place from registered mbuf memory (zero
    copy: ixg_rx_register_memory; frames under IXG_ZC_MIN_LEN are gathered
    anyway, so C2's frames never take it). Beside them, the latency of one
    synchronous ixg_rx_batch_mbufs call at n = 64 / 1K / 64K frames and of
    one 64-frame batch through the asynchronous path (staged copies, and
    IXG_ASYNC_DIRECT: kernels on pinned host memory). Thread 0's first pass
    of the C2 loop and of the zero-copy loop are kept for the oracle check."""
    import tempfile
    from ix_amd import traces
    if not os.path.exists(LOOP_EXE):
        return {"error": f"{LOOP_EXE} not built"}, None
    pool = traces.make_trace("tcp64", 1 << 16, seed=0x1BF000)
    tmp = tempfile.mkdtemp(prefix="ixg_hostpath_")
    fpath = os.path.join(tmp, "frames.bin")
    write_frames_file(pool, fpath)
    res = {"workload": "C2 frames (60 B, 2^16 distinct) in 2112-B IX mbufs on the host; records to host memory",
           "sync_latency": {}, "async_latency": {}, "loop": {}}
    for n in (64, 1024, 65536):
        res["sync_latency"][f"n{n}"] = _loop_run(fpath, "sync", 120, n=n, seconds=1.0)
    for direct in (0, 1):
        res["async_latency"]["direct" if direct else "copy"] = _loop_run(fpath, "async1", 120, n=64, seconds=1.0,
                                                                         direct=direct)
    checks = []

    def loop(path, name, tr, dump_name=None, **kw):
        dump = os.path.join(tmp, dump_name) if dump_name else None
        if dump:
            kw["dump"] = dump
        res["loop"][name] = _loop_run(path, "loop", 300, seconds=seconds, batch=64, **kw)
        if dump:
            recs = np.fromfile(dump, dtype=np.uint8).reshape(-1, 16) if os.path.exists(dump) else None
            if recs is not None and recs.shape[0] == tr.n:
                checks.append(("hostpath", tr, recs, "hostpath_" + name))
            else:
                res["parity"] = "MISMATCH (no records dumped)"

    for t in threads:
        loop(fpath, f"threads{t}", pool, "dump.bin" if t == threads[0] else None, threads=t, arena=1 << 17)
    # 1514-B frames at the largest thread count: gathered, and read in place
    # from the registered mbuf arenas over the host link
    big = traces.make_trace("tcp1514", 1 << 14, seed=0x1BF001)
    bpath = os.path.join(tmp, "frames1514.bin")
    write_frames_file(big, bpath)
    t = threads[-1]
    loop(bpath, f"tcp1514_threads{t}", big, None, threads=t, arena=1 << 15)
    loop(bpath, f"tcp1514_threads{t}_zero_copy", big, "dump_zc.bin", threads=t, arena=1 << 15, register=1)
    res.setdefault("parity", "pending oracle")
    return res, checks


def xgmi_leg(wl, eng, dist, world: int, rank: int, reps: int = 3):
    """SURVEY 8(e) option 1 (opt-in, N > 1): the whole batch starts in GPU
    0's HBM (world slices of the workload), one RCCL scatter over xGMI hands
    every rank its slice, every rank runs the kernels, one RCCL gather brings
    the 16-byte records back to GPU 0. Phases timed with barriers; the max
    over ranks of each. Fixed-stride workloads."""
    import torch
    from ix_amd import shard
    assert wl.off is None
    nbytes = wl.n * wl.stride
    mine = wl.blob[:nbytes]
    full = mine.repeat(world) if rank == 0 else None
    stream = torch.cuda.current_stream()
    best = None
    for _ in range(reps):
        ts = []
        for phase in range(3):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            if phase == 0:
                shard.scatter_slices(full, mine, dist)
            elif phase == 1:
                wl.launch(eng, stream.cuda_stream)
            else:
                back = shard.gather_slices(wl.out, dist)
            torch.cuda.synchronize()
            ts.append(shard.max_over_ranks(time.perf_counter() - t0, dist, device="cuda"))
        best = ts if best is None or sum(ts) < sum(best) else best
    sc, kr, ga = best
    ok = True
    if rank == 0:
        v = back.view(world, wl.reps, -1, 16)
        ok = bool(torch.equal(v, v[:1, :1].expand(world, wl.reps, -1, -1)))
    return {"scatter_ms": round(sc * 1e3, 3), "kernel_ms": round(kr * 1e3, 3), "gather_ms": round(ga * 1e3, 3),
            "mpps_end_to_end": round(world * wl.n / (sc + kr + ga) / 1e6, 2),
            "scatter_gbps": round((world - 1) * nbytes / sc / 1e9, 1),
            "gather_gbps": round((world - 1) * wl.n * 16 / ga / 1e9, 1),
            "note": "batch in GPU 0's HBM -> RCCL scatter over xGMI -> kernels on every GPU -> RCCL gather of "
                    "records to GPU 0", "parity": "tiled-consistent" if ok else "MISMATCH"}


C4_FRAMES = 64 * 1024 * 1024  # BASELINE.json configs[3]: one 64M-frame batch of 1514-B frames


def strong_leg(dev, run_slice, dist, world: int, rank: int, n_total: int = C4_FRAMES, pool: int = 1 << 13,
               reps: int = 3, warmup: int = 10):
    """C4 as BASELINE.json states it (configs[3], SURVEY.md 8(e) option 1):
    ONE batch of n_total 1514-B frames (stride 1516) that starts in GPU 0's
    HBM, split by shard.shard_bounds into contiguous slices; grouped RCCL
    send/recv hand every rank its slice over xGMI, every rank runs the
    kernels on its slice, and the 16-byte records come back into the
    batch's record array on GPU 0. Strong scaling: the batch is the same at
    every N (at N=1 there is nothing to move). Scatter, kernel and gather
    are timed separately, each bracketed by synchronize + barrier, max over
    ranks; the best of `reps` rounds. `run_slice(blob, lens, stride, m, out,
    stream)` runs the hot path on one slice (the HIP engine in bench.py;
    the oracle in the gloo test of this leg, tests/test_multi.py)."""
    import torch
    from ix_amd import shard, traces
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    def barrier():
        sync()
        if world > 1:
            dist.barrier()
        sync()

    # every rank derives the batch's lengths from the same pool; only rank
    # 0 materialises the batch
    pool_tr = traces.make_trace("tcp1514", pool, seed=0x1B4C4)
    S = pool_tr.stride
    bounds = shard.shard_bounds(np.tile(pool_tr.len, n_total // pool), world)
    s, e = bounds[rank]
    wl = Workload("c4", seed=0x1B4C4, dev=dev, n=n_total, pool=pool) if rank == 0 else None
    stream = torch.cuda.current_stream().cuda_stream if cuda else None
    out = wl.out if rank == 0 else torch.empty((e - s, 16), dtype=torch.uint8, device=dev)
    mine = out[s:e] if rank == 0 else out
    # untimed warm-up of the kernel phase (first-launch allocations, the
    # clock settling under load): each rank on its own part of
    # the batch, or the head of it before the slices exist
    if warmup and cuda and e > s:
        m = min(e - s, pool * 128)
        if rank == 0:
            src_blob, src_len = wl.blob, wl.len[:m]
        else:  # the batch's own frames (tiled pool), the slice arrives only in the timed scatter
            reps_w = (m + pool - 1) // pool
            src_blob = torch.zeros(reps_w * pool * S + traces.TAIL_PAD, dtype=torch.uint8, device=dev)
            src_blob[:reps_w * pool * S].view(reps_w, -1).copy_(
                torch.from_numpy(pool_tr.blob[:pool * S]).to(dev).unsqueeze(0).expand(reps_w, -1))
            src_len = torch.from_numpy(pool_tr.len.view(np.int16)).to(dev).repeat(reps_w)[:m].contiguous()
        for _ in range(warmup):
            run_slice(src_blob, src_len, S, m, mine[:m], stream)
        barrier()
        del src_blob, src_len
    best = None
    for _ in range(reps):
        ts = []
        barrier()
        t0 = time.perf_counter()
        if world > 1:
            blob, lens = shard.scatter_frames(wl.blob if wl else None, wl.len if wl else None, S, bounds, dist, dev)
        else:
            blob, lens = wl.blob, wl.len
        barrier()
        ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        if e > s:
            run_slice(blob, lens, S, e - s, mine, stream)
        barrier()
        ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        if world > 1:
            shard.gather_frame_records(mine, bounds, dist, out if rank == 0 else None)
        barrier()
        ts.append(time.perf_counter() - t0)
        if world > 1:
            ts = [shard.max_over_ranks(t, dist, device="cuda" if dist.get_backend() == "nccl" else "cpu")
                  for t in ts]
        best = ts if best is None or sum(ts) < sum(best) else best
        del blob, lens
    sc, kr, ga = best
    sizes = [b - a for a, b in bounds]
    res = {"workload": f"C4 (configs[3]): one batch of {n_total} x 1514B IPv4/TCP frames (stride {S}) in GPU 0's "
                       f"HBM, split by shard_bounds across {world} GPU(s)",
           "scaling": "strong", "frames": n_total, "slice_frames": [min(sizes), max(sizes)],
           "scatter_ms": round(sc * 1e3, 3), "kernel_ms": round(kr * 1e3, 3), "gather_ms": round(ga * 1e3, 3),
           "mpps_device_resident": round(n_total / kr / 1e6, 2),
           "mpps_end_to_end": round(n_total / (sc + kr + ga) / 1e6, 2),
           "note": "kernel = every rank's slice already in its own HBM (slowest rank); end_to_end adds the xGMI "
                   "scatter of frames from GPU 0 (grouped RCCL send/recv, one per peer) and the gather of records"}
    if world > 1:
        res["scatter_gbps"] = round((n_total - sizes[0]) * S / sc / 1e9, 1)
        res["gather_gbps"] = round((n_total - sizes[0]) * 16 / ga / 1e9, 1)
    alg = float(alg_bytes(pool_tr).mean())
    res["alg_bytes_per_pkt"] = round(alg, 1)
    res["roofline_frac_per_gpu"] = round(alg * max(sizes) / kr / 1e9 / PEAK_HBM_GBPS, 4)
    check = None
    if rank == 0:
        tiled, first = wl.snapshot()
        check = ("rx", "c4_strong", wl.pool, wl.flags, first, tiled)
        res["parity"] = "tiled-consistent" if tiled else "MISMATCH"
        del wl
    return res, check


def summary(res: dict) -> dict:
    """Every line of the run in one compact object, the last key of the JSON
    line, so a reader that keeps only the line's tail (the driver's record
    keeps ~2 KB) still sees each config's roofline fraction, kernel time per
    launch, rate and parity."""
    def ent(frac, ms, mpps, par):
        return {"frac": None if frac is None else round(frac, 4), "kernel_ms": None if ms is None else round(ms, 4),
                "mpps": None if mpps is None else round(mpps, 1), "parity": par}
    out = {"c2": ent(res["roofline"]["frac"], res["roofline"]["kernel_ms_avg"], res["value"], res.get("parity"))}
    if "bad_csum" in res:
        b = res["bad_csum"]
        out["c2b"] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
    if "secondary" in res:
        b = res["secondary"]
        out["c4"] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
    for name, b in res.get("lines", {}).items():
        out[name] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
        if "frac_vs_line_floor" in b:
            out[name]["frac_line_floor"] = b["frac_vs_line_floor"]
    if "c4_strong" in res:
        b = res["c4_strong"]
        out["c4_strong"] = ent(b["roofline_frac_per_gpu"], b["kernel_ms"], b["mpps_device_resident"], b.get("parity"))
    if "demux" in res:
        d = res["demux"]
        out["demux_fused"] = ent(d["fused"]["roofline_frac"], d["fused"]["kernel_ms_avg"], d["fused"]["mpps"],
                                 d["parity"])
        out["demux_sep"] = ent(d["separate"]["roofline_frac"], d["separate"]["kernel_ms_avg"], d["separate"]["mpps"],
                               d["parity"])
        if "frac_vs_line_floor" in d["separate"]:
            out["demux_sep"]["frac_line_floor"] = d["separate"]["frac_vs_line_floor"]
        for name in ("mixed", "mixed_nolisten"):
            if name in d:
                m = d[name]
                out["demux_" + name] = ent(m["fused"]["roofline_frac"], m["fused"]["kernel_ms_avg"],
                                           m["fused"]["mpps"], m["parity"])
                out["demux_" + name]["kinds"] = m.get("kinds")
    if "events" in res:
        b = res["events"]
        out["events"] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mevents_per_s"], b["parity"])
    if "tcpx" in res:
        b = res["tcpx"]
        out["tcpx"] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
        if "frac_vs_line_floor" in b:
            out["tcpx"]["frac_line_floor"] = b["frac_vs_line_floor"]
        if "fused" in b:
            f = b["fused"]
            out["rx_tcpx_fused"] = ent(f["roofline_frac"], f["kernel_ms_avg"], f["mpps"], f["parity"])
            out["rx_tcpx_fused"]["x_rx"] = f["ratio_vs_rx_alone"]
    if "icmp" in res:
        b = res["icmp"]
        out["icmp"] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
        if "frac_vs_line_floor" in b:
            out["icmp"]["frac_line_floor"] = b["frac_vs_line_floor"]
    for kind, b in res.get("tx", {}).items():
        out["tx_" + kind] = ent(b["roofline_frac"], b["kernel_ms_avg"], b["mpps"], b["parity"])
    hp = res.get("host_path", {})
    if "loop" in hp:
        lp = hp["loop"]
        out["host_path"] = {k.replace("threads", "t"): lp[k].get("mpps") for k in lp}
        top = max((k for k in lp if k.startswith("threads") and k[7:].isdigit()), key=lambda k: int(k[7:]), default=None)
        if top:
            out["host_path"]["t%s_max_latency_us" % top[7:]] = lp[top].get("latency_us", {}).get("max")
        # the worst batch of the 16-thread and zero-copy lines, split where its
        # time went (ixg_rx_async_stats: open / gpu / visible / returned; wait,
        # outside; poll(wait)'s naps and the longest)
        keys = ("total", "open", "gpu", "visible", "returned", "wait", "outside", "naps", "nap_max")
        zc = next((k for k in lp if k.endswith("_zero_copy")), None)
        for name, k in (("t%s_worst_us" % top[7:] if top else None, top), ("zc_worst_us", zc)):
            if name and k and "worst_batch_us" in lp[k]:
                w = lp[k]["worst_batch_us"]
                out["host_path"][name] = {x: w[x] for x in keys if x in w}
        out["host_path"]["parity"] = hp.get("parity")
    if "cpu_baseline" in res:
        out["cpu_baseline_mpps"] = res["cpu_baseline"]["value"]
    return out


def load_traffic(workload: str):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary, or None."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None, None
    d = json.load(open(p))
    e = d.get(workload)
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), e.get("source")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # (the first launches of a memory-heavy run go through a power-management
    # transient: C2 runs 0.217 ms for ~8 launches, 0.25 ms around launch 20,
    # 0.232 ms by launch 40 and ~0.217 ms after that)
    ap.add_argument("--warmup", type=int, default=60)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--secondary", default="c4", help="second workload line ('' to skip)")
    ap.add_argument("--extra", default="c3,c5,c5r", help="further workload lines (BASELINE configs[2] and [4], "
                                                          "[4] also in the reference's semantics; '' to skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-copy", action="store_true")
    ap.add_argument("--host-seconds", type=float, default=3.0, help="seconds per host_path loop run")
    ap.add_argument("--no-demux", action="store_true")
    ap.add_argument("--no-tx", action="store_true")
    ap.add_argument("--no-bad", action="store_true", help="skip the C2 bad-checksum line")
    ap.add_argument("--xgmi", action="store_true", help="N > 1: add the equal-slice RCCL scatter/gather leg")
    ap.add_argument("--no-strong", action="store_true", help="skip the C4 one-batch strong-split line")
    ap.add_argument("--strong-n", type=int, default=C4_FRAMES, help="C4 strong-split batch size (frames)")
    ap.add_argument("--frames", "--n", dest="n", type=int, default=None, help="override frames per GPU")
    args = ap.parse_args()

    import torch
    from ix_amd import ixgrx, traces

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # IXG_BENCH_BACKEND=gloo (with ranks sharing a card: device = LOCAL_RANK
    # mod the device count) rehearses the N > 1 path on a one-GPU box; the
    # driver's multi-GPU runs use the default, nccl (RCCL), one rank per GPU
    backend = os.environ.get("IXG_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    key = traces.RSS_KEY
    engs = {}

    def engine(flags):
        if flags not in engs:
            engs[flags] = ixgrx.RxEngine(ixgrx.Config(key, 128, rank % 128, flags), device=local)
        return engs[flags]

    wl = Workload(args.workload, seed=0x1B0000 + 2 + 97 * rank, dev=dev, n=args.n)
    el, kavg, kmin = time_steps(wl, engine(wl.flags), args.steps, args.warmup, dist, world)
    tiled, first = wl.snapshot()
    checks = [("rx", wl.name, wl.pool, wl.flags, first, tiled)]
    primary = (wl.name, wl.pool, wl.flags)
    wl_name = wl.name
    total = wl.n * args.steps * world
    mpps = total / el / 1e6
    bpl = wl.bytes_per_pkt * wl.n  # algorithmic bytes per launch (one GPU)
    achieved = bpl / kavg / 1e9
    traffic, tsrc = load_traffic(args.workload)
    res = {
        "metric": METRIC,
        "value": round(mpps, 2),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic ({wl.pool.n} distinct frames tiled to {wl.n} per GPU, valid checksums)",
        "config": {"workload": wl.desc, "frames_per_gpu": wl.n, "wire_bytes_per_frame": wl.wire_bytes,
                   "layout": "fixed stride" if wl.off is None else "packed + u64 offsets",
                   "parallelism": f"shard{world}"},
        "gbps_algorithmic": round(mpps * wl.bytes_per_pkt / 1e3, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                     "alg_bytes_per_pkt": round(wl.bytes_per_pkt, 2), "kernel_ms_avg": round(kavg * 1e3, 4),
                     "kernel_ms_min": round(kmin * 1e3, 4),
                     "kernel": kernels(wl),
                     "traffic_source": tsrc},
        "parity": "tiled-consistent" if tiled else "MISMATCH",
    }
    if args.workload == "c2" and not args.no_bad:
        # the same shape with checksum failures: the verdict/flag paths of
        # the fixed-shape kernel (a bad frame stays on the fast path)
        del wl
        torch.cuda.empty_cache()
        wlb = Workload("c2b", seed=0x1B0000 + 2 + 0x100 + 97 * rank, dev=dev)
        kb = max(5, args.steps // 2)
        elb, kbavg, _ = time_steps(wlb, engine(wlb.flags), kb, args.warmup, dist, world)
        tb, fb = wlb.snapshot()
        checks.append(("rx", wlb.name, wlb.pool, wlb.flags, fb, tb))
        vb = np.ascontiguousarray(fb).view(ixgrx.REC_DTYPE).reshape(-1)["verdict"]
        res["bad_csum"] = {"workload": wlb.desc, "mpps": round(wlb.n * kb * world / elb / 1e6, 2),
                           "kernel_ms_avg": round(kbavg * 1e3, 4),
                           "roofline_frac": round(wlb.bytes_per_pkt * wlb.n / kbavg / 1e9 / PEAK_HBM_GBPS, 4),
                           "verdicts_per_pool": {ixgrx.VERDICTS[int(v)]: int(c) for v, c in
                                                 zip(*np.unique(vb, return_counts=True))},
                           "parity": "tiled-consistent" if tb else "MISMATCH"}
        wl = wlb
    if args.xgmi and world > 1 and wl.off is None:
        res["xgmi"] = xgmi_leg(wl, engine(wl.flags), dist, world, rank)
    if args.secondary and args.secondary != args.workload:
        del wl
        torch.cuda.empty_cache()
        wl2 = Workload(args.secondary, seed=0x1B0000 + 4 + 97 * rank, dev=dev)
        el2, k2, _ = time_steps(wl2, engine(wl2.flags), max(5, args.steps // 2), args.warmup, dist, world)
        tiled2, first2 = wl2.snapshot()
        checks.append(("rx", wl2.name, wl2.pool, wl2.flags, first2, tiled2))
        m2 = wl2.n * max(5, args.steps // 2) * world / el2 / 1e6
        a2 = wl2.bytes_per_pkt * wl2.n / k2 / 1e9
        res["secondary"] = {"workload": wl2.desc, "mpps": round(m2, 2),
                            "gbps_algorithmic": round(m2 * wl2.bytes_per_pkt / 1e3, 1),
                            "roofline_frac": round(a2 / PEAK_HBM_GBPS, 4), "kernel_ms_avg": round(k2 * 1e3, 4),
                            "alg_bytes_per_pkt": round(wl2.bytes_per_pkt, 1),
                            "parity": "tiled-consistent" if tiled2 else "MISMATCH"}
        wl = wl2
    # the other configs as lines of their own: C3 (IMIX) and C5 (IPv4
    # options + IPv6), weak-scaled like the primary at N > 1; 40 warm-up
    # launches (C5's first ~35 launches after its batch is built run slower,
    # DESIGN.md 4.8)
    extras = [w for w in (args.extra.split(",") if args.extra else [])
              if w and w not in (args.workload, args.secondary)]
    for k, name in enumerate(extras):
        del wl
        wl = None
        torch.cuda.empty_cache()
        wle = Workload(name, seed=0x1B0000 + 6 + k + 97 * rank, dev=dev)
        ke = max(20, args.steps)
        ele, kea, kem = time_steps(wle, engine(wle.flags), ke, max(40, args.warmup), dist, world)
        te, fe = wle.snapshot()
        checks.append(("rx", wle.name, wle.pool, wle.flags, fe, te))
        me = wle.n * ke * world / ele / 1e6
        tr_e, _ = load_traffic(name)
        res.setdefault("lines", {})[name] = {
            "workload": wle.desc, "mpps": round(me, 2), "gbps_algorithmic": round(me * wle.bytes_per_pkt / 1e3, 1),
            "roofline_frac": round(wle.bytes_per_pkt * wle.n / kea / 1e9 / PEAK_HBM_GBPS, 4),
            "kernel_ms_avg": round(kea * 1e3, 4), "kernel_ms_min": round(kem * 1e3, 4),
            "alg_bytes_per_pkt": round(wle.bytes_per_pkt, 1), "traffic": tr_e, "kernel": kernels(wle),
            "parity": "tiled-consistent" if te else "MISMATCH"}
        if wle.off is not None:
            # the same launch against the bytes whole 128-B lines make it move
            fl = line_floor_bytes(wle.pool, wle.flags)
            res["lines"][name]["line_floor_bytes_per_pkt"] = round(fl, 1)
            res["lines"][name]["frac_vs_line_floor"] = round(fl * wle.n / kea / 1e9 / PEAK_HBM_GBPS, 4)
        wl = wle
    if not args.no_strong and args.workload == "c2":
        del wl
        wl = None
        torch.cuda.empty_cache()

        # one batch, one configuration: every rank's slice is processed as
        # the same device's frames (dev_idx 0), whatever the rank
        seng = ixgrx.RxEngine(ixgrx.Config(key, 128, 0, 0), device=local)

        def run_slice(blob, lens, S, m, out, stream):
            seng.batch_dev(blob.data_ptr(), None, lens.data_ptr(), S, m, out.data_ptr(), None, stream)
        res["c4_strong"], schk = strong_leg(dev, run_slice, dist, world, rank, n_total=args.strong_n)
        seng.close()
        if schk:
            checks.append(schk)
        torch.cuda.empty_cache()
    if not args.no_demux and args.workload == "c2":
        del wl
        torch.cuda.empty_cache()
        res["demux"], dchk = demux_line(dev, key, max(5, args.steps // 2), rank, engine)
        checks.extend(dchk)
        wl = None
    if not args.no_demux and args.workload == "c2":
        torch.cuda.empty_cache()
        res["events"], echk = events_line(dev, key, max(5, args.steps // 2), rank, engine)
        checks.append(echk)
        torch.cuda.empty_cache()
    if not args.no_demux and args.workload == "c2":
        torch.cuda.empty_cache()
        res["tcpx"], xchk = tcpx_line(dev, max(5, args.steps // 2), rank, engine)
        checks.append(xchk)
        torch.cuda.empty_cache()
    if not args.no_demux and args.workload == "c2":
        torch.cuda.empty_cache()
        res["icmp"], ichk = icmp_line(dev, max(5, args.steps // 2), rank, engine)
        checks.append(ichk)
        torch.cuda.empty_cache()
    if not args.no_tx and args.workload == "c2":
        torch.cuda.empty_cache()
        res["tx"] = {}
        for kind, n in (("tcp64", 16 * 1024 * 1024), ("tcp1514", 4 * 1024 * 1024)):
            res["tx"][kind], tchk = tx_line(dev, max(5, args.steps // 2), engine(0), kind, n)
            checks.append(tchk)
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_copy and args.workload == "c2":
        res["mbuf_path"], mchk = mbuf_path(engine(0), 1 << 21, seed=0x1BF000)
        checks.append(mchk)
    if rank == 0 and world == 1 and not args.no_copy and args.workload == "c2":
        res["host_path"], hchk = host_path(seconds=args.host_seconds)
        checks.extend(hchk)
    if rank == 0 and world == 1 and not args.no_copy:
        del wl
        torch.cuda.empty_cache()
        wlc = Workload(args.workload, seed=0x1B0000 + 2, dev=dev, n=args.n)
        res["copy_inclusive"] = copy_inclusive(wlc, engine(wlc.flags), key)
        if wlc.off is None:
            e2 = ixgrx.RxEngine(ixgrx.Config(key, 128, 0, wlc.flags), device=local)
            res["copy_inclusive"]["overlapped"] = copy_overlapped(wlc, [engine(wlc.flags), e2])
            e2.close()
        del wlc
    if rank == 0 and not args.no_cpu:
        # the CPU baseline is timed at N = 1 only; the oracle checks rank 0's
        # lines (and the records gathered back from every rank) at every N
        if world == 1:
            threads = min(16, os.cpu_count() or 1)
            pname, ptr, pflags = primary
            res["cpu_baseline"] = cpu_baseline(ptr, pflags, key, args.cpu_seconds, threads, pname)
        par = parity_leg(checks, key)
        res["parity_vs_oracle"] = par
        res["parity"] = par[wl_name]
        if "secondary" in res:
            res["secondary"]["parity"] = par[args.secondary]
        for name in res.get("lines", {}):
            res["lines"][name]["parity"] = par[name]
        if "c4_strong" in res:
            res["c4_strong"]["parity"] = par["c4_strong"]
        if "demux" in res:
            res["demux"]["parity"] = par["demux"]
            res["demux"]["kinds"] = par["demux_kinds"]
            for name in ("mixed", "mixed_nolisten"):
                if name in res["demux"]:
                    res["demux"][name]["parity"] = par["demux_" + name]
                    res["demux"][name]["kinds"] = par["demux_" + name + "_kinds"]
        if "host_path" in res and res["host_path"].get("parity") == "pending oracle":
            hp = [v for k, v in par.items() if k.startswith("hostpath_")]
            res["host_path"]["parity"] = "ok" if hp and all(v == "ok" for v in hp) else "MISMATCH"
        if "mbuf_path" in res:
            res["mbuf_path"]["parity"] = par["mbufs"] if res["mbuf_path"]["parity"] != "MISMATCH" else "MISMATCH"
        for kind in res.get("tx", {}):
            res["tx"][kind]["parity"] = par["tx_" + kind]
        if "events" in res:
            res["events"]["parity"] = par["events"]
        if "tcpx" in res:
            res["tcpx"]["parity"] = par["tcpx"]
            f = res["tcpx"].get("fused")
            if f and f["parity"] != "MISMATCH":
                f["parity"] = par["tcpx"]  # the separate passes' results, which the oracle checked
        if "icmp" in res:
            res["icmp"]["parity"] = par["icmp"]
        if "bad_csum" in res:
            res["bad_csum"]["parity"] = par["c2b"]
    if rank == 0:
        res["summary"] = summary(res)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    for e in engs.values():
        e.close()


if __name__ == "__main__":
    main()
