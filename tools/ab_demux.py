#!/usr/bin/env python3
"""Interleaved A/B of library builds on the fused RX + PCB demux launch
(ixg_rx_demux_batch_dev) over bench.py's demux workload (C2's shape, 2^16
established connections), in one process.

usage: ab_demux.py --libs ix_amd/libixgrx.so,tools/ablib/base.so
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--separate", action="store_true",
                    help="time the separate demux pass (ixg_demux_batch_dev) over RX records made once")
    ap.add_argument("--plain", action="store_true", help="time the RX launch alone (no demux) on the same frames")
    ap.add_argument("--tables", default="established", choices=["established", "mixed", "mixed_nolisten"],
                    help="bench.py demux_line's table sets")
    args = ap.parse_args()
    import torch
    import bench
    from ix_amd import demux, ixgrx, traces
    dev = torch.device("cuda:0")
    wl = bench.Workload("c2", seed=0x1BD000, dev=dev, pool=1 << 16)
    pool = wl.pool
    keys = demux.tcp_keys(pool.blob, pool.offsets())
    rng = np.random.default_rng(1)
    tw = keys[rng.random(keys.size) < 0.01].copy()
    tw["id"] += 1 << 20
    tw["remote_port"] ^= 1
    lis = np.array([(0, 80, 0, 7, 0)], dtype=demux.LISTEN_DTYPE)
    u = np.random.default_rng(2).random(keys.size)
    act = keys
    if args.tables != "established":  # 90 % active, 5 % TIME-WAIT, 5 % unknown (bench.py demux_line)
        act, tw = keys[u < 0.90], keys[(u >= 0.90) & (u < 0.95)]
        if args.tables == "mixed_nolisten":
            lis = np.zeros(0, demux.LISTEN_DTYPE)
    s = torch.cuda.current_stream()
    engs, outs = {}, {}
    for path in args.libs.replace("+", ",").split(","):
        e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY), lib_path=os.path.join(ROOT, path))
        demux.load(e, demux.DemuxTables.build(e.cfg, act, tw, lis))
        engs[os.path.basename(path)] = e
        outs[os.path.basename(path)] = (torch.zeros((wl.n, 16), dtype=torch.uint8, device=dev),
                                        torch.zeros((wl.n, 8), dtype=torch.uint8, device=dev))

    if args.separate:
        for v, e in engs.items():
            wl.launch(e, s.cuda_stream)
            outs[v][0].copy_(wl.out)
        torch.cuda.synchronize()

    def launch(v):
        r, d = outs[v]
        if args.plain:
            wl.launch(engs[v], s.cuda_stream)
        elif args.separate:
            demux.batch_dev(engs[v], wl.blob.data_ptr(), None, wl.stride, wl.n, r.data_ptr(), d.data_ptr(),
                            s.cuda_stream)
        else:
            demux.rx_demux_dev(engs[v], wl.blob.data_ptr(), None, wl.len.data_ptr(), wl.stride, wl.n, r.data_ptr(),
                               d.data_ptr(), s.cuda_stream)
    for v in engs:
        for _ in range(3):
            launch(v)
    torch.cuda.synchronize()
    first = next(iter(outs.values()))
    same = {v: bool(torch.equal(o[0], first[0]) and torch.equal(o[1], first[1])) for v, o in outs.items()}
    times = {v: [] for v in engs}
    for _ in range(args.rounds):
        for v in engs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(args.k):
                launch(v)
            b.record(s)
            torch.cuda.synchronize()
            times[v].append(a.elapsed_time(b) / args.k)
    res = {v: {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4),
               "frac80": round(wl.n * 80 / (np.median(t) * 1e-3) / 8e12, 4), "same_as_first": same[v]}
           for v, t in times.items()}
    kind = "plain RX (no demux)" if args.plain else ("separate" if args.separate else "fused") + " demux"
    print(json.dumps({"workload": kind + " over C2, tables " + args.tables, "results": res}),
          flush=True)


if __name__ == "__main__":
    main()
