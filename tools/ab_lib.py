#!/usr/bin/env python3
"""Interleaved A/B of library BUILDS in one process: the working tree's
ix_amd/libixgrx.so against builds of other revisions (tools/build_rev.sh).
Box-to-box variance on the pool is larger than most kernel changes, so a
change is judged only against a reference timed in the same process.

usage: ab_lib.py --workload c4 --libs ix_amd/libixgrx.so,tools/ablib/base.so [--general]
"""
import argparse
import re
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--general", action="store_true", help="general kernel alone (ixg_rx_set_split) for every build")
    ap.add_argument("--splits", default=None, help="comma list of ixg_rx_set_split modes to time per build "
                                                     "(auto, fast, short, long, general)")
    args = ap.parse_args()
    import torch
    import bench
    from ix_amd import ixgrx, traces
    dev = torch.device("cuda:0")
    wl = bench.Workload(args.workload, seed=0x1B0002, dev=dev)
    engs = {}
    splits = args.splits.split(",") if args.splits else ["general" if args.general else "auto"]
    import ctypes
    for path in re.split("[,+]", args.libs):
        # builds of older revisions may carry an older ABI version; the A/B
        # only calls the RX entry points, which have not changed
        full = os.path.join(ROOT, path)
        v = ctypes.CDLL(full).ixg_abi_version()
        if v != ixgrx.ABI_VERSION:
            cur, ixgrx.ABI_VERSION = ixgrx.ABI_VERSION, v
            try:
                ixgrx.load_library(full)
            finally:
                ixgrx.ABI_VERSION = cur
        for sp in splits:
            name = os.path.basename(path) + ("" if len(splits) == 1 else ":" + sp)
            engs[name] = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=wl.flags),
                                        lib_path=os.path.join(ROOT, path), split=sp)
    s = torch.cuda.current_stream()
    # parity: every build's records equal the first build's, and each tiled
    # batch is self-consistent (the oracle checks the first build in tests/)
    ok, first = {}, None
    for v, e in engs.items():
        for _ in range(3):
            wl.launch(e, s.cuda_stream)
        torch.cuda.synchronize()
        tiled, rec = wl.snapshot()
        first = rec if first is None else first
        ok[v] = bool(tiled and np.array_equal(rec, first))
    times = {v: [] for v in engs}
    for _ in range(args.rounds):
        for v, e in engs.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.k)]
            for a, b in ev:
                a.record(s)
                wl.launch(e, s.cuda_stream)
                b.record(s)
            torch.cuda.synchronize()
            times[v] += [a.elapsed_time(b) for a, b in ev]
    res = {}
    for v, t in times.items():
        t = np.array(t)
        res[v] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                  "frac": round(wl.bytes_per_pkt * wl.n / (np.median(t) * 1e-3) / 8e12, 4), "parity": ok[v]}
    print(json.dumps({"workload": args.workload, "general_only": args.general, "results": res}))


if __name__ == "__main__":
    main()
