#!/usr/bin/env python3
"""Interleaved A/B of kernel builds in ONE process (guide rule 24).

Creates one engine per IXGRX_FAST_VARIANT (plus the general-only path),
runs R rounds x K launches each, round-robin over the variants, and prints
median/min per-launch milliseconds per variant (events around each launch).
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
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--variants", default="0,1,2,3,g")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--lib", default="tools/ablib/ab.so", help="an A/B build (make -C ix_amd/csrc AB=1 OUT=...)")
    args = ap.parse_args()
    import torch
    import bench
    from ix_amd import ixgrx, traces
    dev = torch.device("cuda:0")
    wl = bench.Workload(args.workload, seed=0x1B0002, dev=dev, n=args.n)
    engs = {}
    for v in args.variants.split(","):
        # "3" = fast variant 3; "0:1" = fast variant 0 + general variant 1;
        # "0:0:2" = + short variant 2; "g1" = general-only with general variant 1
        # (variants exist only in an A/B build: make -C ix_amd/csrc AB=1 OUT=...)
        parts = (["0", v[1:] or "0"] if v.startswith("g") else v.split(":")) + ["0", "0"]
        os.environ["IXGRX_FAST_VARIANT"] = parts[0] or "0"
        os.environ["IXGRX_GEN_VARIANT"] = parts[1] or "0"
        os.environ["IXGRX_SHORT_VARIANT"] = parts[2] or "0"
        engs[v] = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY, flags=wl.flags), lib_path=os.path.join(ROOT, args.lib),
                                 split="general" if v.startswith("g") else "auto")
    s = torch.cuda.current_stream()
    times = {v: [] for v in engs}
    # parity: every variant's records equal the first variant's, and each
    # tiled batch is self-consistent (the oracle checks the kernels in tests/)
    ok, first = {}, None
    for v, e in engs.items():  # warm + parity
        for _ in range(3):
            wl.launch(e, s.cuda_stream)
        torch.cuda.synchronize()
        tiled, rec = wl.snapshot()
        first = rec if first is None else first
        ok[v] = bool(tiled and np.array_equal(rec, first))
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
                  "gpkt_s": round(wl.n / np.median(t) / 1e6, 2),
                  "frac": round(wl.bytes_per_pkt * wl.n / (np.median(t) * 1e-3) / 8e12, 4), "parity": ok[v]}
    print(json.dumps({"workload": args.workload, "n": wl.n, "results": res}))


if __name__ == "__main__":
    main()
