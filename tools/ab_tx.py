#!/usr/bin/env python3
"""Interleaved A/B of library builds on the TX kernel (same process):
ab_tx.py --libs ix_amd/libixgrx.so,tools/ablib/base.so --kind tcp64 --n N"""
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
    ap.add_argument("--kind", default="tcp64")
    ap.add_argument("--n", type=int, default=16 * 1024 * 1024)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--k", type=int, default=10)
    args = ap.parse_args()
    import torch
    from ix_amd import ixgrx, traces, tx
    dev = torch.device("cuda:0")
    b = tx.make_segments(args.kind, args.n, seed=5, pool=1 << 16, layout="packed")
    buf = torch.from_numpy(b.buf).to(dev)
    segs = torch.from_numpy(b.segs.view(np.uint8)).to(dev)
    outs, lens, engs = {}, {}, {}
    for path in args.libs.split(","):
        e = ixgrx.RxEngine(ixgrx.Config(traces.RSS_KEY), lib_path=os.path.join(ROOT, path))
        tx.set_macs(e, b.src_mac, b.dmacs)
        engs[path] = e
        outs[path] = torch.zeros(b.out_size, dtype=torch.uint8, device=dev)
        lens[path] = torch.zeros(args.n, dtype=torch.int16, device=dev)
    s = torch.cuda.current_stream()
    times = {p: [] for p in engs}
    for _ in range(args.rounds):
        for p, e in engs.items():
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.k)]
            for a, c in ev:
                a.record(s)
                tx.batch_dev(e, buf.data_ptr(), segs.data_ptr(), args.n, outs[p].data_ptr(), lens[p].data_ptr(), 0,
                             s.cuda_stream)
                c.record(s)
            torch.cuda.synchronize()
            times[p] += [a.elapsed_time(c) for a, c in ev]
    first = next(iter(engs))
    L = b.segs["seg_len"].astype(np.float64)
    alg = float((40 + L + 34 + L + np.where(b.segs["proto"] == 17, 8, 0) + 2).mean())
    res = {}
    for p in engs:
        t = float(np.median(times[p]))
        res[os.path.basename(p)] = {"median_ms": round(t, 4), "frac": round(alg * args.n / (t * 1e-3) / 8e12, 4),
                                    "same_as_first": bool(torch.equal(outs[p], outs[first]) and
                                                          torch.equal(lens[p], lens[first]))}
    print(json.dumps({"kind": args.kind, "n": args.n, "results": res}))


if __name__ == "__main__":
    main()
