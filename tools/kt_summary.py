#!/usr/bin/env python3
"""Per-launch summary of a `rocprofv3 --kernel-trace --stats` run of bench.py.

One RX launch (ixg_rx_batch_dev / ixg_rx_demux_batch_dev) is a short
sequence of dispatches on one stream: the coalesced fixed-shape kernel
alone (C2's shape); or the self-sampling short kernel (ixg_rx_short_*) +
the long kernel (ixg_rx_general_*); or, in forced splits, [ixg_rx_sample] +
a fixed-shape kernel (ixg_rx_fast*) + the short kernel + the long kernel.
Kernels of a class with nothing to do exit at once. The
demux, TX and event kernels are launches of their own. This groups the trace
into launches, then into runs of consecutive launches with the same kernel
sequence (bench.py's phases), and prints per run the launch count, the mean
and min launch span (first dispatch start -> last dispatch end: what the HIP
events around a launch measure) and the mean duration of each kernel.

The last phase of bench.py (the overlapped copy-inclusive leg) runs two
streams, so its launches interleave and show up as short mixed runs.

usage: kt_summary.py KT_DIR
"""
import csv
import glob
import os
import statistics
import sys


def launches(rows):
    out, cur = [], []
    for r in rows:
        n = r["Kernel_Name"]
        if n.startswith("ixg_rx"):
            after_sampler = len(cur) == 1 and cur[0]["Kernel_Name"] == "ixg_rx_sample"
            # the self-sampling short kernel opens a launch of its own
            # (default plan for offset / wide-stride batches)
            self_first = n.startswith("ixg_rx_short") and cur and \
                not cur[-1]["Kernel_Name"].startswith(("ixg_rx_sample", "ixg_rx_fast"))
            if cur and (n == "ixg_rx_sample" or (n.startswith("ixg_rx_fast") and not after_sampler) or self_first):
                out.append(cur)
                cur = []
            cur.append(r)
            # the long kernel ends a launch, and so does the coalesced
            # fixed-shape kernel in the default plan
            if n.startswith("ixg_rx_general") or n.startswith("ixg_rx_fastc"):
                out.append(cur)
                cur = []
        else:
            if cur:
                out.append(cur)
                cur = []
            out.append([r])
    if cur:
        out.append(cur)
    return out


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("ixg_")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    L = launches(rows)
    runs = []
    for ln in L:
        key = tuple(r["Kernel_Name"] for r in ln)
        if runs and runs[-1][0] == key:
            runs[-1][1].append(ln)
        else:
            runs.append((key, [ln]))

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = ["| # | kernel sequence of a launch | launches | span mean us | span min us | per-kernel mean us |",
           "|---|---|---|---|---|---|"]
    for i, (key, lns) in enumerate(runs):
        sp = [(int(ln[-1]["End_Timestamp"]) - int(ln[0]["Start_Timestamp"])) / 1e3 for ln in lns]
        per = [statistics.mean(dur(ln[k]) for ln in lns) for k in range(len(key))]
        out.append(f"| {i} | {' + '.join(key)} | {len(lns)} | {statistics.mean(sp):.1f} | {min(sp):.1f} | "
                   f"{', '.join(f'{p:.1f}' for p in per)} |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
