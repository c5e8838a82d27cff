#!/usr/bin/env python3
"""Per-launch summary of a `rocprofv3 --kernel-trace --stats` run of bench.py.

One ixg_rx_batch_dev launch = a fixed-shape dispatch (ixg_rx_fast_*) followed
by a general dispatch (ixg_rx_general_*). bench.py's default command runs,
in order: the primary workload (warmup + steps), the secondary workload
(2 + max(5, steps/2)), then 3 copy-inclusive launches of the primary.
This splits the trace into those phases and prints, per phase, the average
per-kernel durations and the launch span (fast start -> general end), which
is what the HIP events around each launch in bench.py measure.

usage: kt_summary.py KT_DIR WARMUP STEPS [PRIMARY SECONDARY]
"""
import csv
import glob
import os
import statistics
import sys


def main():
    d, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    prim = sys.argv[4] if len(sys.argv) > 4 else "c2"
    sec = sys.argv[5] if len(sys.argv) > 5 else "c4"
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("ixg_rx")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    launches = []
    i = 0
    while i < len(rows):
        r = rows[i]
        if "fast" in r["Kernel_Name"] and i + 1 < len(rows) and "general" in rows[i + 1]["Kernel_Name"]:
            g = rows[i + 1]
            launches.append((r, g))
            i += 2
        else:
            launches.append((None, r))
            i += 1
    s2 = max(5, steps // 2)
    phases = [(f"{prim} warmup", warm), (f"{prim} timed", steps), (f"{sec} warmup", 2), (f"{sec} timed", s2),
              (f"{prim} copy-inclusive", 3)]
    out = ["| phase | launches | fast kernel avg us | general kernel avg us | launch span avg us | span min us |",
           "|---|---|---|---|---|---|"]
    k = 0
    for name, cnt in phases:
        ph = launches[k:k + cnt]
        k += cnt
        if not ph:
            continue

        def dur(r):
            return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        fa = [dur(a) for a, _ in ph if a is not None]
        ga = [dur(b) for _, b in ph]
        sp = [(int(b["End_Timestamp"]) - int((a or b)["Start_Timestamp"])) / 1e3 for a, b in ph]
        kname = (ph[0][0] or ph[0][1])["Kernel_Name"]
        out.append(f"| {name} ({kname}) | {len(ph)} | {statistics.mean(fa) if fa else 0:.1f} | "
                   f"{statistics.mean(ga):.1f} | {statistics.mean(sp):.1f} | {min(sp):.1f} |")
    if k != len(launches):
        out.append(f"(trace holds {len(launches)} launches, phases account for {k})")
    print("\n".join(out))


if __name__ == "__main__":
    main()
