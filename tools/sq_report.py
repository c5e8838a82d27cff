#!/usr/bin/env python3
"""Per-kernel SQ counters normalised per 64-frame chunk (tools/sq_counters.sh output).
Cycle counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_*, SQ_BUSY_CYCLES) are in quad-cycles on gfx950."""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    d = sys.argv[1]
    import bench
    for w in sys.argv[2:]:
        nchunks = bench.WORKLOADS[w][1] / 64
        vals = {}
        for f in glob.glob(os.path.join(d, f"{w}_p*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].startswith("ixg_rx"):
                    vals.setdefault((r["Kernel_Name"], r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        kerns = sorted({k for k, _ in vals})
        print(f"== {w} ({int(nchunks)} chunks)")
        for k in kerns:
            row = {c: statistics.median(v) for (kk, c), v in vals.items() if kk == k}
            per = {c: round(v / nchunks, 1) for c, v in row.items() if c != "SQ_BUSY_CYCLES"}
            print(f"  {k}: per chunk {json.dumps(per)}")


if __name__ == "__main__":
    main()
