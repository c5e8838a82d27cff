#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of bench.py's primary
# line for each workload given: tools/kt_workloads.sh TAG W1 W2 ... (on the
# GPU box via gpurun). Prints "workload kernel calls avg_us" rows.
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for W in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$W" -o kt -- python3 bench.py \
    --workload "$W" --secondary "" --extra "" --no-cpu --no-copy --no-demux --no-tx --no-bad --no-strong --steps 10 --warmup 2 \
    > "$O/$W.json" 2> "$O/$W.log" || { echo "kt $W failed"; tail -20 "$O/$W.log"; exit 1; }
  rm -f "$O/$W"/*kernel_trace.csv
  python3 - "$O/$W/kt_kernel_stats.csv" "$W" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith("ixg_"):
        print(sys.argv[2], r["Name"], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
