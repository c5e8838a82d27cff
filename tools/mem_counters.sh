#!/bin/bash
# Memory-pipe counter pass (TA/TD/TCP + GRBM) for bench workloads on the GPU
# box: tools/mem_counters.sh TAG "c5 c2"  -> per-chunk values per kernel
TAG=$1; WLS=$2
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
for W in $WLS; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$O/${W}_p1" -o p -- python3 bench.py --workload $W \
    --secondary "" --extra "" --no-cpu --no-copy --no-demux --no-tx --no-bad --steps 3 --warmup 1 > "$O/${W}_p1.json" 2> "$O/${W}_p1.log" \
    || { echo "pass $W failed"; tail -20 "$O/${W}_p1.log"; exit 1; }
done
python3 tools/sq_report.py "$O" $WLS
