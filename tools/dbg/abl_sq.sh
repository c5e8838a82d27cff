#!/bin/bash
# tools/dbg/abl_sq.sh OUT W LIB... - one SQ counter pass (issue and VALU
# counters) per library build over workload W (tools/dbg/run_lib.py), and
# the per-chunk report (tools/sq_report.py). GPU box, from the repo root.
set -o pipefail
O=${1:?out}; W=${2:?workload}; shift 2
mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
for L in "$@"; do
  n=$(basename "$L" .so)
  timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d "$O/$n/${W}_p1" -o p -- python3 tools/dbg/run_lib.py "$L" "$W" > "$O/$n.log" 2>&1 || exit $?
  python3 tools/sq_report.py "$O/$n" "$W" > "$O/$n.txt" || exit $?
done
