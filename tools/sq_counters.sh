#!/bin/bash
# SQ counter passes for the RX kernels (run on the GPU box via gpurun):
#   tools/sq_counters.sh TAG "c3 c4 c5" [extra bench args]
# Two --pmc passes per workload (kernel dispatches only, no other tracing).
TAG=$1; WLS=$2; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
for W in $WLS; do
  for k in 1 2; do
    [ $k = 1 ] && C=$P1 || C=$P2
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$O/${W}_p$k" -o p -- python3 bench.py --workload $W \
      --secondary "" --extra "" --no-cpu --no-copy --no-demux --no-tx --no-bad --no-strong --steps 3 --warmup 1 "$@" > "$O/${W}_p$k.json" 2> "$O/${W}_p$k.log" \
      || { echo "pass $k $W failed"; tail -20 "$O/${W}_p$k.log"; exit 1; }
  done
done
python3 tools/sq_report.py "$O" $WLS
