#!/bin/bash
# Counter passes for the fused demux kernel against the plain RX kernel on
# the same C2 frames (run on the GPU box via gpurun):
#   tools/dmx_counters.sh TAG
# One --pmc pass per counter group, kernel dispatches only.
TAG=$1
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
P4="TCC_HIT_sum TCC_MISS_sum"
P5="FETCH_SIZE"
k=0
for C in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  k=$((k+1))
  for M in fused plain; do
    A=""; [ $M = plain ] && A="--plain"
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$O/c2_p${k}_$M" -o p -- python3 tools/ab_demux.py \
      --libs ix_amd/libixgrx.so --rounds 1 --k 2 $A > "$O/p${k}_$M.json" 2> "$O/p${k}_$M.log" \
      || { echo "pass $k $M failed"; tail -20 "$O/p${k}_$M.log"; exit 1; }
  done
done
python3 tools/sq_report.py "$O" c2
