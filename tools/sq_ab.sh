#!/bin/bash
# SQ counter passes over an A/B library's variants (run on the GPU box via
# gpurun): tools/sq_ab.sh TAG WORKLOAD VARIANTS [lib]
# Kernel names differ per variant, so tools/sq_report.py separates them.
TAG=$1; W=$2; V=$3; LIB=${4:-tools/ablib/ab.so}
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
for k in 1 2; do
  [ $k = 1 ] && C=$P1 || C=$P2
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$O/${W}_p$k" -o p -- python3 tools/ab_fast.py \
    --workload $W --variants "$V" --rounds 1 --k 3 --lib "$LIB" > "$O/${W}_p$k.json" 2> "$O/${W}_p$k.log" \
    || { echo "pass $k failed"; tail -20 "$O/${W}_p$k.log"; exit 1; }
done
python3 tools/sq_report.py "$O" $W
