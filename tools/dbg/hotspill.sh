#!/bin/bash
# Scratch (spill) instructions near the flat walk's row loads in the
# ixg_rx_glong_o kernel (diagnostic): tools/dbg/hotspill.sh [SRC]
SRC=${1:-/root/repo/ix_amd/csrc/ixgrx_kernels.hip}
D=$(mktemp -d)
cd "$D" || exit 1
timeout 600 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 --cuda-device-only -c "$SRC" -o k.o \
  --save-temps -Rpass-analysis=kernel-resource-usage > remarks.txt 2>&1
grep -A16 "Function Name: ixg_rx_glong_o" remarks.txt | grep -E "VGPRs Spill|Occupancy" | sed 's/^.*remark: //'
S=$(ls "$D"/*gfx950*.s 2>/dev/null | head -1)
[ -n "$S" ] || { echo "no asm"; grep error remarks.txt | head; exit 1; }
awk '/^ixg_rx_glong_o:/,/\.Lfunc_end.*ixg_rx_glong_o/' "$S" > g.s
F=$(grep -n "buffer_load_dwordx4.*offen" g.s | head -1 | cut -d: -f1)
L=$(grep -n "buffer_load_dwordx4.*offen" g.s | tail -1 | cut -d: -f1)
echo "row loads at lines $F..$L; scratch ops within [F-300, L+2500]:"
awk -v f="$F" -v l="$L" 'NR>f-300 && NR<l+2500 && /scratch_/ {print NR": "$0}' g.s
rm -rf "$D"
