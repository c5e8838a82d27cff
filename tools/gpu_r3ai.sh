#!/bin/bash
# round 3: the memory ceiling of C5's span pattern: tools/probe_c3.hip's
# whole-span reads (1, 2, 4, 16, 64 chunks per wave step) on C5's and C3's
# buffers next to the product launch
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ai}; mkdir -p $O
for W in c5 c5r c3; do
  timeout -k 10 300 python3 -u tools/probe_c3.py $W > $O/probe_$W.json 2> $O/probe_$W.err
done
echo ok
