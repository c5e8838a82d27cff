#!/bin/bash
# round 3: C3/C4 long-kernel prefix prefetch variants after the FDIR scalar-load fix
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3t}; mkdir -p $O
for W in c3 c4 c5; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/c3late.so,tools/ablib/c3early.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
echo ok
