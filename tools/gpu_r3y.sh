#!/bin/bash
# round 3: C3 time breakdown by ablation (timing-only builds: no streaming
# rounds; no parse; 4 pieces per lane per round; fixed-shape parse only)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3y}; mkdir -p $O
timeout -k 10 300 python3 -u tools/ab_lib.py --workload c3 --libs tools/ablib/head.so,tools/ablib/norounds.so,tools/ablib/noparse.so,tools/ablib/kt4.so,tools/ablib/fixedonly.so --rounds 5 > $O/ab_c3.json 2>$O/ab_c3.err
timeout -k 10 300 python3 -u tools/ab_lib.py --workload c4 --libs tools/ablib/head.so,tools/ablib/norounds.so,tools/ablib/noparse.so,tools/ablib/kt4.so --rounds 4 > $O/ab_c4.json 2>$O/ab_c4.err
echo ok
