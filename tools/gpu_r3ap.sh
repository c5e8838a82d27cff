#!/bin/bash
# round 3: event records, chunk runs of 2 per wave and 2x / 0.5x the
# resident grid, same-process A/B against the HEAD build
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ap}; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_ev.py tools/ablib/head.so,tools/ablib/evrun2.so,tools/ablib/evgrid2.so,tools/ablib/evgridh.so 5 > $O/ab_ev.json 2> $O/ab_ev.err
echo ok
