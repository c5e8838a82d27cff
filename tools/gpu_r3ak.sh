#!/bin/bash
# round 3: single-pass event records, tile size 16 / 32 / 64 chunks (kCW 4 /
# 8 / 16) against the four-launch HEAD build, same process
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ak}; mkdir -p $O
timeout -k 10 400 python3 -u tools/ab_ev.py tools/ablib/head.so,ix_amd/libixgrx.so,tools/ablib/evcw8.so,tools/ablib/evcw16.so,tools/ablib/evcw16ns.so 4 > $O/ab_ev.json 2> $O/ab_ev.err
echo ok
