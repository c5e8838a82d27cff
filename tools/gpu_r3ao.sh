#!/bin/bash
# round 3: the separate demux pass with non-temporal record / header loads,
# same-process A/B against the HEAD build, then the demux tests with it
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ao}; mkdir -p $O
timeout -k 10 300 python3 -u tools/ab_demux.py --libs tools/ablib/head.so,tools/ablib/dmxnt.so --separate --rounds 8 > $O/ab_sep.json 2> $O/ab_sep.err
echo ok
