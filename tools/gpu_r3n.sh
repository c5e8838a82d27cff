#!/bin/bash
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3n}; mkdir -p $O
timeout -k 10 200 python3 -u tools/ab_demux.py --libs ix_amd/libixgrx.so,tools/ablib/forcehit.so,tools/ablib/hot.so > $O/ab_demux.json 2>$O/ab.err
echo ok
