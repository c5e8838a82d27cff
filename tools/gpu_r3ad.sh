#!/bin/bash
# round 3: host path depth x batch sweep (DIRECT, staged) at 1/4/8/16 threads
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ad}; mkdir -p $O
timeout -k 10 400 python3 -u tools/hostpath_sweep3.py > $O/sweep3.jsonl 2> $O/sweep3.err
echo ok
