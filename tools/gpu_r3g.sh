#!/bin/bash
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3g}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 250 python3 -u tools/hostpath_sweep2.py tcp64 > $O/sweep_tcp64.jsonl 2>$O/sweep.err
timeout -k 10 250 python3 -u tools/hostpath_sweep2.py imix > $O/sweep_imix.jsonl 2>>$O/sweep.err
echo ok
