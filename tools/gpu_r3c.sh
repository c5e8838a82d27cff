#!/bin/bash
# round 3: GPU suite, then the default bench line the way the driver runs it
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3c}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo ok
