#!/bin/bash
# round 3 re-entry: GPU suite, the default bench line as the driver runs it, kernel trace of the same
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3p}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kt -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --extra "" --no-cpu --no-copy --no-strong --no-demux --no-tx --no-bad > $O/bench_prof.json 2> $O/bench_prof.err
echo ok
