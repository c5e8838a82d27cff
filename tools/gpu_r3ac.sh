#!/bin/bash
# round 3 final kernels: GPU suite, the default bench line on the driver's
# protocol, the same under rocprofv3 --kernel-trace --stats, SQ counters
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ac}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
bash tools/sq_counters.sh r3ac/sq "c2 c3 c5 c5r" > $O/sq.txt 2>&1
echo ok
