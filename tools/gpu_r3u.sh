#!/bin/bash
# round 3 checkpoint: the default bench line as the driver runs it, and the
# kernel trace of the same command (C2 kernel duration cross-check)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3u}; mkdir -p $O
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err
echo ok
