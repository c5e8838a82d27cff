#!/bin/bash
# round 3: tcp_input-head ext kernel (tests + bench line), C2 kernel-trace stats as CSV
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3q}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_tcp_ext.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --extra "" --secondary "" --no-cpu --no-copy --no-strong --no-tx --no-bad > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --extra "" --secondary "" --no-cpu --no-copy --no-strong --no-demux --no-tx --no-bad > $O/bench_prof.json 2> $O/bench_prof.err
echo ok
