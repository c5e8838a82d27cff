#!/bin/bash
# round 3 closing check on a fresh box, as the driver runs it: the GPU suite,
# smoke(), and bench.py on the driver's protocol (W = 5, K = 20)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3aq}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_w5k20.json 2> $O/bench_w5k20.err
echo ok
