#!/bin/bash
# round 3 final check: the GPU suite, smoke(), and bench.py with no flags (the
# default run) timed end to end
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ag}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
start=$(date +%s)
timeout -k 10 900 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "default bench seconds: $(( $(date +%s) - start ))" > $O/bench_default.time
echo ok
