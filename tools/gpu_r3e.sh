#!/bin/bash
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3e}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_async.py tests/test_integration_example.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python3 -u -c "import json,bench; r,c=bench.host_path(seconds=2.0); print(json.dumps(r))" > $O/hostpath.json 2> $O/hostpath.err
echo ok
