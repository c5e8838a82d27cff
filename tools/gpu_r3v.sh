#!/bin/bash
# round 3: the span kernel's parse pool (frames dropped on the Ethernet type
# never take a parse lane; pools parsed full): parity + A/B of pool thresholds
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3v}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_tcp_ext.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c5r c5 c3; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/pool40.so,tools/ablib/pool48.so,tools/ablib/pool56.so --rounds 5 > $O/ab_$W.json 2>$O/ab_$W.err
done
echo ok
