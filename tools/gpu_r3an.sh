#!/bin/bash
# round 3: the span kernel over chunk pairs (13-KiB copies, 8 waves per CU):
# the RX GPU tests, then same-process A/Bs against the HEAD build
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3an}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_tcp_ext.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_rx.log 2>&1
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c5 c5r c2o c3; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,ix_amd/libixgrx.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
echo ok
