#!/bin/bash
# round 3: single-pass event records (decoupled look-back over 1024-frame
# tiles): the event tests first (bounded), then the GPU suite, then the
# same-process A/B of the events line against the HEAD build
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3aj}; mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_events.py -m gpu -x -v --timeout 60 --timeout-method thread > $O/pytest_ev.log 2>&1
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u tools/ab_ev.py tools/ablib/head.so,ix_amd/libixgrx.so 5 > $O/ab_ev.json 2> $O/ab_ev.err
echo ok
