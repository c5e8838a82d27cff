#!/bin/bash
# round 3: HEAD check after the events experiment: the event tests (incl. the
# back-to-back launches), the GPU suite and smoke()
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3am}; mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_events.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_ev.log 2>&1
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo ok
