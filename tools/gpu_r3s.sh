#!/bin/bash
# round 3: two chunks ahead in the coalesced kernel (a2) vs HEAD
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3s}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python3 -u tools/ab_lib.py --workload c2 --libs tools/ablib/a2.so,tools/ablib/head.so --rounds 10 > $O/ab_c2.json 2>$O/ab_c2.err
timeout -k 10 200 python3 -u tools/ab_lib.py --workload c2b --libs tools/ablib/a2.so,tools/ablib/head.so --rounds 6 > $O/ab_c2b.json 2>$O/ab_c2b.err
timeout -k 10 100 python3 -u tools/launch_times.py c2 60 0 > $O/lt_a2.json 2>$O/lt_a2.err
timeout -k 10 200 python3 -u tools/ab_demux.py --libs tools/ablib/a2.so,tools/ablib/head.so > $O/ab_demux.json 2>$O/ab_demux.err
echo ok
