#!/bin/bash
# round 3: the long walk's transposed prefix issued a chunk ahead into LDS
# (global_load_lds, pre_t_issue) vs synchronous (tpnopre) vs HEAD
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ab}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c3 c4 c5; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/tpnopre.so,tools/ablib/tpa.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
timeout -k 10 200 python3 -u tools/ab_demux.py --libs tools/ablib/head.so,tools/ablib/tpa.so > $O/ab_demux.json 2>$O/ab_demux.err
echo ok
