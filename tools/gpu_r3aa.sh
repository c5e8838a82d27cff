#!/bin/bash
# round 3: the long walk's transposed prefix load (gen_pre_t), with and
# without the first round issued before the parse: GPU suite (product = tp),
# same-process A/Bs on C3 / C4 / C5 and the fused demux
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3aa}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c3 c4 c5; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/tp.so,tools/ablib/tpnopre.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
echo ok
