#!/bin/bash
# round 3: the long kernel's first streaming round issued before the parse
# (list built from the frame lengths) + the pipelined event emit: GPU suite,
# same-process A/Bs
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3z}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c3 c4 c5; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/c3pre.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
timeout -k 10 250 python3 -u tools/ab_ev.py tools/ablib/evhead.so,tools/ablib/evpipe.so 4 > $O/ab_ev.json 2>$O/ab_ev.err
timeout -k 10 200 python3 -u tools/ab_demux.py --libs tools/ablib/head.so,tools/ablib/c3pre.so > $O/ab_demux.json 2>$O/ab_demux.err
echo ok
