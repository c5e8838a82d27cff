#!/bin/bash
# round 3: the big-chunk kernel (C4's chunks at 4 waves/SIMD): GPU suite,
# same-process A/Bs on C4 / C3 / C5 and the one-batch C4 line
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3af}; mkdir -p $O
timeout -k 10 450 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c4 c3 c5; do
  timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/tpnopre.so,tools/ablib/big.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
timeout -k 10 300 python3 -u bench.py --workload c4 --secondary "" --extra "" --no-cpu --no-copy --no-demux --no-tx --steps 20 --warmup 20 > $O/bench_c4.json 2> $O/bench_c4.err
echo ok
