#!/bin/bash
# round 3: FDIR header as a scalar load (no vmcnt(0) mid-chunk) + branch-free
# fixed-shape checks: GPU suite, same-process A/B vs HEAD, fresh-process
# launch curves, SQ counters
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3r}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for W in c2 c3 c5 c5r c4; do
  timeout -k 10 200 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/new.so,tools/ablib/base.so --rounds 6 > $O/ab_$W.json 2>$O/ab_$W.err
done
timeout -k 10 100 python3 -u tools/launch_times.py c2 60 0 > $O/lt_new.json 2>$O/lt_new.err
cp ix_amd/libixgrx.so $O/keep.so && cp tools/ablib/base.so ix_amd/libixgrx.so
timeout -k 10 100 python3 -u tools/launch_times.py c2 60 0 > $O/lt_base.json 2>$O/lt_base.err
cp $O/keep.so ix_amd/libixgrx.so && rm $O/keep.so
bash tools/sq_counters.sh r3r/sq "c2 c3 c5" > $O/sq.txt 2>&1
echo ok
