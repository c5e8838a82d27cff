#!/bin/bash
# round 3: (1) round 2's flat long kernel re-measured without the prefetch
# stall (A/B build of 494ea39^ with the scalar FDIR header, IXGRX_FLAT=1)
# against the product; (2) the N > 1 bench path on one card (gloo)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3x}; mkdir -p $O
for W in c3 c4; do
  IXGRX_FLAT=1 timeout -k 10 250 python3 -u tools/ab_lib.py --workload $W --libs tools/ablib/head.so,tools/ablib/flat.so --rounds 6 > $O/ab_flat_$W.json 2>$O/ab_flat_$W.err
done
timeout -k 10 250 python3 -u tools/ab_lib.py --workload c3 --libs tools/ablib/head.so,tools/ablib/flat.so --rounds 6 > $O/ab_noflat_c3.json 2>$O/ab_noflat_c3.err
OUTDIR=r3x bash tools/gpu_r3w.sh
