#!/bin/bash
# round 3: single-pass event records with the records re-read for the
# emission (8 waves/SIMD, one chunk ahead), tiles of 64 / 128 / 256 chunks,
# against the four-launch HEAD build and the register-held 64-chunk tiles
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3al}; mkdir -p $O
timeout -k 10 200 python3 -u -m pytest tests/test_events.py -m gpu -x -q --timeout 60 --timeout-method thread > $O/pytest_ev.log 2>&1
timeout -k 10 400 python3 -u tools/ab_ev.py tools/ablib/head.so,tools/ablib/evcw16.so,ix_amd/libixgrx.so,tools/ablib/evre32.so,tools/ablib/evre64.so 4 > $O/ab_ev.json 2> $O/ab_ev.err
echo ok
