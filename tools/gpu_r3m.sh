#!/bin/bash
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3m}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "demux or dmx or fdir" > $O/pytest.log 2>&1
timeout -k 10 200 python3 -u tools/ab_demux.py --libs ix_amd/libixgrx.so,tools/ablib/coop.so > $O/ab_demux.json 2>$O/ab.err
timeout -k 10 200 python3 -u tools/ab_demux.py --separate --libs ix_amd/libixgrx.so,tools/ablib/coop.so > $O/ab_demux_sep.json 2>>$O/ab.err
echo ok
