#!/bin/bash
# round 3: async host path, one stream per context vs one per batch (A/B by swapping the library)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3ae}; mkdir -p $O
cp ix_amd/libixgrx.so $O/keep.so
for L in as_multi as_one as_multi as_one; do
  cp tools/ablib/$L.so ix_amd/libixgrx.so
  timeout -k 10 200 python3 -u tools/hostpath_sweep4.py $L >> $O/sweep4.jsonl 2>> $O/sweep4.err
done
cp tools/ablib/as_one.so ix_amd/libixgrx.so
timeout -k 10 300 python3 -u -m pytest tests/test_async.py tests/test_integration_example.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_one.log 2>&1
cp $O/keep.so ix_amd/libixgrx.so && rm $O/keep.so
echo ok
