cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log; tail -1 gpurun_out/pytest_gpu.log;
timeout -k 10 300 python -u tools/ab_fast.py --workload c2 --variants 0,1,2,3 --rounds 6 > gpurun_out/ab_c2.json 2> gpurun_out/ab_c2.err;
for w in c4 c3 c5; do timeout -k 10 300 python -u tools/ab_fast.py --workload $w --variants 0,g,g1,g2 --rounds 4 > gpurun_out/ab_$w.json 2> gpurun_out/ab_$w.err; done; echo done
