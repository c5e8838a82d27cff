cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log; tail -1 gpurun_out/pytest_gpu.log;
timeout -k 10 300 python -u tools/ab_fast.py --workload c4 --variants 0,g,g1 --rounds 4 > gpurun_out/ab_c4.json 2> gpurun_out/ab_c4.err;
timeout -k 10 300 python -u tools/ab_fast.py --workload c3 --variants 0,g,g1 --rounds 4 > gpurun_out/ab_c3.json 2> gpurun_out/ab_c3.err;
timeout -k 10 300 python -u tools/ab_fast.py --workload c5 --variants 0,g,g1 --rounds 4 > gpurun_out/ab_c5.json 2> gpurun_out/ab_c5.err;
timeout -k 10 300 python -u tools/ab_fast.py --workload c2 --variants 0,g --rounds 4 > gpurun_out/ab_c2.json 2> gpurun_out/ab_c2.err; echo done
