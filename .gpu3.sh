cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u tools/ab_fast.py --workload c2 > gpurun_out/ab_c2.json 2> gpurun_out/ab_c2.err && 
timeout -k 10 300 python -u tools/ab_fast.py --workload c3 --variants 0,g --rounds 4 > gpurun_out/ab_c3.json 2> gpurun_out/ab_c3.err &&
timeout -k 10 300 python -u tools/ab_fast.py --workload c5 --variants 0,g --rounds 4 > gpurun_out/ab_c5.json 2> gpurun_out/ab_c5.err; echo rc=$?
