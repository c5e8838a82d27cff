cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ;
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log;
timeout -k 10 400 python -u bench.py --cpu-seconds 6 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?";
IXGRX_FORCE_GENERAL=1 timeout -k 10 400 python -u bench.py --no-cpu --no-copy > gpurun_out/bench_general.json 2> gpurun_out/bench_general.err; echo "bench-gen rc=$?";
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o kt --output-format csv -- python -u bench.py --no-cpu --no-copy > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err; echo "prof rc=$?";
rocprofv3 -L > gpurun_out/counters.txt 2>&1; echo done
