cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1;
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 ;
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log;
timeout -k 10 600 python -u bench.py --cpu-seconds 6 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"
