#!/bin/bash
# round 3: the N > 1 bench path rehearsed on one card (two gloo ranks on
# cuda:0): every line, oracle parity on rank 0 at N = 2
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3w}; mkdir -p $O
IXG_BENCH_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
timeout -k 10 600 python3 -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest_multi.log 2>&1
echo ok
