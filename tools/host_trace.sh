#!/bin/bash
# Kernel trace of the IX loop example (examples/ix_async_loop.c, the
# asynchronous host path) at 1 and 16 threads over C2's frames: per-batch
# kernel durations in DIRECT mode (the kernels read pinned host memory), for
# DESIGN.md 4.7's host-link bound.
# usage (on the GPU box, from the repo root): bash tools/host_trace.sh OUTDIR
set -e
O=${1:-gpurun_out/host_trace}
mkdir -p "$O"
F="$O/frames.bin"
python3 - "$F" <<'EOF'
import sys
sys.path.insert(0, ".")
import bench
from ix_amd import traces
bench.write_frames_file(traces.make_trace("tcp64", 1 << 16, seed=0x1BF000), sys.argv[1])
EOF
for t in 1 16; do
  for reg in 0; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/t$t" -o kt -- \
      examples/bin/ix_async_loop "$F" loop threads=$t seconds=1 batch=64 arena=131072 register=$reg \
      > "$O/t$t.json" 2> "$O/t$t.log"
  done
done
rm -f "$F"
