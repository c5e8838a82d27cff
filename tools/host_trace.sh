#!/bin/bash
# Kernel trace of the IX loop example (examples/ix_async_loop.c, the
# asynchronous host path): per-batch kernel durations in DIRECT mode (the
# kernels read pinned host memory), for DESIGN.md 4.7's host-link bound.
# usage (on the GPU box, from the repo root):
#   bash tools/host_trace.sh OUTDIR [KIND] [THREADS] [REGS] [BYTES]
#   KIND tcp64 (default) | tcp1514; THREADS e.g. "1 16"; REGS "0" | "0 1"
#   (zero copy); BYTES batch_bytes values, e.g. "1048576 524288"
set -e
O=${1:-gpurun_out/host_trace}
KIND=${2:-tcp64}
THREADS=${3:-1 16}
REGS=${4:-0}
BYTES=${5:-1048576}
mkdir -p "$O"
F="$O/frames.bin"
python3 - "$F" "$KIND" <<'PY'
import sys
sys.path.insert(0, ".")
import bench
from ix_amd import traces
n = 1 << 16 if sys.argv[2] == "tcp64" else 1 << 14
bench.write_frames_file(traces.make_trace(sys.argv[2], n, seed=0x1BF000), sys.argv[1])
PY
arena=$([ "$KIND" = tcp64 ] && echo 131072 || echo 32768)
for t in $THREADS; do
  for reg in $REGS; do
    for bb in $BYTES; do
      d="$O/t${t}_r${reg}_b$((bb >> 10))k"
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o kt -- \
        examples/bin/ix_async_loop "$F" loop threads=$t seconds=1 batch=64 arena=$arena register=$reg \
        cfg_bytes=$bb > "$d.json" 2> "$d.log"
      # keep the per-kernel statistics (the full trace runs to tens of MiB)
      find "$d" -name "*kernel_trace.csv" -delete
    done
  done
done
rm -f "$F"
