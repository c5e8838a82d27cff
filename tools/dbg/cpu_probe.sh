#!/bin/bash
# tools/dbg/cpu_probe.sh OUTDIR [THREADS ...] - where the host path's 16-thread
# tail latency comes from: the box's CPU share (cgroup cpu.max, affinity) and
# the cgroup's throttling counters (cpu.stat) around each ix_async_loop run.
# Run through gpurun from the repo root; each loop run has its own limit.
set -o pipefail
O=${1:?outdir}; shift
mkdir -p "$O"
T=${*:-16}
{
  echo "nproc: $(nproc)"
  grep -E 'Cpus_allowed_list' /proc/self/status
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.weight /sys/fs/cgroup/cpuset.cpus.effective; do
    [ -r "$f" ] && echo "$f: $(cat $f)"
  done
  cat /proc/sys/kernel/sched_min_granularity_ns 2>/dev/null
  grep -m1 'model name' /proc/cpuinfo
} > "$O/box.txt" 2>&1
python3 -c "
import sys; sys.path.insert(0, '.')
import bench
from ix_amd import traces
bench.write_frames_file(traces.make_trace('tcp64', 1 << 16, seed=0x1BF000), '$O/frames.bin')
" || exit 1
for t in $T; do
  cat /sys/fs/cgroup/cpu.stat > "$O/cpustat_before_t$t.txt" 2>/dev/null
  timeout -k 10 60 examples/bin/ix_async_loop "$O/frames.bin" loop threads=$t seconds=3 batch=64 arena=131072 \
    > "$O/loop_t$t.json" 2> "$O/loop_t$t.log" || exit $?
  cat /sys/fs/cgroup/cpu.stat > "$O/cpustat_after_t$t.txt" 2>/dev/null
done
rm -f "$O/frames.bin"
echo ok
