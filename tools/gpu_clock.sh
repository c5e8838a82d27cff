#!/bin/bash
# launch-settling diagnosis: per-launch clocks in fresh processes
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/clk
mkdir -p $O
rocm-smi --showclocks > $O/smi_before.txt 2>&1 || true
timeout -k 10 150 python3 -u tools/clock_trace.py plain 80 $O/plain.json > $O/plain.log 2>&1
timeout -k 10 150 python3 -u tools/clock_trace.py c2 80 $O/c2.json > $O/c2.log 2>&1
timeout -k 10 150 python3 -u tools/clock_trace.py idle 80 $O/idle.json > $O/idle.log 2>&1
timeout -k 10 150 python3 -u tools/clock_trace.py plain 80 $O/plain2.json > $O/plain2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace -d $O/grbm -o run -- python3 tools/launch_times.py c2 60 0 > $O/grbm.log 2>&1
rocprofv3 -L > $O/counters.txt 2>&1 || true
rocm-smi --showclocks > $O/smi_after.txt 2>&1 || true
echo done
