#!/bin/bash
# tools/gpu.sh TAG STEP [STEP ...] - the one driver of GPU-box work (run it
# through gpurun from the repo root: gpurun -- 'bash tools/gpu.sh r4a tests bench').
# Every step runs under its own time limit, in order; the first failure ends
# the run (nothing more touches the GPU after a fault, an abort or a time
# limit). Output lands in gpurun_out/TAG/.
#
#   tests            the whole -m gpu suite              -> pytest.log
#   tests:FILE[:K]   one test file (-m gpu, optional -k K) -> pytest_<file>.log
#   smoke            __graft_entry__.smoke()             -> smoke.log
#   bench            bench.py at the driver's protocol (--steps 20 --warmup 5) -> bench.json
#   bench:A,B,...    bench.py with the arguments A B ... (commas for spaces)  -> bench_<i>.json
#   kt:W+W+...       per-kernel times of each workload's line (tools/kt_workloads.sh)
#   sq:W+W+...       SQ counter passes per workload (tools/sq_counters.sh)
#   mem:W+W+...      memory-pipe counter pass per workload (tools/mem_counters.sh)
#   profile          the round profile: kernel trace of the default bench, PMC traffic (tools/profile_round.sh)
#   ab:W:L1,L2,...   same-process A/B of library builds over workload W (tools/ab_lib.py; tools/build_variant.sh)
#   py:SCRIPT,A,...  python3 SCRIPT A ... (a probe or a one-off measurement) -> py_<i>.log
#   sqlib:W:LIB      SQ counter passes of one workload through a library build (tools/dbg/run_lib.py)
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
i=0
for STEP in "$@"; do
  i=$((i + 1))
  kind=${STEP%%:*}
  arg=""
  [ "$kind" != "$STEP" ] && arg=${STEP#*:}
  args=${arg//,/ }
  echo "== step $i: $STEP ($(date +%T))"
  case $kind in
    tests)
      if [ -z "$arg" ]; then
        timeout -k 10 600 $PYT tests -m gpu > "$O/pytest.log" 2>&1
      else
        f=${arg%%:*}; k=""; [ "$f" != "$arg" ] && k=${arg#*:}
        log="$O/pytest_$(basename "$f" .py).log"
        if [ -n "$k" ]; then timeout -k 10 400 $PYT "$f" -m gpu -k "$k" > "$log" 2>&1
        else timeout -k 10 400 $PYT "$f" -m gpu > "$log" 2>&1; fi
      fi ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench)
      if [ -z "$arg" ]; then timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
      else timeout -k 10 500 python3 bench.py $args > "$O/bench_$i.json" 2> "$O/bench_$i.log"; fi ;;
    kt) timeout -k 10 900 bash tools/kt_workloads.sh "$TAG/kt_$i" ${args//+/ } ;;
    sq) timeout -k 10 900 bash tools/sq_counters.sh "$TAG/sq_$i" "${args//+/ }" ;;
    mem) timeout -k 10 600 bash tools/mem_counters.sh "$TAG/mem_$i" "${args//+/ }" ;;
    profile) timeout -k 10 1000 bash tools/profile_round.sh "$TAG/profile" ;;
    ab) timeout -k 10 900 python3 -u tools/ab_lib.py --workload "${arg%%:*}" --libs "${arg#*:}" > "$O/ab_$i.json" 2> "$O/ab_$i.log" ;;
    py) timeout -k 10 600 python3 -u $args > "$O/py_$i.log" 2>&1 ;;
    sqlib)
      w=${arg%%:*}; lib=${arg#*:}; d="$O/sqlib_$i"; mkdir -p "$d"
      P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
      P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
      timeout -k 10 120 rocprofv3 --pmc $P1 --output-format csv -d "$d/${w}_p1" -o p -- python3 tools/dbg/run_lib.py "$lib" "$w" > "$d/p1.log" 2>&1 &&
      timeout -k 10 120 rocprofv3 --pmc $P2 --output-format csv -d "$d/${w}_p2" -o p -- python3 tools/dbg/run_lib.py "$lib" "$w" > "$d/p2.log" 2>&1 &&
      python3 tools/sq_report.py "$d" "$w" > "$O/sqlib_$i.txt" ;;
    pmclib)
      # pmclib:W:LIB:C1+C2+... one counter pass of one workload through a library build
      w=${arg%%:*}; r=${arg#*:}; lib=${r%%:*}; cs=${r#*:}; d="$O/pmclib_$i"; mkdir -p "$d"
      timeout -k 10 120 rocprofv3 --pmc ${cs//+/ } --output-format csv -d "$d/${w}_p1" -o p -- python3 tools/dbg/run_lib.py "$lib" "$w" > "$d/p1.log" 2>&1 &&
      python3 tools/sq_report.py "$d" "$w" > "$O/pmclib_$i.txt" ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "step $i ($STEP) failed: rc=$rc"
    for f in "$O"/*.log; do [ -f "$f" ] && { echo "--- $f"; tail -15 "$f"; }; done
    exit $rc
  fi
done
echo "all steps ok"
