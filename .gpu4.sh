cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out &&
timeout -k 10 300 python -u tools/probe.py > gpurun_out/probe.json 2> gpurun_out/probe.err; echo probe rc=$?
P="python -u bench.py --workload c2 --secondary c3 --no-cpu --no-copy --steps 5 --warmup 1"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d gpurun_out/pmc$i -o p --output-format csv -- $P > gpurun_out/pmc$i.log 2>&1 || { echo "pmc$i failed"; break; }
  echo "pmc$i ok"
done
