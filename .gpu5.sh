cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python -u tools/probe.py > gpurun_out/probe2.json 2> gpurun_out/probe2.err; echo rc=$?
