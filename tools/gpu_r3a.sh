set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r3a}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python3 -u tools/ab_lib.py --workload c2 --libs ix_amd/libixgrx.so,tools/ablib/base.so --rounds 10 > $O/ab_c2.json 2>$O/ab_c2.err
timeout -k 10 200 python3 -u tools/ab_lib.py --workload c2b --libs ix_amd/libixgrx.so,tools/ablib/base.so --rounds 6 > $O/ab_c2b.json 2>$O/ab_c2b.err
timeout -k 10 150 python3 -u tools/clock_trace.py c2 80 $O/clk_c2.json > $O/clk.log 2>&1
timeout -k 10 150 python3 -u tools/clock_trace.py plain 80 $O/clk_plain.json > $O/clk2.log 2>&1
echo ok
