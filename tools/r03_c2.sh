# C2 latency check: bash tools/r03_c2.sh TAG  (GPU tests, C2 bench, kernel trace,
# VALU issue ceiling from one counter pass)
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2kt -o run --output-format csv -- python3 bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2_kt.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $O/issue4 -o run --output-format csv -- tools/ubench_issue 4 > $O/issue4.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $O/issue8 -o run --output-format csv -- tools/ubench_issue 8 > $O/issue8.log 2>&1 && \
timeout -k 10 60 tools/ubench_issue 4 >> $O/issue4.log 2>&1
rc=$?; tail -3 $O/pytest.log; echo rc=$rc; exit $rc
