# GPU suite of this round: bash tools/r03_tests.sh TAG
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; echo rc=$rc; exit $rc
