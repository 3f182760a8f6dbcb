# fused-decode check + C2 bench + C4 batch sweep: bash tools/r03_run2.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "fused or auto_decode or poisoned or host" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 && \
bash tools/r03_c4sweep.sh $1
rc=$?; tail -3 $O/pytest.log; echo rc=$rc; exit $rc
