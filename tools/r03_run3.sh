# emission + tiles-per-WG check: bash tools/r03_run3.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 300"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
$T python3 bench.py --config c4 --decode-kernel generated --warmup 1 --no-cpu-baseline > $O/c4_gen.log 2>&1 && \
$T python3 bench.py --config c4 --decode-kernel one_matrix --warmup 1 --no-cpu-baseline > $O/c4_tc.log 2>&1 && \
$T python3 bench.py --steps 10 --no-cpu-baseline > $O/c3.log 2>&1 && \
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5.log 2>&1
rc=$?
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
tail -2 $O/pytest.log; exit $rc
