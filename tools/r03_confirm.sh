# GPU suite + C3 / C4 / C5 / C2 bench lines at HEAD: bash tools/r03_confirm.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 300"
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
$T python3 bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
$T python3 bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>&1 || exit 1
$T python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 || exit 1
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
