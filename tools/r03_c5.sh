# C5 / C3 lines with AUTO's encode choice, GPU suite: bash tools/r03_c5.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
T="timeout -k 10 200"
for rep in 1 2; do
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5_$rep.log 2>&1 || exit 1
done
$T python3 bench.py --steps 5 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
tail -1 $O/pytest_gpu.log
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
