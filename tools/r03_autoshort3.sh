# Generated decode from 16 tiles for every layout: GPU suite, C1 geometry
# (16, 8, 64000) and (16, 8, 32000) AUTO, C4
set -o pipefail
O=gpurun_out/r03_autoshort3; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
T="timeout -k 10 200"
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 > $O/k16_s32k_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 64000 --loss-rate 0.5 --blocks 16384 > $O/k16_s64k_auto.log 2>&1 || exit 1
$T python3 bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
for f in $O/*.log; do case $f in *pytest*) continue;; esac; echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
