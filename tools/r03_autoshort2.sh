# AUTO short-row choice at a 6 KB-per-tile code threshold: the decode GPU
# tests, then (64, 16) and (128, 16) at 32000 bytes, AUTO against the other
# kernel, 16384 / 8192 blocks
set -o pipefail
O=gpurun_out/r03_autoshort2; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/pytest_decode.log 2>&1 || { tail -30 $O/pytest_decode.log; exit 1; }
tail -1 $O/pytest_decode.log
T="timeout -k 10 200"
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 64 --symbol-size 32000 --loss-rate 0.25 --blocks 16384 > $O/k64_e16_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 128 --symbol-size 32000 --loss-rate 0.125 --blocks 8192 > $O/k128_e16_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 128 --symbol-size 32000 --loss-rate 0.125 --blocks 8192 --decode-kernel generated > $O/k128_e16_gen.log 2>&1 || exit 1
for f in $O/k*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
