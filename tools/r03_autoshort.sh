# AUTO's short-row decode choice by code size per tile: GPU suite, then
# (16, 8) at 32000 / 64000 bytes and (64, 16, 32000), 16384 blocks each
set -o pipefail
O=gpurun_out/r03_autoshort_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
T="timeout -k 10 200"
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 > $O/k16_s32k_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 64000 --loss-rate 0.5 --blocks 16384 > $O/k16_s64k_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 64000 --loss-rate 0.5 --blocks 16384 --decode-kernel one_matrix > $O/k16_s64k_tc.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 64 --symbol-size 32000 --loss-rate 0.25 --blocks 16384 > $O/k64_s32k_l025_auto.log 2>&1 || exit 1
$T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 64 --symbol-size 32000 --loss-rate 0.25 --blocks 16384 --decode-kernel generated > $O/k64_s32k_l025_gen.log 2>&1 || exit 1
for f in $O/k*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
