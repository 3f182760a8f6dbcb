# generated encode in the two-wave layout for 16 < e <= 32 (HEAD) vs the
# 8-row layout with covers (tools/ab/librsgpu_base.so) vs the compiled
# kernel: GPU suite, C5, C3, (100, 25), (128, 32): bash tools/r03_wenc.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
T="timeout -k 10 200"
B="python3 tools/ab_lib.py tools/ab/librsgpu_base.so"
for rep in 1 2; do
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5_auto_$rep.log 2>&1 || exit 1
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c5_wide_$rep.log 2>&1 || exit 1
$T $B --config c5 --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c5_gen8_$rep.log 2>&1 || exit 1
done
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c3_wide.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline > $O/c3_auto.log 2>&1 || exit 1
for g in "100 0.25 635" "128 0.25 497"; do set -- $g
$T python3 bench.py --steps 4 --no-cpu-baseline --symbols $1 --loss-rate $2 --blocks $3 > $O/k$1_wide.log 2>&1 || exit 1
$T $B --steps 4 --no-cpu-baseline --symbols $1 --loss-rate $2 --blocks $3 > $O/k$1_gen8.log 2>&1 || exit 1
done
tail -1 $O/pytest_gpu.log
for f in $O/*.log; do [ $f = $O/pytest_gpu.log ] && continue; echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items() if 'prepare' not in k and 'emit' not in k})"; done
