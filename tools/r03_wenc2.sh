# generated encode, two-wave layout with covered composites (HEAD): GPU
# suite, C5 AUTO (now generated) x2 vs the base library's compiled kernel,
# C3 AUTO (compiled) vs generated, (100, 25) and (128, 32) generated:
# bash tools/r03_wenc2.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
T="timeout -k 10 200"
B="python3 tools/ab_lib.py tools/ab/librsgpu_base.so"
for rep in 1 2; do
$T python3 bench.py --config c5 --steps 5 --no-cpu-baseline > $O/c5_auto_$rep.log 2>&1 || exit 1
$T $B --config c5 --steps 5 --no-cpu-baseline > $O/c5_base_$rep.log 2>&1 || exit 1
done
$T python3 bench.py --steps 5 --no-cpu-baseline > $O/c3_auto.log 2>&1 || exit 1
$T python3 bench.py --steps 5 --no-cpu-baseline --encode-kernel generated > $O/c3_gen.log 2>&1 || exit 1
$T python3 bench.py --steps 4 --no-cpu-baseline --symbols 100 --loss-rate 0.25 --blocks 635 > $O/k100_gen.log 2>&1 || exit 1
$T python3 bench.py --steps 4 --no-cpu-baseline --symbols 128 --loss-rate 0.25 --blocks 497 > $O/k128_gen.log 2>&1 || exit 1
tail -1 $O/pytest_gpu.log
for f in $O/*.log; do [ $f = $O/pytest_gpu.log ] && continue; echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items() if 'prepare' not in k and 'emit' not in k})"; done
