# same-box A/B: HEAD library vs tools/ab/librsgpu_base.so: bash tools/r03_abptr.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for rep in 1 2; do
for v in base head; do
  if [ $v = base ]; then R="python3 tools/ab_lib.py tools/ab/librsgpu_base.so"; else R="python3 bench.py"; fi
  $T $R --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_${v}_$rep.log 2>&1 || exit 1
  $T $R --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4g_${v}_$rep.log 2>&1 || exit 1
  $T $R --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$rep.log 2>&1 || exit 1
done; done
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
