# tr8 with 64-bit shifts: GPU suite, then same-box A/B of the HEAD library vs
# tools/ab/librsgpu_base.so (32-bit shifts) at C3 and the C4 geometry
# resident, then streamed C4 with / without regeneration + verification:
# bash tools/r03_tr8ab.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
T="timeout -k 10 200"
for rep in 1 2; do
for v in base head; do
  if [ $v = base ]; then R="python3 tools/ab_lib.py tools/ab/librsgpu_base.so"; else R="python3 bench.py"; fi
  $T $R --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_${v}_$rep.log 2>&1 || exit 1
  $T $R --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4g_${v}_$rep.log 2>&1 || exit 1
done; done
$T python3 bench.py --config c4 --no-cpu-baseline > $O/c4s_serial.log 2>&1 || exit 1
$T python3 bench.py --config c4 --no-regen --no-verify --no-cpu-baseline > $O/c4s_bare.log 2>&1 || exit 1
tail -1 $O/pytest_gpu.log
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('streamed',{}).get('batch_ms_rank0'), {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
