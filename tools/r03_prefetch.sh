# code-prefetch A/B of the two-wave generated decode: bash tools/r03_prefetch.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "prefetch or jitw_tiles" > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
for p in 0 1; do
  $T python3 bench.py --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --decode-kernel generated --jitw-prefetch $p --steps 3 --warmup 1 --no-cpu-baseline > $O/c4g_p${p}_$rep.log 2>&1 || exit 1
  $T python3 bench.py --jitw-prefetch $p --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_p${p}_$rep.log 2>&1 || exit 1
done; done
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
