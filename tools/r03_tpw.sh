# tiles-per-workgroup A/B of the two-wave generated decode: bash tools/r03_tpw.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "jitw_tiles or poisoned_decode_every" > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
for t in 1 2 3; do
  $T python3 bench.py --jitw-tiles $t --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_t${t}_$rep.log 2>&1 || exit 1
  $T python3 bench.py --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --decode-kernel generated --jitw-tiles $t --steps 3 --warmup 1 --no-cpu-baseline > $O/c4g_t${t}_$rep.log 2>&1 || exit 1
  $T python3 bench.py --config c5 --jitw-tiles $t --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_t${t}_$rep.log 2>&1 || exit 1
done; done
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
