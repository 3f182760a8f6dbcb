# AUTO decode-kernel thresholds, same box, interleaved reps:
# generated vs threaded-code decode where AUTO's choice rests on a small
# margin.  bash tools/auto_ab.sh TAG -> gpurun_out/auto_TAG/
set -o pipefail
TAG=$1
O=$(pwd)/gpurun_out/auto_$TAG; mkdir -p $O
T="timeout -k 10 200"
for g in "16 0.5 8192 65535" "16 0.5 16384 65535" "64 0.5 32000 16384" "64 0.25 32000 16384" "128 0.125 32000 8192"; do
  set -- $g
  for rep in 1 2 3; do
    for dk in generated one_matrix; do
      $T python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --symbols $1 --loss-rate $2 --symbol-size $3 --blocks $4 --decode-kernel $dk > $O/k$1_l$2_L$3_${dk}_$rep.log 2>&1 || exit 1
    done
  done
done
for f in $O/*.log; do echo $(basename $f) $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items() if 'dec' in k or 'emit' in k or 'prep' in k})"); done
