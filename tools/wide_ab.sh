# e >= 64 at L = 1e6: this build vs another library build (round 4: closed
# form for every e + passes of <= 64 rows, against round 3's k x k inversion
# at e = 64 and passes of 32 rows above):
#   bash tools/wide_ab.sh TAG BASELIB.so    -> gpurun_out/wide_TAG/
set -o pipefail
TAG=$1; BASE=$2
O=$(pwd)/gpurun_out/wide_$TAG; mkdir -p $O
T="timeout -k 10 240"
for g in "150 0.66666 400" "125 1.0 400" "160 0.40625 500" "128 0.5 497"; do
  set -- $g
  for rep in 1 2; do
    $T python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --symbols $1 --loss-rate $2 --blocks $3 > $O/k$1_head_$rep.log 2>&1 || exit 1
    $T python3 tools/ab_lib.py --lib $BASE --no-cpu-baseline --steps 3 --warmup 1 --symbols $1 --loss-rate $2 --blocks $3 > $O/k$1_base_$rep.log 2>&1 || exit 1
  done
done
for f in $O/*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['config']['erased'], d['ms_per_step'], {k:(v['avg_ms'],v['launches']) for k,v in d['kernels'].items()})"; done
