# Geometry sweep at full row length (L = 1e6), AUTO kernels, ~64-96 GB per step:
#   bash tools/geom_sweep.sh TAG  -> gpurun_out/sweep_TAG/k<K>_l<LOSS>.log
set -o pipefail
TAG=${1:-x}
O=$(pwd)/gpurun_out/sweep_$TAG
mkdir -p $O
T="timeout -k 10 200"
# e > 64 (round 4: passes of <= 64 rows): (150, 100), (125, 125), (160, 65)
for g in "150 0.66666 400" "125 1.0 400" "160 0.40625 500"; do
  set -- $g
  $T python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --symbols $1 --loss-rate $2 --blocks $3 > $O/k$1_l$2.log 2>&1 || exit 1
done
for k in 8 16 32 48 64 100 128 200; do
  for loss in 0.25 0.5; do
    B=$(( 96000 / (k * 3 / 2 + 1) ))
    [ $B -gt 2048 ] && B=2048
    $T python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --symbols $k --loss-rate $loss --blocks $B > $O/k${k}_l${loss}.log 2>&1 || exit 1
  done
done
