# round 2: geometries without a compiled kernel at full row length, generated vs threaded encode
set -o pipefail
O=$(pwd)/gpurun_out/r02n
mkdir -p $O
T="timeout -k 10"
for g in "32 0.5 1024" "128 0.5 256" "48 0.25 1024" "200 0.16 256"; do
  set -- $g
  for ek in generated threaded; do
    $T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols $1 --loss-rate $2 --blocks $3 --encode-kernel $ek > $O/k$1_l$2_$ek.log 2>&1 || exit 1
  done
done
