# Decode kernel choice A/B per BASELINE config, same box:
#   bash tools/ab_decode_modes.sh [configs...]   (default: c5 c3 c2)
set -o pipefail
O=gpurun_out/modes; mkdir -p $O
T="timeout -k 10 300"
CFGS=${@:-c5 c3 c2}
for c in $CFGS; do for m in generated one_matrix; do $T python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --decode-kernel $m > $O/${c}_$m.log 2>&1 || exit 1; done; done
