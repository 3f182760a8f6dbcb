# Bench lines of the other BASELINE configs (C3 is bench.py's default workload):
#   bash tools/bench_configs.sh   -> gpurun_out/cfgs/cN.log
set -o pipefail
O=gpurun_out/cfgs; mkdir -p $O
T="timeout -k 10 300"
for c in c2 c4 c5; do $T python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $O/$c.log 2>&1 || exit 1; done
