# Does the batch footprint change per-block kernel time? bash tools/r03_footprint.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for nb in 1024 4096 16384; do
  $T python3 bench.py --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks $nb --steps 5 --warmup 1 --no-cpu-baseline > $O/c4geom_$nb.log 2>&1 || exit 1
done
for nb in 16 64 256 1024; do
  $T python3 bench.py --blocks $nb --steps 5 --warmup 1 --no-cpu-baseline > $O/c3_$nb.log 2>&1 || exit 1
done
for f in $O/c4geom_*.log $O/c3_*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); nb=d['config']['blocks_per_gpu']; print(d['value'], {k:(v['avg_ms'], round(v['avg_ms']/nb*1e3,3)) for k,v in d['kernels'].items()})"; done
