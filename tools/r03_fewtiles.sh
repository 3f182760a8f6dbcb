# Below 16 tiles: (16, 8) at 16000 and 8192 bytes (8 / 4 tiles, 10 KB of
# code per block), AUTO (generated, <= 6 KB per tile) against threaded
set -o pipefail
O=gpurun_out/r03_fewtiles; mkdir -p $O
T="timeout -k 10 200"
for L in 16000 8192; do
  B=$(( 16384 * 32000 / L ))
  $T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size $L --loss-rate 0.5 --blocks $B > $O/L${L}_auto.log 2>&1 || exit 1
  $T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size $L --loss-rate 0.5 --blocks $B --decode-kernel one_matrix > $O/L${L}_tc.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
