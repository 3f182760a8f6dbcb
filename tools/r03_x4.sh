# Four-wave generated decode / encode for 32 < e <= 64: GPU suite, then the
# e > 32 geometries of the sweep (k 100 / 128 at loss 0.5; L = 1e6) and
# (96, 48): bash tools/r03_x4.sh TAG
set -o pipefail
O=gpurun_out/r03_x4_$1; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
T="timeout -k 10 200"
for k in 100 128 64; do
  B=$(( 96000 / (k * 3 / 2 + 1) ))
  $T python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --symbols $k --loss-rate 0.5 --blocks $B > $O/k${k}_l0.5.log 2>&1 || exit 1
done
$T python3 bench.py --no-cpu-baseline --steps 4 --warmup 1 --symbols 96 --loss-rate 0.5 --blocks 600 > $O/k96_l0.5.log 2>&1 || exit 1
for f in $O/k*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['launches'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
