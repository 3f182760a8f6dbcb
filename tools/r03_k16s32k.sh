# (16, 8, 32000), the reference's `--symbols=16 --symbol_size=32000` sweep
# point (README.rst:130) at loss 0.5: decode kernel choices, 16384 blocks
set -o pipefail
O=gpurun_out/r03_k16s32k; mkdir -p $O
T="timeout -k 10 200"
for kern in auto generated one_matrix; do
  $T python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --symbols 16 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --decode-kernel $kern > $O/$kern.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:(v['avg_ms'],v['alg_GBps']) for k,v in d['kernels'].items()})"; done
