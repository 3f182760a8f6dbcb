set -o pipefail
O=gpurun_out/c4probe; mkdir -p $O
T="timeout -k 10 200"
for rep in 1 2; do
$T python3 bench.py --config c4 --steps 1 --no-cpu-baseline > $O/c4_verify_$rep.log 2>&1 || exit 1
$T python3 bench.py --config c4 --steps 1 --no-cpu-baseline --no-verify > $O/c4_noverify_$rep.log 2>&1 || exit 1
$T python3 bench.py --symbols 64 --symbol-size 32000 --loss-rate 0.5 --blocks 16384 --steps 4 --no-cpu-baseline > $O/c4res_$rep.log 2>&1 || exit 1
done
for f in $O/*.log; do echo $(basename $f) $(grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items()}, d.get('streamed',{}).get('batch_ms_rank0'))"); done
