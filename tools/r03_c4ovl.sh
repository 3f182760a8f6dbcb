# streamed C4: decode prepare beside the encode (default) vs after it, two
# (the --serial-prepare A/B of the round-3 overlap experiment; bench.py no longer has the overlap)
# passes; the C4 GPU tests: bash tools/r03_c4ovl.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for rep in 1 2; do
$T python3 bench.py --config c4 --no-cpu-baseline > $O/c4_ovl_$rep.log 2>&1 || exit 1
$T python3 bench.py --config c4 --serial-prepare --no-cpu-baseline > $O/c4_ser_$rep.log 2>&1 || exit 1
done
$T python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1 || exit 1
tail -1 $O/pytest_gpu.log
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('streamed',{}); print(d['value'], d['verified'], s.get('batch_ms_rank0'), s.get('wall_s'), {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
