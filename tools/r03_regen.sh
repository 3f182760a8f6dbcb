# Does the streamed C4's on-device generation slow its timed encode? bash tools/r03_regen.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 200"
for rep in 1 2; do
  $T python3 bench.py --config c4 --warmup 1 --no-cpu-baseline > $O/c4_regen_$rep.log 2>&1 || exit 1
  $T python3 bench.py --config c4 --warmup 1 --no-cpu-baseline --no-regen > $O/c4_noregen_$rep.log 2>&1 || exit 1
done
for f in $O/c4_*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['streamed']['wall_s'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
