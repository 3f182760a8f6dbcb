# C4 streamed: generation after the verification (reference order, default)
# vs beside it (--overlap-gen): bash tools/r03_c4order.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
T="timeout -k 10 300"
for rep in 1 2; do
  $T python3 bench.py --config c4 --no-cpu-baseline > $O/c4_serial_$rep.log 2>&1 || exit 1
  $T python3 bench.py --config c4 --overlap-gen --no-cpu-baseline > $O/c4_overlap_$rep.log 2>&1 || exit 1
done
for f in $O/c*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['streamed']['wall_GiBps'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done
