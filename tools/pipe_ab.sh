# C4 decode with prepare + emission beside the decode (rsgpu_decode_blocks'
# slices), same box, interleaved passes (run from the repo root on the box):
#   bash tools/pipe_ab.sh TAG N1 N2 ...   (N: slices; 1 = off, -1 = AUTO)
# -> gpurun_out/pipe_TAG/p<N>_<rep>.log
set -o pipefail
TAG=$1; shift
O=gpurun_out/pipe_$TAG; mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for n in "$@"; do
    timeout -k 10 300 python3 tools/ab_lib.py --decode-pipeline $n --config c4 --steps 1 --no-cpu-baseline $ARGS > $O/p${n}_$rep.log 2>&1 || { tail -20 $O/p${n}_$rep.log; exit 1; }
    grep '^{' $O/p${n}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('p$n', $rep, d['value'], d['streamed']['batch_ms_rank0'], {k:(v['avg_ms'],v['launches']) for k,v in d['kernels'].items()})"
  done
done
