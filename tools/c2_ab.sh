# C2 small-batch kernels, same box: libraries interleaved over REPS passes
# (run from the repo root on the box):
#   bash tools/c2_ab.sh TAG name:LIB.so [name:LIB.so ...] -> gpurun_out/c2ab_TAG/
# Each library first passes the small-decode GPU tests, then every pass runs
# `bench.py --config c2` once per library.
set -o pipefail
TAG=$1; shift
O=gpurun_out/c2ab_$TAG; mkdir -p $O
for spec in "$@"; do
  n=${spec%%:*}; lib=${spec#*:}
  RSGPU_LIB=$PWD/$lib timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "syn or fused or split or c2 or isal" > $O/tests_$n.log 2>&1 || { tail -20 $O/tests_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/tests_$n.log)"
done
for rep in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    n=${spec%%:*}; lib=${spec#*:}
    timeout -k 10 300 python3 tools/ab_lib.py --lib $lib --config c2 --steps 300 --no-cpu-baseline > $O/${n}_$rep.log 2>&1 || { tail -20 $O/${n}_$rep.log; exit 1; }
    grep '^{' $O/${n}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', $rep, d['value'], d['ms_per_step'], {k:round(v['avg_ms']*1000,2) for k,v in d['kernels'].items()})"
  done
done
