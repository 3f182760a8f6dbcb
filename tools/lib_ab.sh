# Library builds A/B, same box, interleaved passes (run from the repo root on
# the box):
#   CONFIGS="c3 c4" bash tools/lib_ab.sh TAG name:LIB.so[:ab_lib.py knobs] ...
#   -> gpurun_out/libab_TAG/<name>_<config>_<rep>.log
# Each library first passes a filtered GPU suite (TESTS_K, default the
# small-decode tests; TESTS_K=none skips), then every pass runs
# `bench.py --config C` once per library and config (REPS passes, default 3).
set -o pipefail
TAG=$1; shift
O=gpurun_out/libab_$TAG; mkdir -p $O
K=${TESTS_K:-"syn or fused or split or c2 or isal"}
parse() { n=${1%%:*}; r=${1#*:}; lib=${r%%:*}; x=""; [ "$r" != "$lib" ] && x=${r#*:}; }
for spec in "$@"; do
  parse "$spec"
  [ "$K" = none ] && break
  RSGPU_LIB=$PWD/$lib timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$K" > $O/tests_$n.log 2>&1 || { tail -20 $O/tests_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/tests_$n.log)"
done
for rep in $(seq 1 ${REPS:-3}); do
  for c in ${CONFIGS:-c2}; do
    st=5; [ $c = c2 ] && st=300; [ $c = c4 ] && st=1
    for spec in "$@"; do
      parse "$spec"
      timeout -k 10 300 python3 tools/ab_lib.py --lib $lib $x --config $c --steps $st --no-cpu-baseline > $O/${n}_${c}_$rep.log 2>&1 || { tail -20 $O/${n}_${c}_$rep.log; exit 1; }
      grep '^{' $O/${n}_${c}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', '$c', $rep, d['value'], d['ms_per_step'], {k:round(v['avg_ms'],3) for k,v in d['kernels'].items()})"
    done
  done
done
