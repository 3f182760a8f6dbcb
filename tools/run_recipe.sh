# One parameterised GPU-box recipe (run from the repo root on the box):
#   bash tools/run_recipe.sh TAG STEP [STEP ...]      -> gpurun_out/TAG/
# Steps (each under its own time limit; the first failure ends the recipe):
#   tests   the GPU suite (pytest -m gpu)         smoke   __graft_entry__.smoke()
#   c2 c3 c4 c5   bench.py --config cN lines       line    the default bench line (+ host IO)
#   sweep   tools/geom_sweep.sh                    bound   tools/bound_run.sh
#   prof    tools/profile_round.sh (kernel trace, PMC traffic)   sq   tools/pmc_sq.sh
#   arith   the isa_arithmetic peer (bin/rs_arithmetic)
# Variants through the environment:
#   BENCH="python3 tools/ab_lib.py --lib X.so --jitw-tiles 2"   (default: python3 bench.py)
#   ARGS="--decode-kernel generated"   extra bench.py arguments
#   REPS=2                             repeat each bench step (same-box A/B)
#   TESTS_K="jitw or poisoned"         pytest -k filter for `tests`
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
B=${BENCH:-python3 bench.py}
T="timeout -k 10 300"
summ() { for f in "$@"; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['verified'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"; done; }
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
           tail -1 $O/pytest_gpu.log ;;
    smoke) $T python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; tail -1 $O/smoke.log ;;
    c2|c3|c4|c5)
      for rep in $(seq 1 ${REPS:-1}); do
        st=5; [ $step = c2 ] && st=300; [ $step = c4 ] && st=1
        $T $B --config $step --steps $st --no-cpu-baseline $ARGS > $O/${step}_$rep.log 2>&1 || { tail -20 $O/${step}_$rep.log; exit 1; }
        summ $O/${step}_$rep.log
      done ;;
    line) timeout -k 10 600 $B --host-io 64 $ARGS > $O/bench.log 2>&1 || exit 1; grep '^{' $O/bench.log > $O/bench.json; summ $O/bench.log ;;
    sweep) bash tools/geom_sweep.sh $TAG || true ;;
    bound) bash tools/bound_run.sh $TAG || exit 1; cat gpurun_out/bound_$TAG/summary.log ;;
    prof) bash tools/profile_round.sh $TAG || exit 1 ;;
    sq) bash tools/pmc_sq.sh $TAG || exit 1 ;;
    arith) timeout -k 10 120 ./storage-benchmarks_amd/bin/rs_arithmetic --vectors 8 16 32 --runs 3 > $O/arithmetic.log 2>&1 || exit 1; tail -5 $O/arithmetic.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
