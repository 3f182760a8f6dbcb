# Round 6: the extended drawn-geometry parity run at HEAD (as round 5's
# fuzz3000) plus three back-to-back default bench lines on one box.
#   gpurun -- bash tools/r06_fuzz.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_fuzz}; mkdir -p $O
export TMPDIR=/tmp
RSGPU_FUZZ_N=2000 RSGPU_FUZZ_GENERAL_N=400 RSGPU_FUZZ_API_N=600 timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_fuzz.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/fuzz3000_pytest.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || exit 1; done
tail -1 $O/fuzz3000_pytest.log
for i in 1 2 3; do grep '^{' $O/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['hbm_roofline_frac_step'])"; done
