# round 2: JIT decode phase profile + code-sharing timing variants, SQ counters,
# C2/C4/C5 bench lines
set -o pipefail
O=$(pwd)/gpurun_out/r02b
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 120 ./tools/jit_profile 1024 64 32 > $O/jit_profile.log 2>&1 && \
$T 120 ./tools/jit_profile_w0 1024 64 32 > $O/jit_profile_w0.log 2>&1 && \
$T 120 ./tools/jit_profile_b0 1024 64 32 > $O/jit_profile_b0.log 2>&1 && \
bash tools/pmc_sq.sh r02 && \
python3 tools/pmc_summary.py gpurun_out/sq_r02 > $O/sq_summary.txt 2>&1 && \
$T 300 python3 bench.py --config c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 && \
$T 200 python3 bench.py --config c5 --no-cpu-baseline --steps 5 > $O/bench_c5.log 2>&1 && \
$T 200 python3 bench.py --config c2 --no-cpu-baseline --steps 20 > $O/bench_c2.log 2>&1
