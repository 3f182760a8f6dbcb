# Session-2 GPU call: full parity suite (default + Horner syndrome variant),
# fused profile and A/B bench of the two syndrome phases on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s2x}
mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
RSGPU_FUSED_SYN=horner $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or round_trip or oracle_decode or sign_bit or erasure_counts" > $O/pytest_horner.log 2>&1 && \
$T 120 ./tools/fused_profile 1024 > $O/fused_profile.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_tc.log 2>&1 && \
RSGPU_FUSED_SYN=horner $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_horner.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_tc2.log 2>&1 && \
RSGPU_FUSED_SYN=horner $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_horner2.log 2>&1
echo "exit $?"
