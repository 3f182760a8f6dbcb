# Session-2 GPU call: decode parity + profile + bench (default and C=16).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s2b}
mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or round_trip or oracle_decode or sign_bit or erasure_counts" > $O/pytest_dec.log 2>&1 && \
RSGPU_FUSED_C=16 $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or round_trip or oracle_decode or sign_bit or erasure_counts" > $O/pytest_dec16.log 2>&1 && \
$T 120 ./tools/fused_profile 256 > $O/fused_profile_c8.log 2>&1 && \
RSGPU_FUSED_C=16 $T 120 ./tools/fused_profile 256 > $O/fused_profile_c16.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c8.log 2>&1 && \
RSGPU_FUSED_C=16 $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_c16.log 2>&1
echo "exit $?"
