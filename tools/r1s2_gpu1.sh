# Session-2 GPU call 1 (run from the repo root on the GPU box): parity suite,
# variant parity, fused-decode phase profiles, bench per kernel variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s2a
mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
RSGPU_BS_VARIANT=1 RSGPU_FUSED_C=16 $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or round_trip or oracle_decode or sign_bit or erasure_counts" > $O/pytest_variants.log 2>&1 && \
$T 120 ./tools/fused_profile 256 > $O/fused_profile_c8.log 2>&1 && \
RSGPU_FUSED_C=16 $T 120 ./tools/fused_profile 256 > $O/fused_profile_c16.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_v0.log 2>&1 && \
RSGPU_BS_VARIANT=1 RSGPU_FUSED_C=16 $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_v1.log 2>&1
echo "exit $?"
