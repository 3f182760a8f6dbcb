# Session-2 GPU call: decode parity (default + DMA variant) + A/B bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s2x}
mkdir -p $O
T="timeout -k 10"
K="golden or round_trip or oracle_decode or sign_bit or erasure_counts"
$T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest_a.log 2>&1 && \
RSGPU_FUSED_LOAD=dma $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest_b.log 2>&1 && \
for i in 1 2; do
  $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_a$i.log 2>&1 && \
  RSGPU_FUSED_LOAD=dma $T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_b$i.log 2>&1 || exit 1
done
echo "exit $?"
