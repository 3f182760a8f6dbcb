# Session-2 GPU call: full parity suite + fused profile + two bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s2x}
mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 120 ./tools/fused_profile 256 > $O/fused_profile.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 && \
$T 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench2.log 2>&1
echo "exit $?"
