# round 2: sliced >65535-block batches, per-(block, wave) code emission; GPU suite + C3 line
set -o pipefail
O=$(pwd)/gpurun_out/r02i
mkdir -p $O
T="timeout -k 10"
$T 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1
