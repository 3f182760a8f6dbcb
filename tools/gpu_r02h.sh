# round 2: one-workgroup-per-block code emission; GPU suite + C3/C2 bench lines
set -o pipefail
O=$(pwd)/gpurun_out/r02h
mkdir -p $O
T="timeout -k 10"
$T 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1 && \
$T 120 python3 bench.py --config c2 --no-cpu-baseline --steps 50 > $O/c2.log 2>&1
