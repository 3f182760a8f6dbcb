# round 2: generated code for the general (k x k) decode; GPU suite + (128, 64) and (200, 50) lines
set -o pipefail
O=$(pwd)/gpurun_out/r02r
mkdir -p $O
T="timeout -k 10"
$T 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 128 --loss-rate 0.5 --blocks 256 > $O/k128_gen.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 128 --loss-rate 0.5 --blocks 256 --decode-kernel one_matrix > $O/k128_tc.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 200 --loss-rate 0.25 --blocks 256 > $O/k200_gen.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 200 --loss-rate 0.25 --blocks 256 --decode-kernel one_matrix > $O/k200_tc.log 2>&1
