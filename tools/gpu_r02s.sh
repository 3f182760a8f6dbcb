# round 2: closed-form generated decode for 32 < e <= 63; GPU suite + (200, 50) and (128, 40) lines
set -o pipefail
O=$(pwd)/gpurun_out/r02s
mkdir -p $O
T="timeout -k 10"
$T 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 200 --loss-rate 0.25 --blocks 256 > $O/k200_gen.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 128 --loss-rate 0.3 --blocks 256 > $O/k128_l03_gen.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbols 128 --loss-rate 0.3 --blocks 256 --decode-kernel general > $O/k128_l03_general.log 2>&1
