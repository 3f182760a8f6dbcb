# round 2: GPU suite + C2-C5 bench lines after the coalesced code emission and the AUTO tile heuristic
set -o pipefail
O=$(pwd)/gpurun_out/r02f
mkdir -p $O
T="timeout -k 10"
$T 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline > $O/c3.log 2>&1 && \
$T 300 python3 bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 && \
$T 120 python3 bench.py --config c2 --no-cpu-baseline --steps 50 > $O/c2.log 2>&1 && \
$T 120 python3 bench.py --config c2 --no-cpu-baseline --steps 50 --decode-kernel generated > $O/c2_gen.log 2>&1 && \
$T 200 python3 bench.py --config c5 --no-cpu-baseline --steps 5 > $O/c5.log 2>&1
