# round 2: C4 with the generated decode in XCD-contiguous order vs threaded code
set -o pipefail
O=$(pwd)/gpurun_out/r02p
mkdir -p $O
T="timeout -k 10"
$T 300 python3 bench.py --config c4 --no-cpu-baseline --decode-kernel generated > $O/c4_gen_xcd.log 2>&1 && \
$T 300 python3 bench.py --config c4 --no-cpu-baseline --decode-kernel one_matrix > $O/c4_tc.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbol-size 128000 --decode-kernel generated > $O/l128k_gen_xcd.log 2>&1 && \
$T 200 python3 bench.py --no-cpu-baseline --steps 5 --symbol-size 128000 --decode-kernel one_matrix > $O/l128k_tc.log 2>&1
