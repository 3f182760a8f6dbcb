# round 2: C4 (streamed, generation off the timed kernels) generated vs threaded-code decode; C2 both
set -o pipefail
O=$(pwd)/gpurun_out/r02d
mkdir -p $O
T="timeout -k 10"
$T 300 python3 bench.py --config c4 --no-cpu-baseline --decode-kernel generated > $O/c4_gen.log 2>&1 && \
$T 300 python3 bench.py --config c4 --no-cpu-baseline --decode-kernel one_matrix > $O/c4_tc.log 2>&1 && \
$T 120 python3 bench.py --config c2 --no-cpu-baseline --steps 50 --decode-kernel generated > $O/c2_gen.log 2>&1 && \
$T 120 python3 bench.py --config c2 --no-cpu-baseline --steps 50 --decode-kernel one_matrix > $O/c2_tc.log 2>&1 && \
$T 200 python3 bench.py --config c5 --no-cpu-baseline --steps 5 --decode-kernel one_matrix > $O/c5_tc.log 2>&1 && \
$T 200 python3 bench.py --config c5 --no-cpu-baseline --steps 5 --decode-kernel fused > $O/c5_fused.log 2>&1
