set -o pipefail
O=gpurun_out/r03_base; mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10 300"
$T python3 bench.py --no-cpu-baseline --steps 10 > $O/c3.log 2>&1 && \
$T python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 && \
$T rocprofv3 --kernel-trace --stats -d $O/c2kt -o run --output-format csv -- python3 bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2_kt.log 2>&1 && \
$T python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1
echo rc=$?
