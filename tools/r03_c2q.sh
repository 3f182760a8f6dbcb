# C2 bench + kernel trace only: bash tools/r03_c2q.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2kt -o run --output-format csv -- python3 bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > $O/c2_kt.log 2>&1
rc=$?; tail -1 $O/c2.log | cut -c1-400; find $O/c2kt -name "*kernel_stats.csv" -exec grep -E "fused|split" {} \; ; echo rc=$rc; exit $rc
