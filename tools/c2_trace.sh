# C2 kernel trace: per-kernel durations and the gaps between consecutive
# kernels of the timed steps (run from the repo root on the box):
#   bash tools/c2_trace.sh TAG  -> gpurun_out/c2trace_TAG/
set -o pipefail
TAG=${1:-x}
O=$(pwd)/gpurun_out/c2trace_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --config c2 --steps 300 --no-cpu-baseline $ARGS > $O/bench.log 2>&1 && \
python3 tools/trace_gaps.py $O/kt/run_kernel_trace.csv > $O/gaps.txt && cat $O/gaps.txt
