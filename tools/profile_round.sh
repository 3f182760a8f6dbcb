# Collect the round's profile evidence on the GPU box (run from the repo root):
#   bash tools/profile_round.sh r01
# -> gpurun_out/prof_<tag>/ (kernel trace + stats, PMC FETCH/WRITE, traffic json,
#    bench line with --traffic).  Copy the summaries into profiles/.
set -o pipefail
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 && \
python3 tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/traffic.json > $O/traffic.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --traffic $O/traffic.json > $O/bench_under_rocprof.log 2>&1 && \
timeout -k 10 600 python3 bench.py --traffic $O/traffic.json --host-io 64 > $O/bench.log 2>&1
