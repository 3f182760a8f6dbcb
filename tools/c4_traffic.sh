# C4 HBM traffic per kernel (FETCH_SIZE, WRITE_SIZE in separate passes) over
# one streamed run (run on the GPU box from the repo root):
#   bash tools/c4_traffic.sh TAG  -> gpurun_out/c4traffic_TAG/traffic.json
set -o pipefail
TAG=${1:-x}
O=$(pwd)/gpurun_out/c4traffic_$TAG
mkdir -p $O
export TMPDIR=/tmp
B=${C4_BENCH:-"python3 bench.py --config c4 --steps 1 --no-cpu-baseline --no-verify"}  # C4_BENCH: another run
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B > $O/pmc_write.log 2>&1 && \
python3 tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv $O/traffic.json > $O/traffic.log 2>&1 && cat $O/traffic.log
