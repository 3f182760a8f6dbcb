# Round 6 final evidence at HEAD in one GPU call: the round's refresh
# (suite, smoke, PMC traffic, kernel trace, SQ counters, the bench lines of
# C1-C5, host IO) plus C4's PMC traffic and the driver's exact command.
#   gpurun -- bash tools/final_r06.sh TAG
set -o pipefail
TAG=${1:-r06b}
bash tools/refresh_r06.sh $TAG &&
bash tools/c4_traffic.sh $TAG &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/refresh_$TAG/bench_driver_cmd.log 2>&1
