# The round's bench line against the round's committed counters (after
# refresh_round.sh copied them into profiles/): bash tools/r03_bench_line.sh TAG
set -o pipefail
O=gpurun_out/r03_$1; mkdir -p $O
timeout -k 10 600 python3 bench.py --host-io 64 > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log > $O/bench.json
