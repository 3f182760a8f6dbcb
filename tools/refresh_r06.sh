# Round-6 evidence at HEAD in one GPU call (run from the repo root on the box):
#   GPU suite, smoke, PMC traffic + kernel trace (profile_round.sh), SQ
#   counters (pmc_sq.sh), the bench line on this call's own counter files,
#   the default `python bench.py` line (the driver's command), the C1 CPU
#   line and the C2 / C4 / C5 lines.   bash tools/refresh_r06.sh TAG
set -o pipefail
TAG=${1:-r06}
O=$(pwd)/gpurun_out/refresh_$TAG
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
$T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
bash tools/profile_round.sh $TAG && \
bash tools/pmc_sq.sh $TAG && \
python3 tools/pmc_summary.py gpurun_out/sq_$TAG > $O/sq_summary.txt 2>&1 && \
$T 600 python3 bench.py --traffic gpurun_out/prof_$TAG/traffic.json --sq-counters $O/sq_summary.txt --host-io 64 > $O/bench.log 2>&1 && \
$T 300 python3 bench.py > $O/bench_default.log 2>&1 && \
$T 300 python3 bench.py --config c1 > $O/c1.log 2>&1 && \
$T 300 python3 bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.log 2>&1 && \
$T 300 python3 bench.py --config c4 --no-cpu-baseline > $O/c4.log 2>&1 && \
$T 300 python3 bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>&1
