# One GPU call that regenerates the round's evidence from the current tree
# (run on the GPU box from the repo root):  bash tools/refresh_round.sh r01
#   GPU parity suite, profile_round.sh (PMC traffic, kernel trace, bench),
#   pmc_sq.sh (SQ counters), phase profile of the generated-code decode
#   (tools/jit_profile: k_rs_jit over 64 sources x 32 rows, built beforehand
#   with the hipcc line in its header), isa_arithmetic peer.
set -o pipefail
TAG=${1:-r01}
O=$(pwd)/gpurun_out/refresh_$TAG
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
bash tools/profile_round.sh $TAG && \
bash tools/pmc_sq.sh $TAG && \
python3 tools/pmc_summary.py gpurun_out/sq_$TAG > $O/sq_summary.txt 2>&1 && \
$T 120 ./tools/jit_profile 1024 64 32 > $O/jit_profile.log 2>&1 && \
$T 120 ./storage-benchmarks_amd/bin/rs_arithmetic --vectors 8 16 32 --runs 3 > $O/arithmetic.log 2>&1
