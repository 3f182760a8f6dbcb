# round 2, first GPU call: GPU parity suite, then the profile round
set -o pipefail
O=$(pwd)/gpurun_out/r02a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
bash tools/profile_round.sh r02
