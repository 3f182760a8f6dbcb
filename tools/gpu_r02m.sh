# round 2: generated (host-built, shared) encode: GPU suite, then C3 compiled vs generated encode, twice
set -o pipefail
O=$(pwd)/gpurun_out/r02m
mkdir -p $O
T="timeout -k 10"
$T 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
for pass in 1 2; do
  for ek in compiled generated; do
    $T 200 python3 bench.py --no-cpu-baseline --steps 10 --encode-kernel $ek > $O/c3_${ek}_$pass.log 2>&1 || exit 1
  done
done
