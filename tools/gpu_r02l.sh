# round 2: timing-only A/B of the decode's composite count per source (22 / 18 / 13), random data
set -o pipefail
O=$(pwd)/gpurun_out/r02l
mkdir -p $O
for pass in 1 2; do
  for v in base c18 c13; do
    echo "== $v pass $pass" >> $O/ab.log
    timeout -k 10 60 ./tools/jit_profile_$v 1024 64 32 >> $O/ab.log 2>&1 || exit 1
  done
done
