# round 2: k_rs_jit instruction-cache invalidation A/B (every wave / wave 0 only / none), random data
set -o pipefail
O=$(pwd)/gpurun_out/r02k
mkdir -p $O
for pass in 1 2; do
  for v in base inv0 noinv; do
    echo "== $v pass $pass" >> $O/ab.log
    timeout -k 10 60 ./tools/jit_profile_$v 1024 64 32 >> $O/ab.log 2>&1 || exit 1
  done
done
