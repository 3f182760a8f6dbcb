# round 2: k_rs_jit tiles per workgroup (1 / 2 / 4), per-block code and one shared program
set -o pipefail
O=$(pwd)/gpurun_out/r02o
mkdir -p $O
for pass in 1 2; do
  for nt in 1 2 4; do
    echo "== per-block nt=$nt pass $pass" >> $O/ab.log
    timeout -k 10 60 ./tools/jit_profile 1024 64 32 0 $nt >> $O/ab.log 2>&1 || exit 1
    echo "== shared nt=$nt pass $pass" >> $O/ab.log
    timeout -k 10 60 ./tools/jit_profile_b0 1024 64 32 0 $nt >> $O/ab.log 2>&1 || exit 1
  done
done
