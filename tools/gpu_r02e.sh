# round 2: VGPR bank microbenchmark; k_rs_jit occupancy (4 / 3 / 2 workgroups per CU via extra LDS)
set -o pipefail
O=$(pwd)/gpurun_out/r02e
mkdir -p $O
T="timeout -k 10"
$T 60 ./tools/ubench_bank > $O/ubench_bank.log 2>&1 && \
for x in 0 24576 49152 0; do echo "== extra LDS $x" >> $O/jit_occ.log; $T 60 ./tools/jit_profile 1024 64 32 $x >> $O/jit_occ.log 2>&1 || exit 1; done
