# The 8-row generated decode (k_rs_jit) with / without XCD-contiguous order at
# the C3 and C5 shapes; run on the GPU box from the repo root
set -o pipefail
O=gpurun_out/ab_xcd8; mkdir -p $O
for i in 1 2; do for shape in "1024 64 32" "512 100 20"; do for x in 0 1; do
  echo "== $shape xcd $x pass $i" >> $O/ab.log
  timeout -k 10 120 ./tools/jit_profile $shape 0 0 $x | grep "^rep" >> $O/ab.log || exit 1
done; done; done
