# A/B of the generated decode's multiply-accumulate order within a source
# (tools/jit_profile argv[5]: 0 as emitted, 1 by (L, H) operands, 2 by (H, L));
# run on the GPU box from the repo root:  bash tools/ab_mac_order.sh
set -o pipefail
O=gpurun_out/ab_mac_order; mkdir -p $O
for i in 1 2; do for m in 0 1 2; do
  echo "== order $m pass $i" >> $O/ab.log
  timeout -k 10 120 ./tools/jit_profile 1024 64 32 0 $m | grep "^rep" >> $O/ab.log || exit 1
done; done
