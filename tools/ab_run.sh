# A/B timing of fused_ab variants in one GPU call:
#   bash tools/ab_run.sh TAG V1[:mode[:ENV=VAL]] ...   (mode "tc": k_rs_tc one-matrix decode)
set -o pipefail
TAG=$1; shift
O=gpurun_out/ab_$TAG; mkdir -p $O
T="timeout -k 10 120"
for i in 1 2; do for vm in "$@"; do
  IFS=: read -r v m ev <<< "$vm"; m=${m:-fused}
  env $ev $T ./tools/fused_ab_$v 1024 7 "$vm" $m >> $O/ab.log 2>&1 || exit 1; done; done
