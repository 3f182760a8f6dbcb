# A/B timing of enc_ab variants in one GPU call:  bash tools/ab_enc.sh TAG V1 V2 ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/abe_$TAG; mkdir -p $O
for i in 1 2; do for v in "$@"; do
  timeout -k 10 120 ./tools/enc_ab_$v 1024 7 $v >> $O/ab.log 2>&1 || exit 1; done; done
