# Column tiles per workgroup of k_rs_jitw (decode and the shared generated
# encode), same-process ABBA at C5 and at C3 with the generated encode:
#   bash tools/tpw_ab.sh -> gpurun_out/tpw_a/
set -o pipefail
O=gpurun_out/tpw_a; mkdir -p $O
K="timeout -k 10 600 python3 tools/ab_knob.py --reps 4 --knob rsgpu_internal_set_jitw_tiles --values=2,3,1"
$K --symbols 100 --erased 20 --blocks 512 --out $O/c5.json > $O/c5.log 2>&1 && \
$K --encode-kernel generated --out $O/c3_gen.json > $O/c3_gen.log 2>&1
rc=$?
python3 tools/ab_summary.py $O/*.json
exit $rc
