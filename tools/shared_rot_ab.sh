# Start-time chunk rotation in the shared generated program (every block on
# the same code; round 5), same process ABBA per geometry (tools/ab_knob.py).
#   bash tools/shared_rot_ab.sh TAG   -> gpurun_out/shrot_TAG/
set -o pipefail
O=gpurun_out/shrot_${1:-x}; mkdir -p $O
K="timeout -k 10 600 python3 tools/ab_knob.py --reps ${REPS:-6}"
$K --encode-kernel generated --knob rsgpu_internal_set_jitw_rot --values=0,-1 --out $O/c3_generated_rot.json > $O/c3_generated_rot.log 2>&1 && \
$K --knob encode_kernel --values compiled,generated --out $O/c3_compiled_vs_generated.json > $O/c3_cvg.log 2>&1 && \
$K --symbols 100 --erased 20 --blocks 512 --knob rsgpu_internal_set_jitw_rot --values=0,-1 --out $O/c5_rot.json > $O/c5_rot.log 2>&1 && \
$K --symbols 48 --erased 24 --blocks 1024 --knob rsgpu_internal_set_jitw_rot --values=0,-1 --out $O/k48e24_rot.json > $O/k48e24_rot.log 2>&1 && \
$K --symbol-size 32000 --blocks 16384 --knob rsgpu_internal_set_jitw_rot --values=0,-1 --out $O/c4_rot.json > $O/c4_rot.log 2>&1
rc=$?
for f in $O/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); vals=[k for k in d if isinstance(d[k],dict) and 'step_ms_median' in d[k]]
print('$f', d['verified'], [(v, d[v]['step_ms_median'], d[v]['kernels_ms_median']) for v in vals], [d[v].get([x for x in d[v] if x.startswith('paired')][0]) for v in vals[1:]])"; done
exit $rc
