# k_rs_jitw's row pointers from an LDS copy of the block's table vs scalar
# (The knob rsgpu_internal_set_jitw_ptr_lds and the LDS table were removed after
# this A/B -- profiles/r05_plds/README.md; the script is kept as the record.)
# loads (round 5), same-process ABBA per config (tools/ab_knob.py), after
# the GPU tests of the kernel.   bash tools/ptr_lds_ab.sh TAG -> gpurun_out/plds_TAG/
set -o pipefail
O=gpurun_out/plds_${1:-x}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "pointer_table or chunk_rotation or poisoned" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 600 python3 tools/ab_knob.py --reps ${REPS:-6} --knob rsgpu_internal_set_jitw_ptr_lds --values=0,1"
$K --out $O/c3.json > $O/c3.log 2>&1 && \
$K --symbol-size 32000 --blocks 16384 --out $O/c4.json > $O/c4.log 2>&1 && \
$K --symbols 100 --erased 20 --blocks 512 --out $O/c5.json > $O/c5.log 2>&1
rc=$?
for f in $O/*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); vals=[k for k in d if isinstance(d[k],dict) and 'step_ms_median' in d[k]]
print('$f', d['verified'], [(v, d[v]['step_ms_median'], d[v]['kernels_ms_median']) for v in vals], [d[v].get([x for x in d[v] if x.startswith('paired')][0]) for v in vals[1:]])"; done
exit $rc
