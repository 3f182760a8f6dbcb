# Start-time chunk rotation in k_rs_jit (8 rows per wave, e <= 16; round 5):
# (The rotation in k_rs_jit was removed after this A/B -- profiles/r05_rot/jit8/.)
# its GPU tests, then same-process ABBA (rotation off = 0, the library's
# choice = -1) at three full-row geometries.
#   bash tools/jit8_rot_ab.sh TAG -> gpurun_out/jit8rot_TAG/
set -o pipefail
O=gpurun_out/jit8rot_${1:-x}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py tests/test_gpu_encode.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K="timeout -k 10 600 python3 tools/ab_knob.py --reps ${REPS:-6} --knob rsgpu_internal_set_jitw_rot --values=0,-1"
$K --symbols 64 --erased 16 --blocks 989 --out $O/k64e16.json > $O/k64e16.log 2>&1 && \
$K --symbols 32 --erased 8 --blocks 1959 --out $O/k32e8.json > $O/k32e8.log 2>&1 && \
$K --symbols 48 --erased 12 --blocks 1315 --out $O/k48e12.json > $O/k48e12.log 2>&1
rc=$?
python3 tools/ab_summary.py $O/*.json
exit $rc
