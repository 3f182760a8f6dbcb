# The pipelined C4 decode with a short first slice (round 5) against equal
# (The knob rsgpu_internal_set_decode_pipe_first and the short first slice were
# removed after this A/B -- profiles/r05_c4/README.md.)
# slices: GPU tests of the slicing, then a same-process ABBA at C4's batch.
#   bash tools/pipe_first_ab.sh TAG -> gpurun_out/pfirst_TAG/
set -o pipefail
O=gpurun_out/pfirst_${1:-x}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "pipelined or c4 or poisoned" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python3 tools/ab_knob.py --reps ${REPS:-8} --symbol-size 32000 --blocks 16384 \
    --knob rsgpu_internal_set_decode_pipe_first --values=0,-1 --out $O/c4.json > $O/c4.log 2>&1
rc=$?
python3 tools/ab_summary.py $O/c4.json
exit $rc
