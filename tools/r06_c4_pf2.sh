# Round 6: the C4 decode's code prefetch also pulling the NEXT block's code
# into L2 (mode 2) against the product's own-block prefetch (1), one process,
# ABBA x8.   gpurun -- bash tools/r06_c4_pf2.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_c4_pf2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_jitw_prefetch --values=1,2 --reps 8 --symbol-size 32000 --blocks 16384 --out $O/ab_c4.json > $O/ab_c4.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode.py -x -q -m gpu -k "c4 or pipelined or rotation" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 ;
python3 - "$O" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/ab_c4.json"))
vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
print(d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs}, [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
tail -1 $O/pytest.log
