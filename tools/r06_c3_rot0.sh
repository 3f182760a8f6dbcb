# Round 6: C3 chunk rotation off vs on with the wave priority on (one
# process, ABBA x8).   gpurun -- bash tools/r06_c3_rot0.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_c3_rot0}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_jitw_rot --values=-1,0 --reps 8 --out $O/ab_c3.json > $O/ab_c3.log 2>&1 &&
python3 - "$O" <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/ab_c3.json"))
vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
print(d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs}, [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
