# Round 6: re-check layout knobs with the wave priority on (same process,
# ABBA x6 each): the rotation period, tiles per decode workgroup (C3, C4).
# (The same run measured the instruction-cache invalidation per workgroup /
# none / once per CU per launch at C3 and C4: all within noise; that code is
# gone, profiles/r06_knobs/ab_*noinv.json.)
#   gpurun -- bash tools/r06_c3_knobs.sh NAME -> gpurun_out/NAME/
set -o pipefail
O=gpurun_out/${1:-r06_c3_knobs}; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob $2 --values=$3 --reps 6 --out $O/ab_$1.json "${@:4}" > $O/ab_$1.log 2>&1; }
ab rot rsgpu_internal_set_jitw_rot 600,450,800 &&
ab tiles rsgpu_internal_set_jitw_tiles 2,1 &&
ab c4rot rsgpu_internal_set_jitw_rot -1,342 --symbol-size 32000 --blocks 16384 &&
ab c4tiles rsgpu_internal_set_jitw_tiles 2,1 --symbol-size 32000 --blocks 16384 &&
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(f.split("/")[-1], d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs},
          [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
