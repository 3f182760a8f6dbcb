# Round 6: C4 (one 16384-block batch, four pipelined slices) decode knobs with
# the wave priority on, same process, ABBA x6 each: code prefetch, rotation,
# tiles per workgroup.   gpurun -- bash tools/r06_c4_knobs.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_c4_knobs}; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob $2 --values=$3 --reps 6 --symbol-size 32000 --blocks 16384 --out $O/ab_$1.json > $O/ab_$1.log 2>&1; }
ab prefetch rsgpu_internal_set_jitw_prefetch -1,0 &&
ab rot rsgpu_internal_set_jitw_rot -1,600,300 &&
ab tiles rsgpu_internal_set_jitw_tiles 2,1 &&
ab pipe rsgpu_internal_set_decode_pipeline -1,1,8 &&
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(f.split("/")[-1], d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs},
          [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
