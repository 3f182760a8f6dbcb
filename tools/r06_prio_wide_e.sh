# Round 6: the wave priority in the wide layouts (e > 16: J12, four waves, passes above 64 rows)
# same process, ABBA x6,
# both knobs on (the default) vs both off.   gpurun -- bash tools/r06_prio_wide_e.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_prio_wide_e}; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_prio+rsgpu_internal_set_jitw_prio --values=2+2,0+0 --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
ab k100e50 --symbols 100 --erased 50 --blocks 635 &&
ab k150e100 --symbols 150 --erased 100 --blocks 400 &&
ab k48e24 --symbols 48 --erased 24 --blocks 1315 &&
ab k100e25 --symbols 100 --erased 25 --blocks 635 &&
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(f.split("/")[-1], d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs},
          [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
