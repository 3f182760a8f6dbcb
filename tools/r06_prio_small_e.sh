# Round 6: the wave priority in the 8-row generated decode (k_rs_jit, e <= 16)
# and the compiled encodes of (16, 4) / (64, 16), same process, ABBA x6,
# both knobs on (the default) vs both off.   gpurun -- bash tools/r06_prio_small_e.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_prio_small_e}; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_prio+rsgpu_internal_set_jitw_prio --values=2+2,0+0 --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
ab k32e8 --symbols 32 --erased 8 --blocks 1959 &&
ab k64e16 --symbols 64 --erased 16 --blocks 989 &&
ab k16e4 --symbols 16 --erased 4 --blocks 2048 &&
ab k8e2 --symbols 8 --erased 2 --blocks 2048 &&
python3 - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    d = json.load(open(f))
    vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(f.split("/")[-1], d["verified"], {v: (d[v]["step_ms_median"], {k: x for k, x in d[v]["kernels_ms_median"].items() if "rs_" in k}) for v in vs},
          [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
PY
