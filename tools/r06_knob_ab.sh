# Round 6: same-process ABBA x REPS of one librsgpu_testhooks knob at C3, C4
# (one 16384-block batch, four pipelined slices) and C5.
#   gpurun -- bash tools/r06_knob_ab.sh NAME KNOB VALUES [REPS]  -> gpurun_out/NAME/
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
K=$2; V=$3; R=${4:-6}
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob $K --values $V --reps $R --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
ab c3 && ab c4 --symbol-size 32000 --blocks 16384 && ab c5 --symbols 100 --erased 20 --blocks 512 &&
python3 - "$O" "$V" <<'PY'
import json, sys
O, V = sys.argv[1], sys.argv[2].split(",")
for c in ("c3", "c4", "c5"):
    d = json.load(open(f"{O}/ab_{c}.json"))
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"]) for v in V},
          [d[v].get("paired_delta_ms_vs_" + V[0]) for v in V[1:]])
PY
