# Round 6: lane-held row pointers in k_rs_jitw (no scalar loads in the
# chunk loop).  The GPU suite at this build, then same-process ABBA x6 of
# the knob at C3, C4 (one 16384-block batch, four pipelined slices) and C5.
#   gpurun -- bash tools/r06_lp.sh   -> gpurun_out/r06_lp/
set -o pipefail
O=gpurun_out/r06_lp; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_jitw_lane_ptrs --values 0,1 --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
ab c3 && ab c4 --symbol-size 32000 --blocks 16384 && ab c5 --symbols 100 --erased 20 --blocks 512 &&
python3 - <<'PY'
import json
for c in ("c3", "c4", "c5"):
    d = json.load(open(f"gpurun_out/r06_lp/ab_{c}.json"))
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"]) for v in ("0", "1")},
          d["1"]["paired_delta_ms_vs_0"])
PY
