# Round 6: the (64, 32) compiled encode as two waves of 16 rows (187 VGPRs,
# 2 waves per SIMD) against four of 8, both with the wave priority; same-
# process ABBA at C3 and C4.   gpurun -- bash tools/r06_bs_wide.sh -> gpurun_out/r06_bs_wide/
set -o pipefail
O=gpurun_out/r06_bs_wide; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_wide --values=0,1 --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py -k "16_row_waves or priority_either" > $O/tests.log 2>&1 &&
ab c3 && ab c4 --symbol-size 32000 --blocks 16384 &&
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for c in ("c3", "c4"):
    d = json.load(open(f"{O}/ab_{c}.json"))
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"]) for v in ("0", "1")},
          d["1"].get("paired_delta_ms_vs_0"))
PY
