# Round 6: the (64, 32) encode as the host-built generated program (16-row
# waves, hand-placed registers, 3 waves per SIMD) against the compiled
# k_rs_bs, both with the wave priority; same-process ABBA at C3 and C4.
#   gpurun -- bash tools/r06_enc_gen.sh -> gpurun_out/r06_enc_gen/
set -o pipefail
O=gpurun_out/r06_enc_gen; mkdir -p $O
export TMPDIR=/tmp
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob encode_kernel --values=compiled,generated --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
ab c3 && ab c4 --symbol-size 32000 --blocks 16384 &&
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for c in ("c3", "c4"):
    d = json.load(open(f"{O}/ab_{c}.json"))
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"]) for v in ("compiled", "generated")},
          d["generated"].get("paired_delta_ms_vs_compiled"))
PY
