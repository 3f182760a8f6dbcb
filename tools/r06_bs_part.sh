# Round 6: sources per LDS part of the one- and two-wave compiled encodes
# (8: 32 KB of double buffer per workgroup, 1.25 waves per SIMD for one-wave
# workgroups; 4; 2), parity first, then same-process ABBA per geometry.
#   gpurun -- bash tools/r06_bs_part.sh -> gpurun_out/r06_bs_part/
set -o pipefail
O=gpurun_out/r06_bs_part; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py -k "lds_part_sizes" > $O/tests.log 2>&1 &&
ab() { timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_part --values=8,4,2 --reps 6 --out $O/ab_$1.json "${@:2}" > $O/ab_$1.log 2>&1; }
ab k16e4 --symbols 16 --erased 4 --blocks 2048 && ab k16e8 --symbols 16 --erased 8 --blocks 2048 &&
ab k64e16 --symbols 64 --erased 16 --blocks 989 && ab k20e7 --symbols 20 --erased 7 --blocks 1500 &&
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for c in ("k16e4", "k16e8", "k64e16", "k20e7"):
    d = json.load(open(f"{O}/ab_{c}.json"))
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"]) for v in ("8", "4", "2")},
          [d[v].get("paired_delta_ms_vs_8") for v in ("4", "2")])
PY
