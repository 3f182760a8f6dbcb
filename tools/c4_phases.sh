# Phases of the generated decode (diagnostic variant 6, per-wave s_memtime
# sums) at C4's row length (L 32000, 4096 blocks) and at C3, one box:
#   make -C storage-benchmarks_amd diag DIAG_VARIANT=6 ; bash tools/c4_phases.sh
set -o pipefail
O=gpurun_out/c4ph; mkdir -p $O
L=tools/diag/librsgpu_diag_v6.so
RSGPU_LIB=$L timeout -k 10 120 python3 -u tools/bound_probe.py --symbol-size 32000 --blocks 4096 --seconds 1.5 \
    --order enc:rand,dec:rand --out $O/v6_c4.json > $O/v6_c4.log 2>&1 && \
RSGPU_LIB=$L timeout -k 10 120 python3 -u tools/bound_probe.py --seconds 1.5 --order enc:rand,dec:rand \
    --out $O/v6_c3.json > $O/v6_c3.log 2>&1 && \
python3 - <<'PY'
import json
for f in ("c4", "c3"):
    d = json.load(open("gpurun_out/c4ph/v6_%s.json" % f))
    for p in d["phases"]:
        if "phase_frac" in p:
            print(f, p["median_ms"], p["phase_cycles_per_wave"], p["phase_frac"])
PY
