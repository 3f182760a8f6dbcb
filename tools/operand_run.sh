# Does the multiply-accumulates' operand toggling cost energy?  Diagnostic
# variants 11 (the low-nibble composite operand fixed) and 12 (both composite
# operands fixed) of the generated decode against the diagnostic product
# build, each in its own process, one box, C3 (tools/bound_probe.py; timing
# only -- the variants' outputs are wrong).  Build first:
#   for v in "" 11 12; do make -C storage-benchmarks_amd diag DIAG_VARIANT=$v; done
#   bash tools/operand_run.sh TAG -> gpurun_out/operand_TAG/
set -o pipefail
O=gpurun_out/operand_${1:-x}; mkdir -p $O
D=tools/diag
run() {
    RSGPU_LIB=$2 timeout -k 10 120 python3 -u tools/bound_probe.py --seconds 2 --order dec:rand,enc:rand,dec:rand \
        --out $O/$1.json > $O/$1.log 2>&1 && python3 - "$O/$1.json" "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], [(p["phase"], p["median_ms"], p.get("clock_MHz_median")) for p in d["phases"]])
PY
}
run p1 $D/librsgpu_diag.so && run v11 $D/librsgpu_diag_v11.so && run v12 $D/librsgpu_diag_v12.so && \
run p2 $D/librsgpu_diag.so && run v11b $D/librsgpu_diag_v11.so
