# Round 6: SQ counters of the C3 kernels with the wave priority off and on
# (one counter pass each; tools/ab_knob.py with one configuration, 1 rep).
#   gpurun -- bash tools/r06_prio_counters.sh NAME
set -o pipefail
O=$(pwd)/gpurun_out/${1:-r06_prio_counters}; mkdir -p $O
export TMPDIR=/tmp
K=rsgpu_internal_set_bs_prio+rsgpu_internal_set_jitw_prio
for v in 0+0 2+2; do
  n=${v/+/_}
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p_$n -o run --output-format csv -- python3 tools/ab_knob.py --knob $K --values=$v --reps 1 --steps 2 --warmup 1 > $O/p_$n.log 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for n in ("0_0", "2_2"):
    f = glob.glob(f"{O}/p_{n}/**/run_counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_rs_bs<64" in k or "k_rs_jitw" in k:
            agg[k[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m["SQ_WAVES"]
        print(n, k, {c: round(x / w) for c, x in m.items() if c.startswith("SQ_") and c != "SQ_WAVES"},
              "GRBM", round(m["GRBM_GUI_ACTIVE"]), "valu/simd-cycle", round(m["SQ_INSTS_VALU"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024), 4))
PY
