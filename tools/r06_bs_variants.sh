# Round 6: the encode's priority instantiations (0 none, 1 s_setprio, 3 the
# same padded to 8 bytes with s_nop) -- same-process ABBA x8 at C3 and C4,
# and one counter pass for their instruction-cache misses.
#   gpurun -- bash tools/r06_bs_variants.sh NAME
set -o pipefail
O=gpurun_out/${1:-r06_bs_variants}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_prio --values=1,0,3 --reps 8 --out $O/ab_c3.json > $O/ab_c3.log 2>&1 &&
timeout -k 10 300 python3 -u tools/ab_knob.py --knob rsgpu_internal_set_bs_prio --values=1,0,3 --reps 6 --symbol-size 32000 --blocks 16384 --out $O/ab_c4.json > $O/ab_c4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 tools/bs_prio_icache.py > $O/pmc.log 2>&1 &&
python3 - "$O" <<'PY'
import csv, json, sys, glob, collections
O = sys.argv[1]
for c in ("c3", "c4"):
    d = json.load(open(f"{O}/ab_{c}.json"))
    vs = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(c, d["verified"], {v: (d[v]["step_ms_median"], d[v]["kernels_ms_median"].get("k_rs_bs(encode)")) for v in vs}, [d[v].get("paired_delta_ms_vs_" + vs[0]) for v in vs[1:]])
f = glob.glob(f"{O}/pmc/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "k_rs_bs" in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
