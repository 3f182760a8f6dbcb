"""SIMD-cycles per wave64 VALU instruction from ONE rocprofv3 --pmc pass that
holds GRBM_GUI_ACTIVE and SQ_INSTS_VALU (no wall clock): per dispatch,
(GRBM_GUI_ACTIVE / 8 XCDs) * 1024 SIMDs / SQ_INSTS_VALU.

usage: python3 tools/valu_ceiling.py RUN_counter_collection.csv [kernel-substring ...]
Prints one JSON object per kernel (the longest dispatch of each)."""
import csv
import json
import sys
from collections import defaultdict

SIMDS, XCDS = 1024, 8


def per_dispatch(path):
    d = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    return d, names


def main():
    d, names = per_dispatch(sys.argv[1])
    want = sys.argv[2:]
    best = {}
    for disp, c in d.items():
        n = names[disp]
        if want and not any(w in n for w in want):
            continue
        if "SQ_INSTS_VALU" not in c or "GRBM_GUI_ACTIVE" not in c or c["SQ_INSTS_VALU"] <= 0:
            continue
        key = n.split("(")[0][-60:]
        if key not in best or c["GRBM_GUI_ACTIVE"] > best[key]["GRBM_GUI_ACTIVE"]:
            best[key] = dict(c)
    for key, c in best.items():
        cpi = c["GRBM_GUI_ACTIVE"] / XCDS * SIMDS / c["SQ_INSTS_VALU"]
        out = {"kernel": key, "simd_cycles_per_valu": round(cpi, 4),
               "frac_of_2cycle_issue": round(2.0 / cpi, 4), **{k: v for k, v in c.items()}}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
