#!/usr/bin/env python3
"""bound_summary.py -- per-phase counters of tools/bound_probe.py runs under
rocprofv3 --pmc.  usage:
    python3 tools/bound_summary.py OUT.json PASSDIR[:PROBE.json] ...
Each PASSDIR holds one rocprofv3 pass (run_counter_collection.csv, found
recursively) of `bound_probe.py --launches N --out PROBE.json`; the probe's
"dispatches" list names every dispatch of k_rs_bs / k_rs_jitw in issue order,
so the n-th dispatch of a kernel belongs to a known phase.  Per phase: the
mean of each counter over the phase's dispatches (the first 3 dropped), the
effective clock GRBM_GUI_ACTIVE / 8 / duration (when the CSV has
timestamps), and SIMD-cycles per wave64 VALU = GRBM / 8 x 1024 / SQ_INSTS_VALU.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KEYS = {"k_rs_bs": "k_rs_bs(encode)", "k_rs_jitw": "k_rs_jit16(decode)"}


def kernel_of(name: str):
    for key, v in KEYS.items():
        if key in name:
            return v
    return None


def one_pass(passdir: str, probe: dict):
    rows = defaultdict(dict)
    meta = {}
    for f in glob.glob(os.path.join(passdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = kernel_of(r["Kernel_Name"])
            if kn is None:
                continue
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            ts = (r.get("Start_Timestamp"), r.get("End_Timestamp"))
            meta[d] = (kn, ts)
    order = defaultdict(list)
    for d in sorted(rows):
        order[meta[d][0]].append(d)
    out = defaultdict(lambda: defaultdict(list))
    pos = defaultdict(int)
    for kn, label, n in probe["dispatches"]:
        ids = order[kn][pos[kn]: pos[kn] + n]
        pos[kn] += n
        if label == "setup":
            continue
        for i, d in enumerate(ids):
            if i < 3:
                continue
            for c, v in rows[d].items():
                out[label][c].append(v)
            a, b = meta[d][1]
            if a and b:
                out[label]["_dur_ns"].append(float(b) - float(a))
    return out


def main():
    dst = sys.argv[1]
    merged = defaultdict(dict)
    for spec in sys.argv[2:]:
        passdir, _, probe_path = spec.partition(":")
        probe = json.load(open(probe_path or os.path.join(passdir, "probe.json")))
        for label, cs in one_pass(passdir, probe).items():
            for c, vs in cs.items():
                merged[label].setdefault(c, []).extend(vs)
    res = {}
    for label, cs in merged.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items() if v}
        r = {"dispatches": len(next(iter(cs.values()))), **{c: round(v, 1) for c, v in avg.items()}}
        g, valu = avg.get("GRBM_GUI_ACTIVE"), avg.get("SQ_INSTS_VALU")
        if g and valu:
            r["simd_cycles_per_valu"] = round(g / 8 * 1024 / valu, 3)
        if g and avg.get("_dur_ns"):
            r["clock_GHz_grbm"] = round(g / 8 / avg["_dur_ns"], 3)
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in avg:
                    r["frac_" + c] = round(avg[c] / wc, 3)
        res[label] = r
    json.dump(res, open(dst, "w"), indent=1)
    for label, r in res.items():
        print(label, json.dumps(r))


if __name__ == "__main__":
    main()
