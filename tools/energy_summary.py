#!/usr/bin/env python3
"""energy_summary.py -- table of tools/energy_run.sh: per variant and kernel
the median launch time (ms, median over the variant's phases) and the
in-kernel clock (MHz, median over stamped workgroups, then over phases).
usage: python3 tools/energy_summary.py DIR  (reads DIR/*.json)"""
import glob
import json
import os
import statistics
import sys

ORDER = ["p1", "v1_hbmq", "v2_zplane", "v3_valuq", "v4_nowait", "v5_notr", "p2", "product"]
WHAT = {
    "p1": "diagnostic product build",
    "v1_hbmq": "HBM I/O quiet (2-block x 16 KB window in L2)",
    "v2_zplane": "zero planes written by the transposes (LDS planes, VALU, stores quiet)",
    "v3_valuq": "LDS plane reads kept, VALU on zero planes",
    "v4_nowait": "no per-source LDS wait in the generated decode",
    "v5_notr": "no source transposes",
    "p2": "diagnostic product build again (drift)",
    "product": "product library (no stamps; times only)",
}


def main(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "*.json")):
        name = os.path.basename(f)[:-5]
        rows[name] = json.load(open(f))
    print("| variant | what | kernel | data | ms (median) | clock MHz |")
    print("|---|---|---|---|---|---|")
    for name in ORDER + sorted(set(rows) - set(ORDER)):
        if name not in rows:
            continue
        by = {}
        for ph in rows[name]["phases"]:
            kind, data = ph["phase"].split(":")
            by.setdefault((ph["kernel"], data), []).append(ph)
        for (kern, data), phs in sorted(by.items()):
            ms = statistics.median(p["median_ms"] for p in phs)
            clk = [p["clock_MHz_median"] for p in phs if "clock_MHz_median" in p]
            c = f"{statistics.median(clk):.0f}" if clk else "-"
            print(f"| {name} | {WHAT.get(name, '')} | {kern} | {data} | {ms:.3f} | {c} |")


if __name__ == "__main__":
    main(sys.argv[1])
