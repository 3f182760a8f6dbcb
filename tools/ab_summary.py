#!/usr/bin/env python3
"""ab_summary.py -- one line per tools/ab_knob.py JSON: the knob values with
their median step and kernel times, and the paired step differences.
usage: python3 tools/ab_summary.py FILE.json ..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    vals = [k for k in d if isinstance(d[k], dict) and "step_ms_median" in d[k]]
    print(f, "verified" if d.get("verified") else "NOT VERIFIED")
    for v in vals:
        pd = {k: x for k, x in d[v].items() if k.startswith("paired")}
        print("  ", v, d[v]["step_ms_median"], d[v]["kernels_ms_median"], pd or "")
