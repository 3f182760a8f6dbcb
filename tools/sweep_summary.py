#!/usr/bin/env python3
"""sweep_summary.py -- one line per bench log of tools/geom_sweep.sh:
k, e, blocks, goodput GiB/s and the apply kernels' average ms.
usage: python3 tools/sweep_summary.py gpurun_out/sweep_TAG"""
import glob
import json
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            if d.get("value") is None:  # a failed run's line (e.g. k + e > 250)
                print("failed:", os.path.basename(f), d.get("error", {}).get("first", {}).get("error"))
                continue
            c = d["config"]
            ks = {k: v["avg_ms"] for k, v in d["kernels"].items() if "emit" not in k and "prepare" not in k}
            rows.append((c["symbols"], c["erased"], c["blocks_per_gpu"], d["value"], ks))
for r in sorted(rows):
    print(*r)
