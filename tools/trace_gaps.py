"""Kernel durations and the idle gaps between consecutive kernels of a
rocprofv3 --kernel-trace CSV (a tool): for each kernel name, the median
duration and the median gap from the previous kernel's end to its start
(same queue), over the last 80 % of the dispatches (the timed steps).
usage: python3 tools/trace_gaps.py run_kernel_trace.csv"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 5:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][-48:]
    dur[name].append(e - s)
    if prev_end is not None:
        gap[name].append(s - prev_end)
    prev_end = e
for name in dur:
    g = gap.get(name, [0])
    print(f"{name:48s} n={len(dur[name]):5d} dur_med_us={statistics.median(dur[name]) / 1e3:8.2f} "
          f"gap_before_med_us={statistics.median(g) / 1e3:8.2f} gap_p90_us={sorted(g)[int(len(g) * 0.9)] / 1e3:8.2f}")
