"""One line per kernel from a rocprofv3 --kernel-trace --stats CSV
(run_kernel_stats.csv): calls, average ms, share of kernel time.
usage: python3 tools/kernel_stats_summary.py run_kernel_stats.csv "header line" """
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2] if len(sys.argv) > 2 else sys.argv[1])
for r in rows:
    name = r["Name"].replace('"', "")[:60]
    print(f"{name:60s} calls={int(r['Calls']):3d} avg_ms={float(r['AverageNs']) / 1e6:9.3f} "
          f"pct={float(r['Percentage']):6.2f}")
