"""Print the top kernels of a rocprofv3 kernel_stats.csv (percent, calls, average us)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}% calls={r['Calls']:>5} avg={float(r['AverageNs'])/1000:8.1f}us  {r['Name'][:100]}")
print(f"total {tot/1e6:.3f} ms")
