"""Print a rocprofv3 kernel_stats.csv as a short per-kernel table."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = r["Name"].replace("(anonymous namespace)::", "")[:60]
    print(f"{name:60s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.1f}us {float(r['TotalDurationNs']) / tot * 100:5.1f}%")
print(f"{tot / 1e6:.3f} ms total")
