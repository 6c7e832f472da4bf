"""Timeline of one converge from a rocprofv3 kernel_trace.csv: every dispatch
between the N-th and (N+1)-th occurrence of a marker kernel, with gaps."""
import csv
import sys

path, marker = sys.argv[1], sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else -2
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a = idx[nth]
b = idx[nth + 1] if nth + 1 < len(idx) and nth != -1 else len(rows)
prev_end = None
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:50]
    print(f"{(s - t0) / 1e3:9.1f}us  +gap {gap:7.1f}  dur {(e - s) / 1e3:8.1f}  {name}")
    prev_end = e
print(f"span {(prev_end - t0) / 1e3:.1f} us")
if b < len(rows):
    print(f"next {marker} at {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us (call period)")
