"""Last `count` kernels of a rocprofv3 kernel-trace CSV: start, duration and the idle gap before each
(us). usage: timeline.py <kernel_trace.csv> [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
count = int(sys.argv[2]) if len(sys.argv) > 2 else 30
seg = rows[-count:]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
busy = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {r['Kernel_Name'][:80]}")
    prev = max(prev or e, e)
print(f"span {(prev - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us")
