"""Kernel timeline of the last MSM in a rocprofv3 kernel-trace CSV: per kernel start/duration and
the idle gap before it (us). usage: gap_report.py <kernel_trace.csv> [first_kernel_name]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_glv_split"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
seg = rows[starts[-2]:starts[-1]] if len(starts) >= 2 else rows[starts[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
prev_end = None
busy = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {r['Kernel_Name'][:70]}")
    prev_end = e
span = (prev_end - t0) / 1e3
print(f"span {span:.1f} us, kernels {busy / 1e3:.1f} us, gaps {span - busy / 1e3:.1f} us")
