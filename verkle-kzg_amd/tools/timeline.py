"""Last `count` kernels of a rocprofv3 kernel-trace CSV: start, duration and the idle gap before each
(us); with a memory-copy-trace CSV the copies inside that window are interleaved (marked "copy").
usage: timeline.py <kernel_trace.csv> [count] [memory_copy_trace.csv]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
count = int(sys.argv[2]) if len(sys.argv) > 2 else 30
seg = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80]) for r in rows[-count:]]
if len(sys.argv) > 3:
    t_lo = seg[0][0]
    for r in csv.DictReader(open(sys.argv[3])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t_lo:
            kind = r.get("Direction", r.get("Operation", "?"))
            seg.append((s, e, f"copy {kind} {r.get('Size', r.get('Bytes', '?'))} B"))
    seg.sort()
t0 = seg[0][0]
prev = None
busy = 0
for s, e, name in seg:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {name}")
    prev = max(prev or e, e)
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
