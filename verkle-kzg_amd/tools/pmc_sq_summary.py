"""Per-kernel averages of SQ counters from a rocprofv3 --pmc run (counter_collection.csv): VALU
instructions and wave lifetime split into issuing (ACTIVE_INST_ANY), parked on s_waitcnt /
barriers (WAIT_ANY) and issue-stalled (WAIT_INST_ANY), per wave, in quad-cycles.
usage: pmc_sq_summary.py run_counter_collection.csv [name-substring ...]"""
import collections
import csv
import sys

path, subs = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.Counter()
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if subs and not any(s in name for s in subs):
        continue
    key = name.split("<")[0].replace("void ", "")
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES":
        launches[key] += 1
print(f"{'kernel':28s} {'launches':>8s} {'waves':>8s} {'VALU/wave':>10s} {'cyc/wave':>9s} "
      f"{'active':>7s} {'wait':>7s} {'stall':>7s}")
for k, d in agg.items():
    n, w = launches[k], d["SQ_WAVES"]
    if not n or not w:
        continue
    cyc = d["SQ_WAVE_CYCLES"]
    print(f"{k:28s} {n:8d} {w / n:8.0f} {d['SQ_INSTS_VALU'] / w:10.0f} {cyc / w:9.0f} "
          f"{d['SQ_ACTIVE_INST_ANY'] / cyc:7.2f} {d['SQ_WAIT_ANY'] / cyc:7.2f} {d['SQ_WAIT_INST_ANY'] / cyc:7.2f}")
