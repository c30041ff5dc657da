"""Mean SQ counters per dispatch for kernels matching a substring: pmc_sq.py DIR SUBSTR"""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
acc = defaultdict(list)
for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(m):
    print(f"{k:28s} {m[k]:16.1f}")
w = m.get("SQ_WAVES", 0)
if w:
    print("per wave:")
    for k in ("SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU",
              "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
              "SQ_WAIT_INST_ANY"):
        if k in m:
            print(f"  {k:26s} {m[k] / w:12.1f}")
