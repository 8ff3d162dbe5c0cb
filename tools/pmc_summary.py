"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/*) per kernel: mean per dispatch."""
import csv
import collections
import json
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(os.listdir(base)):
    f = os.path.join(base, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = "jpeg_rgba" if "jpeg_rgba" in name else "png_unfilter" if "png_unfilter" in name else None
        if not short:
            continue
        acc[short][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
out = {}
for k, d in acc.items():
    per = collections.defaultdict(list)
    for (cn, disp), vals in d.items():
        per[cn].append(sum(vals))
    out[k] = {cn: sum(v) / len(v) for cn, v in per.items()}
print(json.dumps(out, indent=1))
