"""Summarise tools/pmc_mix.sh output: median per-dispatch value of every counter for dx_step_kernel."""
import csv
import glob
import json
import os
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mix"
vals = {}
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for row in csv.DictReader(open(f)):
        if "dx_step_kernel" not in row.get("Kernel_Name", ""):
            continue
        key = (row["Counter_Name"], row.get("Dispatch_Id"))
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    for (name, _), v in per.items():
        vals.setdefault(name, []).append(v)
out = {k: statistics.median(v) for k, v in sorted(vals.items())}
print(json.dumps(out, indent=1))
