"""Median FETCH_SIZE / WRITE_SIZE (KB) per dx_step_kernel dispatch for each
configuration of tools/pmc_ab.sh (gpurun_out/pmc_ab)."""
import csv
import glob
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
base = os.path.join(ROOT, "gpurun_out", "pmc_ab")
for cfg in sorted(os.listdir(base)):
    d = os.path.join(base, cfg)
    if not os.path.isdir(d):
        continue
    out = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        per = {}  # dispatch -> sum over the counter's instances
        for f in glob.glob(os.path.join(d, ctr, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "dx_step_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
        vals = list(per.values())
        out[ctr] = statistics.median(vals) if vals else None
    fs, ws = out["FETCH_SIZE"], out["WRITE_SIZE"]
    tot = (2 * fs + ws) * 1024 if fs is not None and ws is not None else None
    print(f"{cfg}: FETCH_SIZE {fs} KB, WRITE_SIZE {ws} KB, HBM bytes/launch {tot}")
