"""Summarises gpurun_out/prof (tools/profile_round.sh) into profiles/<tag>_*.

usage: python tools/summarize_profiles.py <tag>    e.g. r1
Writes:
  profiles/<tag>_kernel_stats.csv / .md   rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_hbm.csv              per-dispatch FETCH_SIZE / WRITE_SIZE of dx_step_kernel
  profiles/pmc_step_kernel.json           HBM bytes per dx_step_kernel launch (read by bench.py)
  profiles/<tag>_stages.json / .log       per-stage cycle profile
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "prof")
DST = os.path.join(ROOT, "profiles")
tag = sys.argv[1] if len(sys.argv) > 1 else "r1"


def one(pattern):
    hits = glob.glob(os.path.join(SRC, pattern), recursive=True)
    if not hits:
        raise SystemExit(f"missing {pattern} under {SRC}")
    return hits[0]


stats = one("trace/**/run_kernel_stats.csv")
shutil.copy(stats, os.path.join(DST, f"{tag}_kernel_stats.csv"))
rows = list(csv.DictReader(open(stats)))
with open(os.path.join(DST, f"{tag}_kernel_stats.md"), "w") as f:
    f.write(f"# rocprofv3 --kernel-trace --stats ({tag}): python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline\n\n")
    f.write("| kernel | calls | total ms | avg ms | min ms | max ms | % |\n|---|---|---|---|---|---|---|\n")
    for r in rows:
        f.write(f"| {r['Name'][:60]} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                f"{float(r['AverageNs'])/1e6:.4f} | {float(r['MinNs'])/1e6:.4f} | {float(r['MaxNs'])/1e6:.4f} | "
                f"{float(r['Percentage']):.2f} |\n")
    # the bench's timed region: the last 40 step-kernel dispatches (warmup and reset
    # launches excluded), the launches bench.py's HIP-event mean covers
    tr = [r for r in csv.DictReader(open(one("trace/**/run_kernel_trace.csv"))) if "dx_step_kernel" in r["Kernel_Name"]]
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr[-40:]]
    if last:
        f.write(f"\nStep kernel over the timed region (last {len(last)} dispatches): mean {statistics.mean(last):.4f} ms, "
                f"min {min(last):.4f}, max {max(last):.4f}\n")


def pmc(kind, counter):
    path = one(f"{kind}/**/pmc_counter_collection.csv")
    per = {}
    for r in csv.DictReader(open(path)):
        if "dx_step_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return per


fetch = pmc("fetch", "FETCH_SIZE")
write = pmc("write", "WRITE_SIZE")
with open(os.path.join(DST, f"{tag}_pmc_hbm.csv"), "w") as f:
    f.write("pass,dispatch,counter,kilobytes\n")
    for d, v in sorted(fetch.items(), key=lambda x: int(x[0])):
        f.write(f"fetch,{d},FETCH_SIZE,{v}\n")
    for d, v in sorted(write.items(), key=lambda x: int(x[0])):
        f.write(f"write,{d},WRITE_SIZE,{v}\n")
# steady state: drop the first (cold) dispatches
f_kb = statistics.median(sorted(fetch.values())[: max(1, len(fetch))])
w_kb = statistics.median(write.values())
hbm = 2 * f_kb * 1024 + w_kb * 1024  # gfx950: FETCH_SIZE reports half the read bytes (MI355X_MICROARCH.md)
json.dump({
    "envs": 4096,
    "hbm_bytes_per_launch": round(hbm),
    "fetch_size_kb_median": f_kb,
    "write_size_kb_median": w_kb,
    "correction": "read bytes = 2 x FETCH_SIZE (gfx950), write bytes = WRITE_SIZE; separate PMC passes",
    "source": f"profiles/{tag}_pmc_hbm.csv",
    # the measured library's source hash (dx_build_key): bench.py reports these bytes as
    # roofline.traffic only when it runs that same build, else traffic is null
    "build_key": open(os.path.join(SRC, "build_key.txt")).read().strip()
    if os.path.exists(os.path.join(SRC, "build_key.txt")) else None,
}, open(os.path.join(DST, "pmc_step_kernel.json"), "w"), indent=1)
for ext in ("json", "log"):
    p = os.path.join(SRC, f"stages.{ext}")
    if os.path.exists(p):
        shutil.copy(p, os.path.join(DST, f"{tag}_stages.{ext}"))
print("hbm bytes per launch", hbm, "per env-step", hbm / 4096)
