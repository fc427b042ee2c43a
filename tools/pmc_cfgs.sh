#!/bin/bash
# On the GPU box: FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 runs) of a short
# bench run per configuration, and the step kernel's HBM traffic per launch
# (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction):
#   tools/pmc_cfgs.sh OUTNAME name1 "VAR=VAL ..." name2 "" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1; shift
rm -rf "$O"; mkdir -p "$O"
names=()
cd /tmp && export TMPDIR=/tmp
while [ $# -gt 0 ]; do
  name=$1; vars=$2; shift 2; names+=("$name")
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env $vars timeout -k 10 240 rocprofv3 --pmc "$ctr" --kernel-trace -d "$O/$name/$ctr" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > "$O/$name.$ctr.log" 2>&1
    rc=$?; echo "$name $ctr rc=$rc"; [ $rc = 0 ] || exit $rc
  done
done
cd "$R" && python3 - "$O" "${names[@]}" <<'PY'
import csv, glob, os, statistics, sys
root = sys.argv[1]
for name in sys.argv[2:]:
    out = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        per = {}
        for f in glob.glob(os.path.join(root, name, ctr, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "dx_step_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") == ctr:
                    per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
        out[ctr] = statistics.median(per.values()) if per else float("nan")  # KB per dispatch
    tot = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) / 1024
    print(f"{name:8s} FETCH_SIZE {out['FETCH_SIZE'] / 1024:8.1f} MB  WRITE_SIZE {out['WRITE_SIZE'] / 1024:8.1f} MB  "
          f"HBM per launch (2 x fetch + write) {tot:8.1f} MB")
PY
