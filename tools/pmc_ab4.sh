#!/bin/bash
# On the GPU box: FETCH_SIZE and WRITE_SIZE passes of a short bench run under several
# configurations (default, no substep queue, unfused task logic, the round-3 cache
# logic), for the HBM-traffic attribution in DESIGN.md.  Output under
# gpurun_out/pmc_ab4/<config>/{FETCH_SIZE,WRITE_SIZE}; stops at the first failed pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_ab4
rm -rf "$O"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <counter> [ENV=VALUE ...]
  name=$1; ctr=$2; shift 2
  env "$@" timeout -k 10 240 rocprofv3 --pmc "$ctr" --kernel-trace -d "$O/$name/$ctr" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --host-api-steps 0 > "$O/$name.$ctr.log" 2>&1
  rc=$?; echo "$name $ctr rc=$rc"; return $rc
}
for cfg in "default" "noqueue DX_NO_QUEUE=1" "nofuse DX_NO_FUSE=1"; do
  set -- $cfg
  name=$1; shift
  run "$name" FETCH_SIZE "$@" || exit 1
  run "$name" WRITE_SIZE "$@" || exit 1
done
cd "$R" && python3 - <<'PY'
import csv, glob, os, statistics
root = "gpurun_out/pmc_ab4"
for name in ("default", "noqueue", "nofuse"):
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
