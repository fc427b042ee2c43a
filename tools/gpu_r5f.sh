#!/bin/bash
# round 5: the queued step as a kernel of its own (instruction footprint): parity, A/B
# against the round-start tree, instruction-fetch stall counters of both
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
rc=$?
if [ $rc != 0 ]; then
  echo "suite rc=$rc"; grep -E "^FAILED|Error" gpurun_out/t_all.log | head -20; tail -3 gpurun_out/t_all.log
  [ $rc = 1 ] || exit $rc
fi
tail -1 gpurun_out/t_all.log
bash tools/ab_multi.sh 3 new "" prev "DX_LIB=variants/prev/libdx.so" || exit 1
R=$(pwd); O=$R/gpurun_out/icache; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in new prev; do
  lib=""; [ $v = prev ] && lib="DX_LIB=$R/variants/prev/libdx.so"
  env $lib timeout -k 10 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY --kernel-trace -d $O/$v -o pmc --output-format csv -- \
    python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-api-steps 0 > $O/$v.log 2>&1 || exit 1
done
cd $R && python3 - <<'PY'
import csv, glob, statistics
for v in ("new", "prev"):
    agg = {}
    for f in glob.glob(f"gpurun_out/icache/{v}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "dx_step_kernel" in row["Kernel_Name"]:
                agg.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                agg[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    med = {k: statistics.median(d.values()) for k, d in agg.items()}
    print(v, {k: f"{x:.3e}" for k, x in sorted(med.items())},
          "WAIT_INST_ANY/WAVE_CYCLES", round(med["SQ_WAIT_INST_ANY"] / med["SQ_WAVE_CYCLES"], 4))
PY
