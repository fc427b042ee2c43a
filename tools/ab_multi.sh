#!/bin/bash
# Same-box A/B of several environment settings of the reorient bench, round robin:
#   tools/ab_multi.sh ROUNDS base "" last "DX_ORDER_LAST=1" ...
# (name, space-separated VAR=VALUE list) pairs; prints value and ms/step per run.
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out
names=(); envs=()
while [ $# -gt 0 ]; do names+=("$1"); envs+=("$2"); shift 2; done
for r in $(seq 1 "$rounds"); do
  for i in "${!names[@]}"; do
    log=gpurun_out/ab_${names[$i]}_$r.log
    env ${envs[$i]} timeout -k 10 150 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > "$log" 2>&1
    rc=$?
    case $rc in 0) ;; *) echo "${names[$i]} round $r rc=$rc"; exit $rc;; esac
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])" "$log" "${names[$i]}" "$r"
  done
done
