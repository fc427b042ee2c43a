#!/bin/bash
# Same-box A/B of one environment switch: the reorient bench with and without "$@"
# (e.g. DX_DENSE_MSOLVE=1), round robin, twice each, then a stage profile of the switch.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_base_$i.log 2>&1
  env "$@" timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/ab_var_$i.log 2>&1
done
env "$@" timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > gpurun_out/ab_var_stages.log 2>&1
for f in gpurun_out/ab_base_*.log gpurun_out/ab_var_*.log; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$f" || true
done
