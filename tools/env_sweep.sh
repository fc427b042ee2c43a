#!/bin/bash
# Same-box sweep of environment settings on the headline bench: each argument is a
# space-separated list of VAR=VALUE assignments ("-" = none), run round robin, twice.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for i in 1 2; do
  k=0
  for a in "$@"; do
    k=$((k + 1))
    if [ "$a" = "-" ]; then envs=(); else read -ra envs <<< "$a"; fi
    env "${envs[@]}" timeout -k 10 120 python -u bench.py --no-cpu-baseline --host-api-steps 0 --steps 300 > gpurun_out/sw_${k}_$i.log 2>&1 || exit 1
    echo "$i [$a] $(grep -o '"value": [0-9.]*' gpurun_out/sw_${k}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_${k}_$i.log)"
  done
done
