#!/bin/bash
# Same-box sweep of environment settings on one tools/bench_configs.py configuration:
#   bash tools/env_sweep_cfg.sh CONFIG "VAR=V ..." "-" ...   ("-" = none), round robin, twice
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
cfg=$1; shift
for i in 1 2; do
  k=0
  for a in "$@"; do
    k=$((k + 1))
    if [ "$a" = "-" ]; then envs=(); else read -ra envs <<< "$a"; fi
    env "${envs[@]}" timeout -k 10 200 python -u tools/bench_configs.py "$cfg" > gpurun_out/swc_${k}_$i.log 2>&1 || { tail -3 gpurun_out/swc_${k}_$i.log; exit 1; }
    echo "$i [$a] $(grep -o '"env_steps_per_s": [0-9.]*' gpurun_out/swc_${k}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/swc_${k}_$i.log)"
  done
done
