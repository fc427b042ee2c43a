#!/bin/bash
# round 6 close on HEAD: suite, smoke, bench, rocprof + PMC + stages (gpu_r6z.sh), then
# every configuration and the solver configurations' per-env costs
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=r6f bash tools/gpu_r6z.sh || exit 1
timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/r6f_configs.log 2>&1 || { tail -5 gpurun_out/r6f_configs.log; exit 1; }
cut -c1-200 gpurun_out/r6f_configs.log
for sv in CG PGS; do
  timeout -k 10 300 python -u tools/cost_probe.py 4096 40 reorient $sv > gpurun_out/r6f_cost_$sv.log 2>&1 || { tail -5 gpurun_out/r6f_cost_$sv.log; exit 1; }
  echo "== cost $sv"; grep -E "per-step max|slot util" gpurun_out/r6f_cost_$sv.log | cut -c1-200
done
