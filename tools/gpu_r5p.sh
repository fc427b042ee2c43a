#!/bin/bash
# round 5: per-env cost distribution of the PGS / CG / Newton reorient launches
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for s in PGS CG; do
  timeout -k 10 300 python3 tools/cost_probe.py 4096 40 reorient $s > gpurun_out/cost_$s.log 2>&1 || { tail -5 gpurun_out/cost_$s.log; exit 1; }
  echo "== $s"; grep -v amdgpu.ids gpurun_out/cost_$s.log
done
timeout -k 10 300 python3 tools/cost_probe.py 4096 40 reorient > gpurun_out/cost_newton.log 2>&1 || { tail -5 gpurun_out/cost_newton.log; exit 1; }
echo "== Newton"; grep -v amdgpu.ids gpurun_out/cost_newton.log
