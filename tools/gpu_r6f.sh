#!/bin/bash
# round 6: the solver configurations' launches -- per-env costs and per-stage cycles of CG
# and PGS, and the CG iteration profile against the oracle
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for sv in CG PGS; do
  timeout -k 10 300 python -u tools/cost_probe.py 4096 40 reorient $sv > gpurun_out/r6f_cost_$sv.log 2>&1 || { tail -5 gpurun_out/r6f_cost_$sv.log; exit 1; }
  echo "== cost $sv"; head -8 gpurun_out/r6f_cost_$sv.log | cut -c1-300
  timeout -k 10 300 python -u tools/stage_profile.py 4096 4 reorient $sv > gpurun_out/r6f_stages_$sv.log 2>&1 || { tail -5 gpurun_out/r6f_stages_$sv.log; exit 1; }
  echo "== stages $sv"; grep -E "ms/step|newton|np_mpr|top1|iterations" gpurun_out/r6f_stages_$sv.log | head -20 | cut -c1-250
done
timeout -k 10 400 python -u tools/cg_profile.py 4096 256 CG > gpurun_out/r6f_cg_profile.log 2>&1 || { tail -5 gpurun_out/r6f_cg_profile.log; exit 1; }
cut -c1-400 gpurun_out/r6f_cg_profile.log | head -20
