#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cg_profile.py 4096 64 PGS > gpurun_out/pgs_profile.log 2>&1 || { tail -5 gpurun_out/pgs_profile.log; exit 1; }
cat gpurun_out/pgs_profile.log | grep -v "^\[Newton"
bash tools/pmc_cfgs.sh pmc_r5h default "" nofuse "DX_NO_FUSE=1" nosep "DX_NO_SEPCACHE=1" noqueue "DX_NO_QUEUE=1" || exit 1
timeout -k 10 300 python -u tools/cost_probe.py 1024 200 reach_shadow > gpurun_out/cost_reach.log 2>&1 || { tail -5 gpurun_out/cost_reach.log; exit 1; }
cat gpurun_out/cost_reach.log
