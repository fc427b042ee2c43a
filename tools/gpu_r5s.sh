#!/bin/bash
# round 5: CG per-stage profile (heaviest envs)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/stage_profile.py 4096 8 reorient CG > gpurun_out/stages_cg.log 2>&1 || { tail -5 gpurun_out/stages_cg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stages_cg.log | head -80
