#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > gpurun_out/stages_r5m.log 2>&1 || { tail -5 gpurun_out/stages_r5m.log; exit 1; }
head -22 gpurun_out/stages_r5m.log
