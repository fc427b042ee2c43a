#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stage_profile.py 4096 4 bimanual > gpurun_out/r6_stages_bimanual.log 2>&1 || { tail -5 gpurun_out/r6_stages_bimanual.log; exit 1; }
head -40 gpurun_out/r6_stages_bimanual.log | cut -c1-220
