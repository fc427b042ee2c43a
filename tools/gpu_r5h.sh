#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cg_profile.py 4096 64 PGS > gpurun_out/pgs_profile.log 2>&1 || { tail -5 gpurun_out/pgs_profile.log; exit 1; }
cat gpurun_out/pgs_profile.log | grep -v "^\[Newton"
