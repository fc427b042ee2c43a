#!/bin/bash
# two-pass broadphase: parity tests, A/B against the previous tree, stage profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_contact_pool.py -m gpu > gpurun_out/t_bp.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_bp.log; exit 1; }
tail -1 gpurun_out/t_bp.log
bash tools/ab_multi.sh 3 bp2 "" prev "DX_LIB=variants/prev/libdx.so" || exit 1
timeout -k 10 300 python3 tools/stage_profile.py 4096 10 > gpurun_out/stages_bp.log 2>&1; head -8 gpurun_out/stages_bp.log
