#!/bin/bash
# mid tier (device-side join): tier tests, then A/B against DX_NO_MID=1 and a kernel trace
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_contact_pool.py tests/test_gpu_health.py tests/test_gpu_parity.py -k "pool or health or tiers or group_size or deterministic or queue" -m gpu > gpurun_out/t_mid.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_mid.log; exit 1; }
tail -2 gpurun_out/t_mid.log
bash tools/ab_multi.sh 3 mid "" nomid "DX_NO_MID=1" || exit 1
bash tools/gpu_r4e.sh
